"""Injected-tamper property checks for the full-size BASELINE configs (test
infrastructure).

A synthetic workload (fsdkr.synth, every proof valid) gets tampers at known
positions; the oracle (the CPU restatement of the reference) computes the
verdict of every tampered instance and the first error collect() must report
(refresh_message.rs:321-437 order: Feldman, [PDL, range] per (k, i),
ring-Pedersen refresh then join, correct key + size per refresh message, per
join: index, correct key, DLog, size).  The GPU verdict vector must equal
all-valid everywhere except exactly the injected set, where it must equal the
oracle's verdicts."""
import copy
import dataclasses

from oracle import range_proofs, ring_pedersen
from oracle import secp256k1 as ec
from oracle import zk_pdl_with_slack as pdl
from oracle.zk_paillier import CompositeDLogProof, DLogStatement, NiCorrectKeyProof

M = 256


def _own(msgs, k):
    """Give message k its own proof vectors (tiled workloads share objects)."""
    m = copy.copy(msgs[k])
    m.pdl_proof_vec = list(m.pdl_proof_vec)
    m.range_proofs = list(m.range_proofs)
    m.points_committed_vec = list(m.points_committed_vec)
    msgs[k] = m
    return m


PAIR_KINDS = ("pdl_s1", "pdl_s2", "pdl_s3", "pdl_u2", "pdl_z", "range_s", "range_s2", "range_e", "range_z", "enc",
              "feldman")
MSG_KINDS = ("rp_Z", "rp_A", "ck")


def inject(msgs, joins, spec):
    """spec: list of (kind, k, i).  kinds: pdl_s1, pdl_s2, pdl_s3, pdl_u2, pdl_z (pair k, i),
    range_s, range_s2, range_e, range_z (pair), enc (the pair's ciphertext c), feldman
    (pair), rp_Z / rp_A (message k, index i), ck (message k), dlog (join k)."""
    msgs, joins = list(msgs), list(joins)
    for kind, k, i in spec:
        if kind in ("pdl_s1", "pdl_s2", "pdl_s3", "pdl_u2", "pdl_z"):
            m = _own(msgs, k)
            p = m.pdl_proof_vec[i]
            f = kind.split("_")[1]
            m.pdl_proof_vec[i] = dataclasses.replace(p, **{f: getattr(p, f) + 1})
        elif kind == "enc":
            m = _own(msgs, k)
            m.points_encrypted_vec = list(m.points_encrypted_vec)
            m.points_encrypted_vec[i] += 1
        elif kind in ("range_s", "range_s2", "range_e", "range_z"):
            m = _own(msgs, k)
            a = m.range_proofs[i]
            f = kind.split("_")[1]
            m.range_proofs[i] = dataclasses.replace(a, **{f: getattr(a, f) ^ 1 if f == "e" else getattr(a, f) + 1})
        elif kind == "feldman":
            m = _own(msgs, k)
            m.points_committed_vec[i] = ec.mul(ec.G, 12345 + i)
        elif kind in ("rp_Z", "rp_A"):
            m = copy.copy(msgs[k]) if k < len(msgs) else copy.copy(joins[k - len(msgs)])
            pf = m.ring_pedersen_proof
            f = kind.split("_")[1]
            m.ring_pedersen_proof = dataclasses.replace(pf, **{f: tuple(z + (j == i) for j, z in enumerate(getattr(pf, f)))})
            if k < len(msgs):
                msgs[k] = m
            else:
                joins[k - len(msgs)] = m
        elif kind == "ck":
            m = copy.copy(msgs[k]) if k < len(msgs) else copy.copy(joins[k - len(msgs)])
            sv = m.dk_correctness_proof.sigma_vec
            m.dk_correctness_proof = dataclasses.replace(m.dk_correctness_proof, sigma_vec=(sv[0] + 1,) + tuple(sv[1:]))
            if k < len(msgs):
                msgs[k] = m
            else:
                joins[k - len(msgs)] = m
        elif kind == "dlog":
            j = copy.copy(joins[k])
            p = j.composite_dlog_proof_base_h2
            j.composite_dlog_proof_base_h2 = dataclasses.replace(p, x=p.x + 1)
            joins[k] = j
        else:
            raise ValueError(kind)
    return msgs, joins


def _stmt(m, lk, i):
    st = lk.h1_h2_n_tilde_vec[i]
    return pdl.PDLwSlackStatement(m.points_encrypted_vec[i], lk.paillier_key_vec[i], m.points_committed_vec[i], ec.G,
                                  st.g, st.ni, st.N)


def oracle_pair(m, lk, i):
    """(pdl verdict bits as the GPU reports them, range ok) of pair (m, i) by the oracle."""
    st = _stmt(m, lk, i)
    try:
        pdl.verify(m.pdl_proof_vec[i], st)
        bits = 7
    except pdl.PDLwSlackError as e:
        bits = (1 if e.flags[0] else 0) | (2 if e.flags[1] else 0) | (4 if e.flags[2] else 0)
    ok = range_proofs.verify(m.range_proofs[i], st.ciphertext, st.ek, lk.h1_h2_n_tilde_vec[i])
    return bits, bool(ok)


def oracle_message(m):
    """(ring-Pedersen ok, correct-key ok) of a refresh or join message by the oracle."""
    return (bool(ring_pedersen.verify(m.ring_pedersen_proof, m.ring_pedersen_statement, M)),
            bool(NiCorrectKeyProof(m.dk_correctness_proof.sigma_vec).verify(m.ek.n)))


def oracle_dlog(j):
    st = DLogStatement(j.dlog_statement.N, j.dlog_statement.g, j.dlog_statement.ni)
    st2 = DLogStatement(st.N, st.ni, st.g)
    a = CompositeDLogProof(j.composite_dlog_proof_base_h1.x, j.composite_dlog_proof_base_h1.y).verify(st)
    b = CompositeDLogProof(j.composite_dlog_proof_base_h2.x, j.composite_dlog_proof_base_h2.y).verify(st2)
    return (1 if a else 0) | (2 if b else 0)


def expected(msgs, joins, lk, spec, key_bits):
    """Oracle verdicts of the tampered instances and collect()'s first error.
    Returns (pairs {(k,i): (feldman, pdl_bits, range)}, msgs {m: (ped, ck)}, joins {j: dlog}, first_error)."""
    from oracle.vss import VerifiableSS
    R, J = len(msgs), len(joins)
    n = R + J
    pairs, mres, jres = {}, {}, {}
    for kind, k, i in spec:
        if kind in PAIR_KINDS:
            m = msgs[k]
            vss = VerifiableSS(lk.t, n, list(m.coefficients_committed_vec.commitments))
            fel = vss.validate_share_public(m.points_committed_vec[i], i + 1)
            pairs[(k, i)] = (fel,) + oracle_pair(m, lk, i)
        elif kind in MSG_KINDS:
            mm = msgs[k] if k < R else joins[k - R]
            mres[k] = oracle_message(mm)
        elif kind == "dlog":
            jres[k] = oracle_dlog(joins[k])
    # first error in reference order (every other instance is valid)
    first = None
    for (k, i) in sorted(pairs):
        if not pairs[(k, i)][0]:
            first = ("PublicShareValidationError", {})
            break
    if first is None:
        for (k, i) in sorted(pairs):
            fel, bits, rok = pairs[(k, i)]
            if bits != 7:
                first = ("PDLwSlackProof", {"is_u1_eq": bool(bits & 1), "is_u2_eq": bool(bits & 2),
                                            "is_u3_eq": bool(bits & 4)})
                break
            if not rok:
                first = ("RangeProof", {"party_index": i})
                break
    if first is None:
        for m in sorted(mres):
            if not mres[m][0]:
                first = ("RingPedersenProofError", {})
                break
    if first is None:
        for m in range(n):
            ck_ok = mres.get(m, (True, True))[1]
            pi = (msgs[m] if m < R else joins[m - R]).party_index
            if not ck_ok:
                first = ("PaillierVerificationError", {"party_index": pi})
                break
            if m >= R and jres.get(m - R, 3) != 3:
                first = ("DLogProofValidation", {"party_index": pi})
                break
    return pairs, mres, jres, first


def check_verdicts(v, R, J, n, pairs, mres, jres):
    """GPU Verdicts == all valid except the injected set, which equals the oracle's."""
    import numpy as np
    fel = np.ones(R * n, np.uint8)
    pdl_b = np.full(R * n, 7, np.uint8)
    rng = np.ones(R * n, np.uint8)
    ped = np.ones(R + J, np.uint8)
    ck = np.ones(R + J, np.uint8)
    dl = np.full(J, 3, np.uint8)
    for (k, i), (f, bits, rok) in pairs.items():
        fel[k * n + i] = 1 if f else 0
        pdl_b[k * n + i] = bits
        rng[k * n + i] = 1 if rok else 0
    for m, (p, c) in mres.items():
        ped[m] = 1 if p else 0
        ck[m] = 1 if c else 0
    for j, d in jres.items():
        dl[j] = d
    assert np.array_equal(v.feldman[:R * n], fel), np.nonzero(v.feldman[:R * n] != fel)
    assert np.array_equal(v.pdl[:R * n] & 7, pdl_b), np.nonzero((v.pdl[:R * n] & 7) != pdl_b)
    assert not (v.pdl[:R * n] & 8).any()
    assert np.array_equal(v.range[:R * n], rng), np.nonzero(v.range[:R * n] != rng)
    assert np.array_equal(v.ped[:R + J], ped), np.nonzero(v.ped[:R + J] != ped)
    assert np.array_equal(v.ck[:R + J], ck), np.nonzero(v.ck[:R + J] != ck)
    if J:
        assert np.array_equal(v.dlog[:J], dl), (v.dlog[:J], dl)


def to_oracle(msgs, joins=()):
    """Copies of product-typed messages with the oracle's method-bearing types
    (VerifiableSS.validate_share_public, NiCorrectKeyProof.verify,
    CompositeDLogProof.verify) so oracle.protocol.collect can run on them."""
    from oracle.vss import VerifiableSS
    out = []
    for m in msgs:
        m = copy.copy(m)
        v = m.coefficients_committed_vec
        m.coefficients_committed_vec = VerifiableSS(v.threshold, v.share_count, list(v.commitments))
        m.dk_correctness_proof = NiCorrectKeyProof(tuple(m.dk_correctness_proof.sigma_vec))
        out.append(m)
    if not joins:
        return out
    oj = []
    for j in joins:
        j = copy.copy(j)
        j.dk_correctness_proof = NiCorrectKeyProof(tuple(j.dk_correctness_proof.sigma_vec))
        j.composite_dlog_proof_base_h1 = CompositeDLogProof(j.composite_dlog_proof_base_h1.x,
                                                            j.composite_dlog_proof_base_h1.y)
        j.composite_dlog_proof_base_h2 = CompositeDLogProof(j.composite_dlog_proof_base_h2.x,
                                                            j.composite_dlog_proof_base_h2.y)
        oj.append(j)
    return out, oj
