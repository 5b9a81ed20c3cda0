"""Negative operands, per instance.  A negative
BigInt in one sender's proof gets that instance's reference outcome -- the
oracle's panic, error or plain residue -- instead of rejecting the whole batch
with UnsupportedInput (fsdkr/batch.py _Negatives).

CPU part (no device pass): the host layer's rules on top of an all-valid
verdict image give exactly the oracle's outcome (restatement of
refresh_message.rs:321-437; zk_pdl_with_slack.rs:113-167, range_proofs.rs:112-164,
ring_pedersen_proof.rs:126-157, zk-paillier CompositeDLogProof::verify), and
the stand-in rows are what the kernels need (negative bases packed as their
residue mod N^2).  The GPU part is tests/test_negative_operands_gpu.py."""
import copy
import dataclasses

import numpy as np
import pytest

from oracle import protocol
from oracle.rng import Rng

KB = 1024


def _dkr(t, n, seed):
    rng = Rng(seed)
    keys = protocol.simulate_keygen(t, n, rng, KB)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.distribute(key.i, key, n, rng, KB)
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks


def _joins(seed):
    rng = Rng(seed)
    keys = [k.clone() for k in protocol.simulate_keygen(1, 4, rng, KB)[:3]]
    jm, _ = protocol.join_distribute(rng, KB)
    jm.set_party_index(4)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.replace([jm], key, {1: 1, 2: 2, 3: 3}, 4, rng, KB)
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks, jm


@pytest.fixture(scope="module")
def dkr4():
    return _dkr(1, 4, "neg-t1n4")


@pytest.fixture(scope="module")
def joined():
    return _joins("neg-join")


def oracle_outcome(msgs, key, dk, joins=()):
    k = key.clone()
    try:
        protocol.collect(copy.deepcopy(msgs), k, dk, copy.deepcopy(list(joins)), Rng("neg"), KB)
    except protocol.FsDkrError as e:
        return (e.variant, e.fields)
    except Exception:   # PanicError / IndexError: the reference panics
        return ("panic",)
    return None


def host_outcome(msgs, key, joins=()):
    """the host layer over an all-valid device verdict image"""
    from fsdkr.batch import CollectBatch, Verdicts
    from fsdkr.refresh import FsDkrError, FsDkrPanic, _error_of
    b = CollectBatch(msgs, key, list(joins), 256, KB)
    v = Verdicts(b.R, b.J, b.n)
    v.feldman[:], v.pdl[:], v.range[:], v.ped[:], v.ck[:], v.dlog[:] = 1, 7, 1, 1, 1, 3
    e = _error_of(b.first_error(b.settle(v)))
    if isinstance(e, FsDkrPanic):
        return ("panic",)
    if isinstance(e, FsDkrError):
        return (e.variant, e.fields)
    return None


def _pdl(msgs, k, i, **kw):
    m2 = copy.deepcopy(msgs)
    p = m2[k].pdl_proof_vec[i]
    m2[k].pdl_proof_vec[i] = dataclasses.replace(p, **{f: g(p) for f, g in kw.items()})
    return m2


def _alice(msgs, k, i, **kw):
    m2 = copy.deepcopy(msgs)
    a = m2[k].range_proofs[i]
    m2[k].range_proofs[i] = dataclasses.replace(a, **{f: g(a) for f, g in kw.items()})
    return m2


CASES = {
    "pdl_s1": lambda ms: _pdl(ms, 2, 3, s1=lambda p: -p.s1),
    "pdl_s1_small": lambda ms: _pdl(ms, 0, 1, s1=lambda p: -1),
    "pdl_u2": lambda ms: _pdl(ms, 1, 0, u2=lambda p: -p.u2),
    "pdl_u3": lambda ms: _pdl(ms, 3, 2, u3=lambda p: -p.u3),
    "pdl_u2_u3": lambda ms: _pdl(ms, 3, 3, u2=lambda p: -p.u2, u3=lambda p: -p.u3),
    "alice_e": lambda ms: _alice(ms, 1, 2, e=lambda a: -a.e),
    "alice_s1": lambda ms: _alice(ms, 2, 0, s1=lambda a: -a.s1),
    "alice_s2": lambda ms: _alice(ms, 0, 3, s2=lambda a: -a.s2),
    "alice_e_z_not_unit": lambda ms: _alice(ms, 1, 1, s1=lambda a: -a.s1, z=lambda a: 0),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_negative_host_rules_match_oracle(dkr4, case):
    keys, msgs, dks = dkr4
    m2 = CASES[case](msgs)
    want = oracle_outcome(m2, keys[0], dks[0])
    assert want is not None
    if case == "alice_e_z_not_unit":   # z^e not invertible: false before the s1 panic
        assert want == ("RangeProof", {"party_index": 1})
    assert host_outcome(m2, keys[0]) == want


def test_negative_ring_pedersen_z(dkr4):
    keys, msgs, dks = dkr4
    m2 = copy.deepcopy(msgs)
    pf = m2[2].ring_pedersen_proof
    m2[2].ring_pedersen_proof = dataclasses.replace(pf, Z=tuple(-z if k == 7 else z for k, z in enumerate(pf.Z)))
    assert oracle_outcome(m2, keys[0], dks[0]) == ("panic",)
    from fsdkr.batch import CollectBatch
    b = CollectBatch(m2, keys[0], [], 256, KB)
    lens = np.ctypeslib.as_array(b.c.ped_lens, shape=(len(m2), 2))
    # Z "ends" at its negative entry: the device's short-Z rule (ped bit1 unless a
    # check before index 7 fails) -- the GPU test compares the outcome
    assert lens.tolist() == [[256, 256]] * 2 + [[256, 7]] + [[256, 256]]


def test_negative_bases_packed_as_residues(dkr4):
    """PDL s2 and Alice s are bases of x^N mod N^2: s - N^2 (negative, same residue)
    is packed as s, so the device sees the valid proof (GPU test: Ok)."""
    keys, msgs, dks = dkr4
    key = keys[0]
    nn = [k.n ** 2 for k in key.paillier_key_vec]
    m2 = _pdl(msgs, 1, 2, s2=lambda p: p.s2 - nn[2])
    m2 = _alice(m2, 3, 1, s=lambda a: a.s - 3 * nn[1])
    assert oracle_outcome(m2, key, dks[0]) is None
    from fsdkr.batch import CollectBatch
    from fsdkr._native import limbs_to_ints
    b = CollectBatch(m2, key, [], 256, KB)
    P, nl = 16, b.nl
    s2 = limbs_to_ints(np.ctypeslib.as_array(b.c.pdl_s2, shape=(P, nl)))
    s = limbs_to_ints(np.ctypeslib.as_array(b.c.rp_s, shape=(P, nl)))
    assert s2 == [m.pdl_proof_vec[i].s2 for m in msgs for i in range(4)]
    assert s == [m.range_proofs[i].s for m in msgs for i in range(4)]
    assert not b.negs.pdl and not b.negs.range and set(b.negs.rows) == {"pdl_s2", "rp_s"}
    assert host_outcome(m2, key) is None


@pytest.mark.parametrize("case", ["x1", "x2", "x1_y1", "x2_y2", "x1_y2"])
def test_negative_dlog_commitment(joined, case):
    """x < 0: that proof is false (mod_mul(g^y, ni^e) >= 0), unless its y < 0
    panics first in g^y; proof 2 only after proof 1"""
    keys, msgs, dks, jm = joined
    j2 = copy.deepcopy(jm)
    for part in case.split("_"):
        attr = "composite_dlog_proof_base_h1" if part[1] == "1" else "composite_dlog_proof_base_h2"
        p = getattr(j2, attr)
        setattr(j2, attr, dataclasses.replace(p, **{part[0]: -getattr(p, part[0])}))
    want = oracle_outcome(msgs, keys[1], dks[1], [j2])
    assert want is not None
    assert host_outcome(msgs, keys[1], [j2]) == want


@pytest.mark.parametrize("which", ["y1", "y2"])
def test_negative_dlog_response(joined, which):
    keys, msgs, dks, jm = joined
    j2 = copy.deepcopy(jm)
    attr = "composite_dlog_proof_base_h1" if which == "y1" else "composite_dlog_proof_base_h2"
    p = getattr(j2, attr)
    setattr(j2, attr, dataclasses.replace(p, y=-p.y))
    want = oracle_outcome(msgs, keys[1], dks[1], [j2])
    assert want == ("panic",)
    assert host_outcome(msgs, keys[1], [j2]) == want


class _NegGamma:
    """rng proxy for oracle.zk_pdl_with_slack.prove: its third sample_below (gamma,
    below q^3 N~) comes back shifted by -2 q^3 N~, so s3 = e rho + gamma < 0 while
    the proof stays valid (u3 = h1^alpha (h2^-1)^|gamma|, commitment_unknown_order)."""

    def __init__(self, rng):
        self.rng, self.k = rng, 0

    def sample_below(self, bound):
        v = self.rng.sample_below(bound)
        self.k += 1
        return v - 2 * bound if self.k == 3 else v

    def __getattr__(self, name):
        return getattr(self.rng, name)


def dkr_negative_s3(t, n, seed, senders):
    """_dkr with every PDL proof of the given senders (party indices) carrying a
    negative s3 -- valid proofs the reference accepts (h2^-1 raised to |s3|)."""
    from oracle import zk_pdl_with_slack as zpdl
    rng = Rng(seed)
    keys = protocol.simulate_keygen(t, n, rng, KB)
    msgs, dks = [], []
    orig = zpdl.prove
    for key in keys:
        if key.i in senders:
            zpdl.prove = lambda x, r, st, g: orig(x, r, st, _NegGamma(g))
        try:
            m, dk = protocol.distribute(key.i, key, n, rng, KB)
        finally:
            zpdl.prove = orig
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks


def dkr_negative_z(t, n, seed, senders):
    """_dkr with every PDL proof of the given senders carrying z - N~ (the same
    residue, negative): the prover hashes the negative z (|z| through to_bytes),
    so the proofs stay valid -- the reference reduces z in z^e mod N~."""
    from oracle import zk_pdl_with_slack as zpdl
    rng = Rng(seed)
    keys = protocol.simulate_keygen(t, n, rng, KB)
    msgs, dks = [], []
    orig_prove, orig_cuo = zpdl.prove, zpdl.commitment_unknown_order

    def prove(x, r, st, g):
        first = [True]

        def cuo(h1, h2, N, a, b):   # the prover's first commitment is z
            v = orig_cuo(h1, h2, N, a, b)
            if first[0]:
                first[0] = False
                return v - N
            return v
        zpdl.commitment_unknown_order = cuo
        try:
            return orig_prove(x, r, st, g)
        finally:
            zpdl.commitment_unknown_order = orig_cuo
    for key in keys:
        if key.i in senders:
            zpdl.prove = prove
        try:
            m, dk = protocol.distribute(key.i, key, n, rng, KB)
        finally:
            zpdl.prove = orig_prove
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks


def test_negative_z_packed_as_magnitude(dkr4):
    """PDL / Alice z < 0 (hashed as |z|, reduced in z^e): |z| packed with the pair's
    neg_bits bit; valid negative-z proofs verify in the oracle."""
    from fsdkr.batch import CollectBatch
    from fsdkr._native import limbs_to_ints
    keys, msgs, dks = dkr_negative_z(1, 4, "neg-z-t1n4", {2})
    assert all(p.z < 0 for p in msgs[1].pdl_proof_vec)
    assert oracle_outcome(msgs, keys[0], dks[0]) is None
    m2 = _alice(msgs, 3, 2, z=lambda a: -a.z)
    b = CollectBatch(m2, keys[0], [], 256, KB)
    flags = np.ctypeslib.as_array(b.c.neg_bits, shape=(16,)).tolist()
    assert flags == [1 if k == 1 else 0 for k in range(4) for i in range(4)][:12] + [0, 0, 2, 0]
    z = limbs_to_ints(np.ctypeslib.as_array(b.c.pdl_z, shape=(16, b.nl)))
    assert z == [abs(m.pdl_proof_vec[i].z) for m in m2 for i in range(4)]
    assert host_outcome(msgs, keys[0]) is None


@pytest.fixture(scope="module")
def neg_s3():
    return dkr_negative_s3(1, 4, "neg-s3-t1n4", {1, 3})


def test_negative_pdl_s3_valid(neg_s3):
    """Negative s3 (an h2^-1 exponent, zk_pdl_with_slack.rs:177-184): the oracle
    accepts; the batch packs |s3| and flags exactly those pairs (pdl_s3_neg),
    with no host rule (every h2 is a unit)."""
    from fsdkr.batch import CollectBatch
    from fsdkr._native import limbs_to_ints
    keys, msgs, dks = neg_s3
    neg = [k * 4 + i for k in range(4) for i in range(4) if msgs[k].pdl_proof_vec[i].s3 < 0]
    assert neg == [k * 4 + i for k in (0, 2) for i in range(4)]
    assert oracle_outcome(msgs, keys[1], dks[1]) is None
    b = CollectBatch(msgs, keys[1], [], 256, KB)
    assert b.negs.s3.tolist() == [int(p in neg) for p in range(16)]
    assert np.ctypeslib.as_array(b.c.pdl_s3_neg, shape=(16,)).tolist() == b.negs.s3.tolist()
    s3 = limbs_to_ints(np.ctypeslib.as_array(b.c.pdl_s3, shape=(16, b.c.s3l)))
    assert s3 == [abs(m.pdl_proof_vec[i].s3) for m in msgs for i in range(4)]
    assert not b.negs.pdl
    assert host_outcome(msgs, keys[1]) is None


def test_negative_pdl_s3_h2_not_unit(neg_s3):
    """h2 not a unit mod N~: mod_inv(h2).unwrap() panics at the first pair with a
    negative s3 (sender 1 holds the first message: its pair to receiver 2 is the
    first to reach u3 with h2 = N~)."""
    keys, msgs, dks = neg_s3
    key = keys[0].clone()
    st = key.h1_h2_n_tilde_vec[2]
    key.h1_h2_n_tilde_vec[2] = dataclasses.replace(st, ni=st.N)
    assert oracle_outcome(msgs, key, dks[0]) == ("panic",)
    assert host_outcome(msgs, key) == ("panic",)


def dkr_negative_c(t, n, seed, senders):
    """_dkr with the given senders' ciphertexts replaced by c - N_i^2 (the same
    residue, negative) BEFORE their PDL and Alice proofs are made over them, so
    the proofs (which hash |c|) stay valid; the reference reduces c in c^e,
    c^-1 and the share decryption."""
    from oracle import paillier
    rng = Rng(seed)
    keys = protocol.simulate_keygen(t, n, rng, KB)
    msgs, dks = [], []
    orig = paillier.encrypt_with_chosen_randomness
    for key in keys:
        if key.i in senders:
            paillier.encrypt_with_chosen_randomness = lambda ek, m, r: orig(ek, m, r) - ek.nn
        try:
            m, dk = protocol.distribute(key.i, key, n, rng, KB)
        finally:
            paillier.encrypt_with_chosen_randomness = orig
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks


def test_negative_c_packed_as_magnitude():
    """negative ciphertexts: |c| packed (both proofs hash it) with neg_bits bit 2,
    valid in the oracle; the local party's own ciphertexts decrypt as residues"""
    from fsdkr.batch import CollectBatch
    from fsdkr._native import limbs_to_ints
    keys, msgs, dks = dkr_negative_c(1, 4, "neg-c-t1n4", {3})
    assert all(c < 0 for c in msgs[2].points_encrypted_vec)
    assert oracle_outcome(msgs, keys[1], dks[1]) is None
    b = CollectBatch(msgs, keys[1], [], 256, KB)
    assert np.ctypeslib.as_array(b.c.neg_bits, shape=(16,)).tolist() == [4 if k == 2 else 0 for k in range(4)
                                                                         for i in range(4)]
    enc = limbs_to_ints(np.ctypeslib.as_array(b.c.enc, shape=(16, 2 * b.nl)))
    assert enc == [abs(m.points_encrypted_vec[i]) for m in msgs for i in range(4)]
    assert host_outcome(msgs, keys[1]) is None


def dkr_negative_a(t, n, seed, senders):
    """_dkr with the given senders' ring-Pedersen proofs made over A_k - N for
    every third k (the same residues, negative): the challenge hashes |A_k|, the
    check's mod_mul reduces A_k, so the proofs stay valid."""
    from oracle import bigint, ring_pedersen
    rng = Rng(seed)
    keys = protocol.simulate_keygen(t, n, rng, KB)
    msgs, dks = [], []
    orig = ring_pedersen.prove

    def prove(wit, st, M, g):   # ring_pedersen.prove with the shifted commitments
        a = [g.sample_below(st.phi) for _ in range(M)]
        A = [bigint.mod_pow(st.T, ai, st.N) - (st.N if k % 3 == 0 else 0) for k, ai in enumerate(a)]
        bits = ring_pedersen.challenge_bits(A, M)
        Z = [bigint.mod_add(a[i], bits[i] * wit.lam, st.phi) for i in range(M)]
        return ring_pedersen.RingPedersenProof(tuple(A), tuple(Z))
    for key in keys:
        if key.i in senders:
            ring_pedersen.prove = prove
        try:
            m, dk = protocol.distribute(key.i, key, n, rng, KB)
        finally:
            ring_pedersen.prove = orig
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks


def test_negative_ring_pedersen_a_packed():
    """negative A_k: |A_k| packed (the challenge hashes it) with ped_a_neg flags"""
    from fsdkr.batch import CollectBatch
    from fsdkr._native import limbs_to_ints
    keys, msgs, dks = dkr_negative_a(1, 4, "neg-a-t1n4", {4})
    assert oracle_outcome(msgs, keys[0], dks[0]) is None
    b = CollectBatch(msgs, keys[0], [], 256, KB)
    flags = np.ctypeslib.as_array(b.c.ped_a_neg, shape=(4, 256))
    assert flags.tolist() == [[0] * 256] * 3 + [[1 if k % 3 == 0 else 0 for k in range(256)]]
    A = limbs_to_ints(np.ctypeslib.as_array(b.c.ped_A, shape=(4 * 256, b.nl)))
    assert A == [abs(a) for m in msgs for a in m.ring_pedersen_proof.A]
    assert host_outcome(msgs, keys[0]) is None


def test_negative_outside_the_rules_still_unsupported(dkr4):
    """a negative statement field (here the receiver's N~) is outside the
    representable set: UnsupportedInput for the batch"""
    from fsdkr.batch import CollectBatch, UnsupportedInput
    keys, msgs, dks = dkr4
    m2 = msgs
    key = keys[0].clone()
    st = key.h1_h2_n_tilde_vec[1]
    key.h1_h2_n_tilde_vec[1] = dataclasses.replace(st, N=-st.N)
    with pytest.raises(UnsupportedInput):
        CollectBatch(m2, key, [], 256, KB)


def test_session_set_moves_negative_sessions_out(dkr4):
    """SessionSet: a session with a negative operand is packed on its own (its
    instances get their rules); the others stay in the set-wide gather."""
    from fsdkr.batch import SessionSet
    keys, msgs, dks = dkr4
    m2 = _pdl(msgs, 2, 3, s1=lambda p: -p.s1)
    for staged in (False, True):
        ss = SessionSet([(msgs, keys[0], []), (m2, keys[1], []), (msgs, keys[2], [])], 256, KB, staged=staged)
        if staged:
            ss.stage1b()
            ss.stage_z()
            ss.complete()
        assert ss.batches[0] is None and ss.batches[2] is None
        assert ss.batches[1] is not None and ss.batches[1].negs.pdl == {2 * 4 + 3: (8, 0xFF)}
        assert ss.live == [0, 1, 2]
