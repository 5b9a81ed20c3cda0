#!/usr/bin/env python3
"""Generates the golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

The reference (Rust, curv/GMP) cannot be built or run here, so
the vectors come from the oracle (oracle/, the CPU restatement pinned by the
reference's own tests in tests/test_oracle_reference_tests.py) with seeded
randomness.  They freeze the restatement's outputs so the GPU path is checked
against fixed data on the GPU box (no oracle computation at test time) and any
later change to the oracle or the product shows up as a fixture diff.

    python tests/golden/make_golden.py          # rewrites every fixture

Fixtures (gzip JSON, codec.py):
  transcript_t2_n5_kb1024.json.gz   keygen + 5 RefreshMessages, outcome of collect() for
                                    every party, and the tamper table (one vector per
                                    FsDkrError variant collect() can return, PDL x+1)
  transcript_t2_n5_kb2048.json.gz   the same t=2 n=5 transcript and tamper table at the
                                    reference's PAILLIER_KEY_SIZE (lib.rs:26; BASELINE configs[0])
                                    (python make_golden.py t2n5-2048)
  transcript_t1_n3_kb2048.json.gz   a t=1 n=3 transcript at PAILLIER_KEY_SIZE
  transcript_join_t1_n4_kb1024.json.gz  replace() + JoinMessage: collect() of an old party,
                                    JoinMessage::collect() of the joiner, join-path tampers
  job1_kb2048.json.gz               Paillier encryption with chosen randomness (job 1)
  modexp_kat.json.gz                base^exp mod m at 2048/3072/4096/6144-bit moduli
  sampled_pairs_t8_n16_kb2048.json.gz  BASELINE configs[1] shape: 16 sampled (k, i) PDL + Alice
                                    pairs of an n=16 refresh and 8 tampered copies, with the
                                    oracle's per-pair verdicts (python make_golden.py sampled)
"""
import copy
import os
import sys
from types import SimpleNamespace

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, HERE, os.path.dirname(HERE)]

import codec  # noqa: E402
from oracle import bigint, paillier, protocol, range_proofs  # noqa: E402
from oracle import secp256k1 as ec  # noqa: E402
from oracle import zk_pdl_with_slack as pdl  # noqa: E402
from oracle.rng import Rng  # noqa: E402


from codec import _get, apply_ops  # noqa: E402


# ---------------------------------------------------------------- helpers ----
def key_summary(k):
    return {"x_i": k.x_i, "y": k.y, "pk_vec": list(k.pk_vec), "paillier_n": [e.n for e in k.paillier_key_vec],
            "dk": [k.paillier_dk.p, k.paillier_dk.q], "i": k.i, "t": k.t, "n": k.n}


def run_collect(msgs, key, dk, joins, kb):
    k = key.clone()
    try:
        protocol.collect(copy.deepcopy(msgs), k, dk, copy.deepcopy(joins), Rng("a8"), kb)
        res = None
    except protocol.FsDkrError as e:
        res = [e.variant, e.fields]
    except bigint.PanicError:
        res = ["panic"]
    return res, k


def enc_ops(ops):
    """paths stay raw (attribute names / indices); values go through the codec."""
    return [{k: (codec.enc(v) if k == "set" else v) for k, v in op.items()} for op in ops]


def tamper_entry(name, party, ops, state0, keys, dks, kb):
    st = apply_ops(state0, ops)
    res, k = run_collect(st["msgs"], keys[party], dks[party], st["joins"], kb)
    assert res is not None, f"tamper {name} did not break the oracle"
    return {"name": name, "party": party, "ops": enc_ops(ops), "outcome": res,
            "paillier_n_after": [e.n for e in k.paillier_key_vec]}


def dkr(t, n, seed, kb):
    rng = Rng(seed)
    keys = protocol.simulate_keygen(t, n, rng, kb)
    snap = [k.clone() for k in keys]          # distribute() rewrites vss_scheme
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.distribute(key.i, key, n, rng, kb)
        msgs.append(m)
        dks.append(dk)
    # collect() reads the post-distribute key (its vss_scheme threshold is unchanged)
    return keys, msgs, dks, rng, snap


def refresh_fixture(t, n, seed, kb, with_tampers):
    keys, msgs, dks, rng, _ = dkr(t, n, seed, kb)
    expect = []
    for p in range(n):
        res, k = run_collect(msgs, keys[p], dks[p], [], kb)
        assert res is None
        expect.append({"party": p, "outcome": None, "key_after": key_summary(k)})
    tampers = []
    if with_tampers:
        state0 = {"msgs": msgs, "joins": []}
        P = lambda k, i, f: ["msgs", k, "pdl_proof_vec", i, f]            # noqa: E731
        A = lambda k, i, f: ["msgs", k, "range_proofs", i, f]             # noqa: E731
        add = lambda path, d: {"path": path, "set": _get(state0, path) + d}  # noqa: E731
        T = [
            ("threshold", 0, [{"path": ["msgs"], "truncate": t}]),
            ("size_mismatch", 0, [{"path": ["msgs", 3, "pdl_proof_vec"], "truncate": n - 1}]),
            ("feldman", 0, [{"path": ["msgs", 1, "points_committed_vec", 2], "set": ec.mul(ec.G, 12345)}]),
            ("pdl_u1", 0, [add(P(3, 0, "s1"), 1)]),
            ("pdl_u2", 0, [add(P(2, 1, "u2"), 1)]),
            ("pdl_u3", 0, [add(P(0, 4, "s3"), 1)]),
            ("pdl_u1_point", 1, [{"path": P(1, 2, "u1"), "set": ec.mul(ec.G, 777)}]),
            ("range_s2", 0, [add(A(1, 3, "s2"), 1)]),
            ("range_s1_bound", 0, [{"path": A(4, 2, "s1"), "set": ec.Q ** 3 + 1}]),
            ("range_e", 0, [{"path": A(2, 2, "e"), "set": _get(state0, A(2, 2, "e")) ^ 1}]),
            ("range_z_not_unit", 2, [{"path": A(0, 1, "z"), "set": 0}]),
            ("ped_Z", 0, [add(["msgs", 3, "ring_pedersen_proof", "Z", 7], 1)]),
            ("ped_A", 0, [add(["msgs", 4, "ring_pedersen_proof", "A", 200], 1)]),
            ("ck_sigma", 0, [add(["msgs", 2, "dk_correctness_proof", "sigma_vec", 0], 1)]),
            ("ck_sigma_last", 3, [add(["msgs", 4, "dk_correctness_proof", "sigma_vec", 10], 1)]),
        ]
        # PDL soundness vector (zk_pdl_with_slack.rs:268-331): c encrypts x + 1, proof made for x
        k, i = 1, 2
        ek = keys[0].paillier_key_vec[i]
        st0 = keys[0].h1_h2_n_tilde_vec[i]
        x = paillier.decrypt(keys[i].paillier_dk, msgs[k].points_encrypted_vec[i])
        r = rng.sample_below(ek.n)
        c = paillier.encrypt_with_chosen_randomness(ek, x + 1, r)
        stmt = pdl.PDLwSlackStatement(c, ek, msgs[k].points_committed_vec[i], ec.G, st0.g, st0.ni, st0.N)
        T.append(("pdl_x_plus_1", 0, [{"path": ["msgs", k, "points_encrypted_vec", i], "set": c},
                                      {"path": ["msgs", k, "pdl_proof_vec", i], "set": pdl.prove(x, r, stmt, rng)}]))
        # ModuliTooSmall: a valid correct-key proof for a short modulus (side effect: earlier keys applied)
        ek_s, dk_s = paillier.keypair_with_modulus_size(kb - 128, rng)
        T.append(("moduli_too_small", 2, [{"path": ["msgs", 3, "ek"], "set": ek_s},
                                          {"path": ["msgs", 3, "dk_correctness_proof"],
                                           "set": protocol.NiCorrectKeyProof.proof(dk_s.p, dk_s.q)}]))
        for name, party, ops in T:
            tampers.append(tamper_entry(name, party, ops, state0, keys, dks, kb))
        assert tampers[-1]["outcome"][0] == "ModuliTooSmall"
        assert [x for x in tampers if x["name"] == "pdl_x_plus_1"][0]["outcome"] == \
            ["PDLwSlackProof", {"is_u1_eq": True, "is_u2_eq": False, "is_u3_eq": True}]
    return {"meta": {"t": t, "n": n, "key_bits": kb, "M": 256, "seed": seed,
                     "generator": "tests/golden/make_golden.py (oracle restatement, seeded)"},
            "keys": [codec.enc(k) for k in keys], "dks": [codec.enc(d) for d in dks],
            "msgs": [codec.enc(m) for m in msgs], "joins": [], "expect": codec.enc(expect),
            "tampers": tampers}


def join_fixture(seed, kb):
    """test.rs:95-224 shape: t=1, 3 old parties keep indices 1..3, one joiner gets index 4."""
    rng = Rng(seed)
    t, n = 1, 4
    all_keys = protocol.simulate_keygen(t, n, rng, kb)
    keys = [k.clone() for k in all_keys[:3]]
    jm, jkeys = protocol.join_distribute(rng, kb)
    jm.set_party_index(4)
    old_to_new = {1: 1, 2: 2, 3: 3}
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.replace([jm], key, old_to_new, n, rng, kb)
        msgs.append(m)
        dks.append(dk)
    expect = []
    for p in range(3):
        res, k = run_collect(msgs, keys[p], dks[p], [jm], kb)
        assert res is None
        expect.append({"party": p, "outcome": None, "key_after": key_summary(k)})
    jk = protocol.join_collect(jm, copy.deepcopy(msgs), jkeys, [], t, n, Rng("join-a8"), kb)
    join_expect = {"outcome": None, "key": {**key_summary(jk), "y_sum_s": jk.y_sum_s,
                                            "h1_h2_N": [s.N for s in jk.h1_h2_n_tilde_vec]}}
    state0 = {"msgs": msgs, "joins": [jm]}
    tampers = [tamper_entry(nm, party, ops, state0, keys, dks, kb) for nm, party, ops in [
        ("dlog_h2", 1, [{"path": ["joins", 0, "composite_dlog_proof_base_h2", "x"],
                         "set": jm.composite_dlog_proof_base_h2.x + 1}]),
        ("dlog_h1", 1, [{"path": ["joins", 0, "composite_dlog_proof_base_h1", "y"],
                         "set": jm.composite_dlog_proof_base_h1.y + 1}]),
        ("join_unassigned", 1, [{"path": ["joins", 0, "party_index"], "set": None}]),
        ("join_ped_Z", 0, [{"path": ["joins", 0, "ring_pedersen_proof", "Z", 3],
                            "set": jm.ring_pedersen_proof.Z[3] + 1}]),
        ("join_ck_sigma", 2, [{"path": ["joins", 0, "dk_correctness_proof", "sigma_vec", 5],
                               "set": jm.dk_correctness_proof.sigma_vec[5] + 1}]),
    ]]
    # JoinMessage::collect (add_party_message.rs:136-294) error paths, from the joiner's side
    jt = []
    for name, ops in [
        ("jc_threshold", [{"path": ["msgs"], "truncate": 1}]),
        ("jc_feldman", [{"path": ["msgs", 2, "points_committed_vec", 1], "set": ec.mul(ec.G, 99)}]),
        ("jc_ped_refresh", [{"path": ["msgs", 1, "ring_pedersen_proof", "Z", 0],
                             "set": msgs[1].ring_pedersen_proof.Z[0] + 1}]),
        ("jc_unassigned_self", [{"path": ["self", "party_index"], "set": None}]),
        ("jc_public_key", [{"path": ["msgs", 2, "public_key"], "set": ec.mul(ec.G, 5)}]),
    ]:
        st = apply_ops({"msgs": msgs, "joins": [], "self": jm}, ops)
        try:
            protocol.join_collect(st["self"], copy.deepcopy(st["msgs"]), jkeys, st["joins"], t, n,
                                  Rng("join-a8"), kb)
            res = None
        except protocol.FsDkrError as e:
            res = [e.variant, e.fields]
        except bigint.PanicError:
            res = ["panic"]
        assert res is not None, name
        jt.append({"name": name, "ops": enc_ops(ops), "outcome": res})
    return {"meta": {"t": t, "n": n, "key_bits": kb, "M": 256, "seed": seed,
                     "generator": "tests/golden/make_golden.py (oracle restatement, seeded)"},
            "keys": [codec.enc(k) for k in keys], "dks": [codec.enc(d) for d in dks],
            "msgs": [codec.enc(m) for m in msgs], "joins": [codec.enc(jm)], "join_keys": codec.enc(jkeys),
            "expect": codec.enc(expect), "join_expect": codec.enc(join_expect), "tampers": tampers,
            "join_tampers": jt}


def sampled_fixture():
    """BASELINE configs[1] shape (t=8, n=16, 2048-bit keys): 16 sampled (k, i) pairs
    from four senders' RefreshMessages (SURVEY §8c "n=16 sampled pairs"), each with its
    PDL-with-slack and Alice proofs, plus 8 tampered copies; expected verdicts by the
    oracle (pdl bits u1|u2<<1|u3<<2, range ok).  Receivers' keys and DLog statements
    for all 16 parties."""
    from tamper import oracle_pair
    t, n, kb = 8, 16, 2048
    rng = Rng("golden-n16-sampled")
    keys = protocol.simulate_keygen(t, n, rng, kb)
    lk = keys[0].clone()
    senders = [2, 7, 11, 16]
    rx = {2: [0, 5, 9, 15], 7: [1, 6, 7, 12], 11: [2, 3, 10, 14], 16: [4, 8, 11, 13]}
    pairs = []
    for pi in senders:
        key = keys[pi - 1].clone()
        m, _ = protocol.distribute(key.i, key, n, rng, kb)
        for i in rx[pi]:
            pairs.append({"k": pi, "i": i, "enc": m.points_encrypted_vec[i], "commit": m.points_committed_vec[i],
                          "pdl": m.pdl_proof_vec[i], "alice": m.range_proofs[i]})
    tampers = [("pdl", "s1", 1), ("pdl", "u2", 1), ("pdl", "s3", 1), ("pdl", "z", 1),
               ("alice", "s2", 1), ("alice", "e", 1), ("alice", "s", 1), ("alice", "z", 1)]
    import dataclasses
    entries = []
    for j, pr in enumerate(pairs):
        entries.append(dict(pr, tamper=None))
    for j, (which, f, d) in enumerate(tampers):
        pr = dict(pairs[(5 * j + 3) % len(pairs)])
        obj = pr[which]
        pr[which] = dataclasses.replace(obj, **{f: getattr(obj, f) + d})
        entries.append(dict(pr, tamper=f"{which}.{f}+{d}"))
    out = []
    for e in entries:
        msg = SimpleNamespace(points_encrypted_vec=[e["enc"]] * n, points_committed_vec=[e["commit"]] * n,
                              pdl_proof_vec=[e["pdl"]] * n, range_proofs=[e["alice"]] * n)
        bits, ok = oracle_pair(msg, lk, e["i"])
        assert (e["tamper"] is None) == (bits == 7 and ok), e["tamper"]
        out.append({"k": e["k"], "i": e["i"], "tamper": e["tamper"], "enc": codec.enc(e["enc"]),
                    "commit": codec.enc(e["commit"]),
                    "pdl": codec.enc(e["pdl"]), "alice": codec.enc(e["alice"]), "expect_pdl_bits": bits,
                    "expect_range_ok": ok})
    return {"meta": {"t": t, "n": n, "key_bits": kb, "M": 256, "seed": "golden-n16-sampled",
                     "senders": senders, "generator": "tests/golden/make_golden.py (oracle restatement, seeded)"},
            "receivers": {"ek_n": codec.enc([e.n for e in lk.paillier_key_vec]),
                          "dlog": codec.enc([[s.N, s.g, s.ni] for s in lk.h1_h2_n_tilde_vec])},
            "pairs": out}


def job1_fixture():
    rng = Rng("golden-job1")
    eks = [paillier.keypair_with_modulus_size(2048, rng)[0] for _ in range(3)]
    rows = []
    for k in range(12):
        ek = eks[k % 3]
        m = rng.sample_below(ec.Q) if k else 0
        r = rng.sample_below(ek.n)
        rows.append({"n_idx": k % 3, "m": m, "r": r, "c": paillier.encrypt_with_chosen_randomness(ek, m, r)})
    return codec.enc({"N": [e.n for e in eks], "rows": rows})


def modexp_fixture():
    rng = Rng("golden-modexp")
    rows = []
    for limbs in (64, 96, 128, 192):
        for j in range(6):
            m = rng.bits(32 * limbs) | 1 | (1 << (32 * limbs - 1))
            b = rng.sample_below(m) if j else m - 1
            e = [0, 1, 2, rng.bits(256), rng.bits(16 * limbs), rng.bits(32 * limbs)][j]
            rows.append({"limbs": limbs, "base": b, "exp": e, "mod": m, "out": pow(b, e, m)})
    return codec.enc(rows)


def main():
    if sys.argv[1:] == ["sampled"]:    # only the n=16 sampled-pairs fixture
        codec.save("sampled_pairs_t8_n16_kb2048.json.gz", sampled_fixture())
        return
    if sys.argv[1:] == ["t2n5-2048"]:  # only the configs[0] transcript at 2048-bit keys
        codec.save("transcript_t2_n5_kb2048.json.gz", refresh_fixture(2, 5, "golden-t2n5-2048", 2048, True))
        return
    codec.save("transcript_t2_n5_kb1024.json.gz", refresh_fixture(2, 5, "golden-t2n5", 1024, True))
    codec.save("transcript_t2_n5_kb2048.json.gz", refresh_fixture(2, 5, "golden-t2n5-2048", 2048, True))
    codec.save("transcript_t1_n3_kb2048.json.gz", refresh_fixture(1, 3, "golden-t1n3-2048", 2048, False))
    codec.save("transcript_join_t1_n4_kb1024.json.gz", join_fixture("golden-join", 1024))
    codec.save("job1_kb2048.json.gz", job1_fixture())
    codec.save("modexp_kat.json.gz", modexp_fixture())
    codec.save("sampled_pairs_t8_n16_kb2048.json.gz", sampled_fixture())
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".gz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
