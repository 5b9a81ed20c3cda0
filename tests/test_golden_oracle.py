"""The oracle reproduces every committed golden fixture (tests/golden/, made by
tests/golden/make_golden.py).  CPU only: this pins the restatement to the
frozen vectors the GPU tests check against, so an oracle change cannot drift
silently away from what the GPU path was validated on."""
import copy
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import codec  # noqa: E402
from oracle import bigint, paillier, protocol  # noqa: E402
from oracle.rng import Rng  # noqa: E402

TRANSCRIPTS = ["transcript_t2_n5_kb1024.json.gz", "transcript_t2_n5_kb2048.json.gz", "transcript_t1_n3_kb2048.json.gz",
               "transcript_join_t1_n4_kb1024.json.gz"]


@pytest.fixture(scope="module", params=TRANSCRIPTS)
def fx(request):
    raw = codec.load_raw(request.param)
    cls = codec.oracle_classes()
    return raw, {k: codec.dec(raw[k], cls) for k in ("keys", "dks", "msgs", "joins", "expect")}


def _run(msgs, key, dk, joins, kb):
    k = key.clone()
    try:
        protocol.collect(copy.deepcopy(msgs), k, dk, copy.deepcopy(joins), Rng("a8"), kb)
        return None, k
    except protocol.FsDkrError as e:
        return [e.variant, e.fields], k
    except bigint.PanicError:
        return ["panic"], k


def test_collect_outcomes(fx):
    raw, d = fx
    kb = raw["meta"]["key_bits"]
    for e in d["expect"]:
        res, k = _run(d["msgs"], d["keys"][e["party"]], d["dks"][e["party"]], d["joins"], kb)
        assert res is None
        want = e["key_after"]
        assert (k.x_i, k.y, list(k.pk_vec)) == (want["x_i"], want["y"], want["pk_vec"])
        assert [x.n for x in k.paillier_key_vec] == want["paillier_n"]
        assert [k.paillier_dk.p, k.paillier_dk.q] == want["dk"]


def test_tampers(fx):
    raw, d = fx
    kb = raw["meta"]["key_bits"]
    cls = codec.oracle_classes()
    for t in raw["tampers"]:
        st = codec.apply_ops({"msgs": d["msgs"], "joins": d["joins"]}, t["ops"], lambda v: codec.dec(v, cls))
        res, k = _run(st["msgs"], d["keys"][t["party"]], d["dks"][t["party"]], st["joins"], kb)
        assert res == t["outcome"], t["name"]
        assert [x.n for x in k.paillier_key_vec] == [codec.dec(v, cls) for v in t["paillier_n_after"]], t["name"]


def test_join_collect_fixture():
    raw = codec.load_raw("transcript_join_t1_n4_kb1024.json.gz")
    cls = codec.oracle_classes()
    msgs = codec.dec(raw["msgs"], cls)
    jm = codec.dec(raw["joins"], cls)[0]
    jk = codec.dec(raw["join_keys"], cls)
    want = codec.dec(raw["join_expect"], cls)["key"]
    meta = raw["meta"]
    k = protocol.join_collect(jm, copy.deepcopy(msgs), jk, [], meta["t"], meta["n"], Rng("join-a8"), meta["key_bits"])
    assert (k.x_i, k.y, list(k.pk_vec), k.y_sum_s) == (want["x_i"], want["y"], want["pk_vec"], want["y_sum_s"])
    assert [e.n for e in k.paillier_key_vec] == want["paillier_n"]
    assert [s.N for s in k.h1_h2_n_tilde_vec] == want["h1_h2_N"]
    for t in raw["join_tampers"]:
        st = codec.apply_ops({"msgs": msgs, "joins": [], "self": jm}, t["ops"], lambda v: codec.dec(v, cls))
        try:
            protocol.join_collect(st["self"], copy.deepcopy(st["msgs"]), jk, st["joins"], meta["t"], meta["n"],
                                  Rng("join-a8"), meta["key_bits"])
            res = None
        except protocol.FsDkrError as e:
            res = [e.variant, e.fields]
        assert res == t["outcome"], t["name"]


def test_job1_and_modexp_vectors():
    j = codec.dec(codec.load_raw("job1_kb2048.json.gz"), {})
    for r in j["rows"]:
        ek = paillier.EncryptionKey.from_n(j["N"][r["n_idx"]])
        assert paillier.encrypt_with_chosen_randomness(ek, r["m"], r["r"]) == r["c"]
    for r in codec.dec(codec.load_raw("modexp_kat.json.gz"), {}):
        assert bigint.mod_pow(r["base"], r["exp"], r["mod"]) == r["out"]


def test_every_collect_error_variant_is_covered():
    """One golden vector per FsDkrError variant (error.rs:6-60)."""
    seen = set()
    for f in TRANSCRIPTS:
        raw = codec.load_raw(f)
        seen |= {t["outcome"][0] for t in raw.get("tampers", []) + raw.get("join_tampers", [])}
    assert seen >= {"PartiesThresholdViolation", "PublicShareValidationError", "SizeMismatchError", "PDLwSlackProof",
                    "RingPedersenProofError", "RangeProof", "ModuliTooSmall", "PaillierVerificationError",
                    "NewPartyUnassignedIndexError", "BroadcastedPublicKeyError", "DLogProofValidation",
                    "RingPedersenProofValidation"}


def test_sampled_pairs_n16():
    """BASELINE configs[1] shape (n=16, t=8, 2048-bit): the oracle reproduces the
    per-pair verdicts frozen in the sampled-pairs fixture (16 valid, 8 tampered)."""
    from types import SimpleNamespace
    from tamper import oracle_pair
    from oracle.zk_paillier import DLogStatement
    raw = codec.load_raw("sampled_pairs_t8_n16_kb2048.json.gz")
    cls = codec.oracle_classes()
    rec = codec.dec(raw["receivers"], cls)
    lk = SimpleNamespace(paillier_key_vec=[paillier.EncryptionKey.from_n(x) for x in rec["ek_n"]],
                         h1_h2_n_tilde_vec=[DLogStatement(*s) for s in rec["dlog"]])
    n = raw["meta"]["n"]
    assert len(raw["pairs"]) == 24 and sum(p["tamper"] is None for p in raw["pairs"]) == 16
    for p in raw["pairs"]:
        d = codec.dec(p, cls)
        m = SimpleNamespace(points_encrypted_vec=[d["enc"]] * n, points_committed_vec=[d["commit"]] * n,
                            pdl_proof_vec=[d["pdl"]] * n, range_proofs=[d["alice"]] * n)
        assert oracle_pair(m, lk, d["i"]) == (d["expect_pdl_bits"], d["expect_range_ok"]), p["tamper"]
