"""serde wire format (fsdkr.wire): the golden transcripts'
messages and keys survive dumps -> loads unchanged, field order follows the
reference's struct declarations, and malformed encodings are refused.  The
dependency encodings (curv BigInt / Point / Scalar, kzen-paillier, zk-paillier)
are restated, not checked against those crates: parity unpinned."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import codec  # noqa: E402
from fsdkr import types as T, wire  # noqa: E402

TRANSCRIPTS = ["transcript_t2_n5_kb1024.json.gz", "transcript_t1_n3_kb2048.json.gz",
               "transcript_join_t1_n4_kb1024.json.gz"]


@pytest.mark.parametrize("name", TRANSCRIPTS)
def test_round_trip_golden(name):
    raw = codec.load_raw(name)
    cls = codec.product_classes()
    for m in codec.dec(raw["msgs"], cls):
        assert wire.loads(wire.dumps(m), "RefreshMessage") == m
    for j in codec.dec(raw["joins"], cls):
        assert wire.loads(wire.dumps(j), "JoinMessage") == j
    for k in codec.dec(raw["keys"], cls):
        assert wire.loads(wire.dumps(k), "LocalKey") == k


def test_field_order_and_leaf_encodings():
    raw = codec.load_raw(TRANSCRIPTS[0])
    m = codec.dec(raw["msgs"], codec.product_classes())[0]
    d = json.loads(wire.dumps(m))
    assert list(d) == ["old_party_index", "party_index", "pdl_proof_vec", "range_proofs",
                       "coefficients_committed_vec", "points_committed_vec", "points_encrypted_vec",
                       "dk_correctness_proof", "dlog_statement", "ek", "remove_party_indices", "public_key",
                       "ring_pedersen_statement", "ring_pedersen_proof"]          # refresh_message.rs:31-48
    assert list(d["pdl_proof_vec"][0]) == ["z", "u1", "u2", "u3", "s1", "s2", "s3", "_phantom"]
    assert d["pdl_proof_vec"][0]["_phantom"] is None
    assert list(d["ring_pedersen_statement"]) == ["S", "T", "N", "phi", "ek"]
    assert d["points_encrypted_vec"][0] == format(m.points_encrypted_vec[0], "x")
    pt = d["public_key"]
    assert pt["curve"] == "secp256k1" and len(pt["point"]) == 66 and pt["point"][:2] in ("02", "03")


def test_edge_values_and_refusals():
    ss = T.VerifiableSS(1, 3, [None, (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
                                      0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)])
    back = wire._unvss(wire._vss(ss))
    assert back == ss and back.commitments[0] is None
    assert wire._unbi(wire._bi(-255)) == -255 and wire._bi(0) == "0"
    with pytest.raises(ValueError):
        wire._unpt({"curve": "secp256k1", "point": "02" + "ff" * 32})       # x >= p
    with pytest.raises(ValueError):
        wire._unpt({"curve": "secp256k1", "point": "02" + "00" * 31 + "05"})  # x = 5: no y on the curve
    with pytest.raises(ValueError):
        wire._unpt({"curve": "ed25519", "point": "00"})
    with pytest.raises(ValueError):
        wire._unbi(12)
    with pytest.raises(TypeError):
        wire.dumps(object())
