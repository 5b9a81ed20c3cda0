"""serde wire format of the broadcast messages and the LocalKey (SURVEY §8f
item 2): JSON as serde_json writes the reference's `#[derive(Serialize)]`
structs, so reference-produced transcripts can be ingested and ours read back.

Field order and names follow the struct declarations:
  RefreshMessage     refresh_message.rs:29-48 (hash_choice #[serde(skip)])
  JoinMessage        add_party_message.rs:34-45
  PDLwSlackProof     zk_pdl_with_slack.rs:39-50 (_phantom: PhantomData -> null)
  AliceProof         range_proofs.rs:100-108   (_phantom -> null)
  RingPedersenStatement / Proof  ring_pedersen_proof.rs:28-38, 77-84 (phantom skipped)
Dependency encodings, restated from the published crates and NOT checked
against their code (parity unpinned: curv-kzen 0.10, kzen-paillier 0.4.3,
zk-paillier 0.4.4 and multi-party-ecdsa are not in this image):
  BigInt             lowercase hex string, no prefix, "-" for negatives (curv)
  Point<Secp256k1>   {"curve": "secp256k1", "point": hex of the 33-byte SEC1
                     compressed encoding; "00" for the point at infinity}
  Scalar<Secp256k1>  {"curve": "secp256k1", "scalar": hex of the 32-byte value}
  VerifiableSS       {"parameters": {"threshold", "share_count"}, "commitments"}
  EncryptionKey {n, nn}, DecryptionKey {p, q}, DLogStatement {N, g, ni},
  NiCorrectKeyProof {sigma_vec}, CompositeDLogProof {x, y}
  LocalKey           {paillier_dk, pk_vec, keys_linear: {y, x_i}, paillier_key_vec,
                     y_sum_s, h1_h2_n_tilde_vec, vss_scheme, i, t, n}
Decoding yields fsdkr.types objects (the batching layer's input)."""
import json

from . import types as T

_P = (1 << 256) - (1 << 32) - 977   # secp256k1 field prime
CURVE = "secp256k1"


# ---------------------------------------------------------------- leaves ----
def _bi(x):
    return format(x, "x") if x >= 0 else "-" + format(-x, "x")


def _unbi(s):
    if not isinstance(s, str) or not s:
        raise ValueError(f"BigInt: expected a hex string, got {s!r}")
    return -int(s[1:], 16) if s.startswith("-") else int(s, 16)


def _pt(p):
    if p is None:
        return {"curve": CURVE, "point": "00"}
    x, y = p
    return {"curve": CURVE, "point": ("03" if y & 1 else "02") + format(x, "064x")}


def _unpt(d):
    if d.get("curve") != CURVE:
        raise ValueError(f"point on curve {d.get('curve')!r}")
    h = d["point"]
    if h == "00":
        return None
    if len(h) != 66 or h[:2] not in ("02", "03"):
        raise ValueError("point: expected a 33-byte compressed encoding")
    x = int(h[2:], 16)
    if x >= _P:
        raise ValueError("point: x out of range")
    y2 = (pow(x, 3, _P) + 7) % _P
    y = pow(y2, (_P + 1) // 4, _P)
    if y * y % _P != y2:
        raise ValueError("point: x is not on secp256k1")
    if (y & 1) != (h[:2] == "03"):
        y = _P - y
    return (x, y)


def _sc(x):
    return {"curve": CURVE, "scalar": format(x, "064x")}


def _unsc(d):
    if d.get("curve") != CURVE:
        raise ValueError(f"scalar on curve {d.get('curve')!r}")
    return int(d["scalar"], 16)


# ------------------------------------------------------------ structures ----
def _ek(e):
    return {"n": _bi(e.n), "nn": _bi(e.nn)}


def _unek(d):
    return T.EncryptionKey(_unbi(d["n"]), _unbi(d["nn"]))


def _dlog(s):
    return {"N": _bi(s.N), "g": _bi(s.g), "ni": _bi(s.ni)}


def _undlog(d):
    return T.DLogStatement(_unbi(d["N"]), _unbi(d["g"]), _unbi(d["ni"]))


def _vss(v):
    return {"parameters": {"threshold": v.threshold, "share_count": v.share_count},
            "commitments": [_pt(p) for p in v.commitments]}


def _unvss(d):
    p = d["parameters"]
    return T.VerifiableSS(threshold=p["threshold"], share_count=p["share_count"],
                          commitments=[_unpt(x) for x in d["commitments"]])


def _rp_st(s):
    return {"S": _bi(s.S), "T": _bi(s.T), "N": _bi(s.N), "phi": _bi(s.phi), "ek": _ek(s.ek)}


def _unrp_st(d):
    return T.RingPedersenStatement(_unbi(d["S"]), _unbi(d["T"]), _unbi(d["N"]), _unbi(d["phi"]), _unek(d["ek"]))


def _rp_pf(p):
    return {"A": [_bi(a) for a in p.A], "Z": [_bi(z) for z in p.Z]}


def _unrp_pf(d):
    return T.RingPedersenProof(tuple(_unbi(a) for a in d["A"]), tuple(_unbi(z) for z in d["Z"]))


def _pdl(p):
    return {"z": _bi(p.z), "u1": _pt(p.u1), "u2": _bi(p.u2), "u3": _bi(p.u3), "s1": _bi(p.s1), "s2": _bi(p.s2),
            "s3": _bi(p.s3), "_phantom": None}


def _unpdl(d):
    return T.PDLwSlackProof(_unbi(d["z"]), _unpt(d["u1"]), _unbi(d["u2"]), _unbi(d["u3"]), _unbi(d["s1"]),
                            _unbi(d["s2"]), _unbi(d["s3"]))


def _alice(a):
    return {"z": _bi(a.z), "e": _bi(a.e), "s": _bi(a.s), "s1": _bi(a.s1), "s2": _bi(a.s2), "_phantom": None}


def _unalice(d):
    return T.AliceProof(_unbi(d["z"]), _unbi(d["e"]), _unbi(d["s"]), _unbi(d["s1"]), _unbi(d["s2"]))


def _ck(p):
    return {"sigma_vec": [_bi(s) for s in p.sigma_vec]}


def _unck(d):
    return T.NiCorrectKeyProof(tuple(_unbi(s) for s in d["sigma_vec"]))


def _cdl(p):
    return {"x": _bi(p.x), "y": _bi(p.y)}


def _uncdl(d):
    return T.CompositeDLogProof(_unbi(d["x"]), _unbi(d["y"]))


def refresh_message_to_obj(m):
    return {"old_party_index": m.old_party_index, "party_index": m.party_index,
            "pdl_proof_vec": [_pdl(p) for p in m.pdl_proof_vec],
            "range_proofs": [_alice(a) for a in m.range_proofs],
            "coefficients_committed_vec": _vss(m.coefficients_committed_vec),
            "points_committed_vec": [_pt(p) for p in m.points_committed_vec],
            "points_encrypted_vec": [_bi(c) for c in m.points_encrypted_vec],
            "dk_correctness_proof": _ck(m.dk_correctness_proof), "dlog_statement": _dlog(m.dlog_statement),
            "ek": _ek(m.ek), "remove_party_indices": list(m.remove_party_indices),
            "public_key": _pt(m.public_key), "ring_pedersen_statement": _rp_st(m.ring_pedersen_statement),
            "ring_pedersen_proof": _rp_pf(m.ring_pedersen_proof)}


def refresh_message_from_obj(d):
    return T.RefreshMessage(
        old_party_index=d["old_party_index"], party_index=d["party_index"],
        pdl_proof_vec=[_unpdl(p) for p in d["pdl_proof_vec"]],
        range_proofs=[_unalice(a) for a in d["range_proofs"]],
        coefficients_committed_vec=_unvss(d["coefficients_committed_vec"]),
        points_committed_vec=[_unpt(p) for p in d["points_committed_vec"]],
        points_encrypted_vec=[_unbi(c) for c in d["points_encrypted_vec"]],
        dk_correctness_proof=_unck(d["dk_correctness_proof"]), dlog_statement=_undlog(d["dlog_statement"]),
        ek=_unek(d["ek"]), remove_party_indices=list(d["remove_party_indices"]),
        public_key=_unpt(d["public_key"]), ring_pedersen_statement=_unrp_st(d["ring_pedersen_statement"]),
        ring_pedersen_proof=_unrp_pf(d["ring_pedersen_proof"]))


def join_message_to_obj(j):
    return {"ek": _ek(j.ek), "dk_correctness_proof": _ck(j.dk_correctness_proof), "party_index": j.party_index,
            "dlog_statement": _dlog(j.dlog_statement),
            "composite_dlog_proof_base_h1": _cdl(j.composite_dlog_proof_base_h1),
            "composite_dlog_proof_base_h2": _cdl(j.composite_dlog_proof_base_h2),
            "ring_pedersen_statement": _rp_st(j.ring_pedersen_statement),
            "ring_pedersen_proof": _rp_pf(j.ring_pedersen_proof)}


def join_message_from_obj(d):
    return T.JoinMessage(
        ek=_unek(d["ek"]), dk_correctness_proof=_unck(d["dk_correctness_proof"]), party_index=d["party_index"],
        dlog_statement=_undlog(d["dlog_statement"]),
        composite_dlog_proof_base_h1=_uncdl(d["composite_dlog_proof_base_h1"]),
        composite_dlog_proof_base_h2=_uncdl(d["composite_dlog_proof_base_h2"]),
        ring_pedersen_statement=_unrp_st(d["ring_pedersen_statement"]),
        ring_pedersen_proof=_unrp_pf(d["ring_pedersen_proof"]))


def local_key_to_obj(k):
    return {"paillier_dk": {"p": _bi(k.paillier_dk.p), "q": _bi(k.paillier_dk.q)},
            "pk_vec": [_pt(p) for p in k.pk_vec], "keys_linear": {"y": _pt(k.y), "x_i": _sc(k.x_i)},
            "paillier_key_vec": [_ek(e) for e in k.paillier_key_vec], "y_sum_s": _pt(k.y_sum_s),
            "h1_h2_n_tilde_vec": [_dlog(s) for s in k.h1_h2_n_tilde_vec], "vss_scheme": _vss(k.vss_scheme),
            "i": k.i, "t": k.t, "n": k.n}


def local_key_from_obj(d):
    return T.LocalKey(
        paillier_dk=T.DecryptionKey(_unbi(d["paillier_dk"]["p"]), _unbi(d["paillier_dk"]["q"])),
        pk_vec=[_unpt(p) for p in d["pk_vec"]], x_i=_unsc(d["keys_linear"]["x_i"]),
        y=_unpt(d["keys_linear"]["y"]), paillier_key_vec=[_unek(e) for e in d["paillier_key_vec"]],
        y_sum_s=_unpt(d["y_sum_s"]), h1_h2_n_tilde_vec=[_undlog(s) for s in d["h1_h2_n_tilde_vec"]],
        vss_scheme=_unvss(d["vss_scheme"]), i=d["i"], t=d["t"], n=d["n"])


_KINDS = {"RefreshMessage": (refresh_message_to_obj, refresh_message_from_obj),
          "JoinMessage": (join_message_to_obj, join_message_from_obj),
          "LocalKey": (local_key_to_obj, local_key_from_obj)}


def dumps(obj):
    """serde_json text of a RefreshMessage / JoinMessage / LocalKey (compact, field order kept)."""
    kind = type(obj).__name__
    if kind not in _KINDS:
        raise TypeError(f"no wire format for {kind}")
    return json.dumps(_KINDS[kind][0](obj), separators=(",", ":"))


def loads(text, kind):
    """Decode serde_json text of `kind` ("RefreshMessage", "JoinMessage", "LocalKey")."""
    return _KINDS[kind][1](json.loads(text))


__all__ = ["dumps", "loads", "refresh_message_to_obj", "refresh_message_from_obj", "join_message_to_obj",
           "join_message_from_obj", "local_key_to_obj", "local_key_from_obj"]
