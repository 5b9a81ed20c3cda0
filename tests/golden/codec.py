"""JSON codec for the golden fixtures (TEST INFRASTRUCTURE).

Encodes the message / key dataclasses of either side (oracle.* or the product's
fsdkr.types) into plain JSON: integers as "0x..." strings, secp256k1 points as
{"pt": [x, y]} (null = point at infinity), dataclasses as {"__t": name, ...}.
Decoding takes a name -> class table, so the same fixture can be read into the
product's types (GPU tests: no oracle import on the product path) or into the
oracle's types (CPU tests that pin the oracle)."""
import dataclasses
import gzip
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def enc(x):
    if dataclasses.is_dataclass(x) and not isinstance(x, type):
        d = {"__t": type(x).__name__}
        for f in dataclasses.fields(x):
            d[f.name] = enc(getattr(x, f.name))
        return d
    if isinstance(x, bool):
        return x
    if isinstance(x, int):
        return hex(x) if x >= 0 else "-" + hex(-x)
    if isinstance(x, tuple) and len(x) == 2 and all(isinstance(v, int) for v in x):
        return {"pt": [hex(x[0]), hex(x[1])]}
    if isinstance(x, (list, tuple)):
        return {"tuple": [enc(v) for v in x]} if isinstance(x, tuple) else [enc(v) for v in x]
    if isinstance(x, dict):
        return {"dict": [[enc(k), enc(v)] for k, v in x.items()]}
    if x is None or isinstance(x, str):
        return x
    raise TypeError(f"cannot encode {type(x)}")


def _int(s):
    return -int(s[1:], 16) if s.startswith("-") else int(s, 16)


def dec(x, classes):
    if isinstance(x, str):
        return _int(x) if x.startswith(("0x", "-0x")) else x
    if isinstance(x, list):
        return [dec(v, classes) for v in x]
    if isinstance(x, dict):
        if "pt" in x:
            return (_int(x["pt"][0]), _int(x["pt"][1]))
        if "tuple" in x:
            return tuple(dec(v, classes) for v in x["tuple"])
        if "dict" in x:
            return {dec(k, classes): dec(v, classes) for k, v in x["dict"]}
        if "__t" in x:
            cls = classes[x["__t"]]
            return cls(**{k: dec(v, classes) for k, v in x.items() if k != "__t"})
        return {k: dec(v, classes) for k, v in x.items()}
    return x


def product_classes():
    """Decode into the product's message types (fs-dkr_amd/fsdkr/types.py)."""
    from fsdkr import types as T
    names = ["EncryptionKey", "DecryptionKey", "DLogStatement", "PDLwSlackProof", "AliceProof",
             "RingPedersenStatement", "RingPedersenProof", "NiCorrectKeyProof", "CompositeDLogProof",
             "VerifiableSS", "RefreshMessage", "JoinMessage", "LocalKey", "Keys"]
    return {n: getattr(T, n) for n in names}


def oracle_classes():
    """Decode into the oracle's types (CPU tests pinning the restatement)."""
    from oracle import paillier, protocol, range_proofs, ring_pedersen, vss, zk_paillier
    from oracle import zk_pdl_with_slack as pdl
    return {"EncryptionKey": paillier.EncryptionKey, "DecryptionKey": paillier.DecryptionKey,
            "DLogStatement": zk_paillier.DLogStatement, "PDLwSlackProof": pdl.PDLwSlackProof,
            "AliceProof": range_proofs.AliceProof, "RingPedersenStatement": ring_pedersen.RingPedersenStatement,
            "RingPedersenProof": ring_pedersen.RingPedersenProof, "NiCorrectKeyProof": zk_paillier.NiCorrectKeyProof,
            "CompositeDLogProof": zk_paillier.CompositeDLogProof, "VerifiableSS": vss.VerifiableSS,
            "RefreshMessage": protocol.RefreshMessage, "JoinMessage": protocol.JoinMessage,
            "LocalKey": protocol.LocalKey, "Keys": protocol.Keys}


def save(name, obj):
    """gzip with mtime=0 so regenerating identical data gives identical bytes."""
    with open(os.path.join(HERE, name), "wb") as raw:
        with gzip.GzipFile(filename="", mode="wb", fileobj=raw, mtime=0) as gz:
            gz.write(json.dumps(obj, separators=(",", ":"), sort_keys=True).encode())


def load_raw(name):
    with gzip.open(os.path.join(HERE, name), "rt") as f:
        return json.load(f)


def load(name, classes):
    return dec(load_raw(name), classes)


# ------------------------------------------------------------- tamper ops ----
# A tamper vector is a list of ops applied to {"msgs": [...], "joins": [...], "self": ...}:
# {"path": [...], "set": encoded value} or {"path": [...], "truncate": len}.
def _get(root, path):
    x = root
    for p in path:
        x = x[p] if isinstance(p, int) else (x[p] if isinstance(x, dict) else getattr(x, p))
    return x


def _set(x, path, value):
    """Functional update along `path` (frozen dataclasses are rebuilt)."""
    if not path:
        return value
    p, rest = path[0], path[1:]
    if isinstance(p, int):
        cur = list(x)
        cur[p] = _set(cur[p], rest, value)
        return tuple(cur) if isinstance(x, tuple) else cur
    if isinstance(x, dict):
        y = dict(x)
        y[p] = _set(x[p], rest, value)
        return y
    return dataclasses.replace(x, **{p: _set(getattr(x, p), rest, value)})


def apply_ops(state, ops, decode=lambda v: v):
    """state: {"msgs": [...], "joins": [...]}; ops: [{"path", "set"} | {"path", "truncate"}]."""
    for op in ops:
        path = op["path"]
        if "truncate" in op:
            state = _set(state, path, list(_get(state, path))[:op["truncate"]])
        else:
            state = _set(state, path, decode(op["set"]))
    return state
