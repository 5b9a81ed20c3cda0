"""Host-side mirror of RefreshMessage::collect (/root/reference/src/refresh_message.rs:321-467)
over the MI355X C ABI.

Same argument meaning and error behaviour as the reference: returns None on
success after mutating `local_key` exactly as collect() does, raises
FsDkrError with the reference's variant name and payload for the FIRST failing
check (or FsDkrPanic where the reference panics).  All proof verification runs
in one batched GPU pass (fsdkr_verify_collect); share recovery uses the GPU
decryption and MSM entry points.  There is no CPU fallback."""
from ._native import Context
from .batch import CollectBatch

Q = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8

# error.rs:6-60, in declaration order (matches FSDKR_ERR_* in fsdkr.h)
_VARIANTS = {
    1: ("PartiesThresholdViolation", ("threshold", "refreshed_keys")),
    2: ("PublicShareValidationError", ()),
    3: ("SizeMismatchError", ("refresh_message_index", "pdl_proof_len", "points_commited_len",
                              "points_encrypted_len")),
    4: ("PDLwSlackProof", ("is_u1_eq", "is_u2_eq", "is_u3_eq")),
    5: ("RingPedersenProofError", ()),
    6: ("RangeProof", ("party_index",)),
    7: ("ModuliTooSmall", ("party_index", "moduli_size")),
    8: ("PaillierVerificationError", ("party_index",)),
    9: ("NewPartyUnassignedIndexError", ()),
    10: ("BroadcastedPublicKeyError", ()),
    11: ("DLogProofValidation", ("party_index",)),
    12: ("RingPedersenProofValidation", ("party_index",)),
}
_BOOL_FIELDS = {"is_u1_eq", "is_u2_eq", "is_u3_eq"}


class FsDkrError(Exception):
    """FsDkrError (error.rs): `variant` is the Rust variant name, `fields` its payload."""

    def __init__(self, variant, **fields):
        super().__init__(f"{variant}{fields}")
        self.variant = variant
        self.fields = fields


class FsDkrPanic(Exception):
    """The reference panics at this point (unwrap / index / assert)."""


def _lagrange(index, s):
    """curv VerifiableSS::map_share_to_new_params: Lagrange coefficient at 0."""
    xi = index + 1
    num, den = 1, 1
    for j in s:
        if j == index:
            continue
        num = num * (j + 1) % Q
        den = den * ((j + 1) - xi) % Q
    return num * pow(den, -1, Q) % Q


_default_ctx = None


def _ctx(ctx):
    global _default_ctx
    if ctx is not None:
        return ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx


def verify(refresh_messages, local_key, join_messages, ctx=None, m_security=256, key_bits=2048):
    """Verification half of collect(): (error or None, keys_applied, batch)."""
    batch = CollectBatch(refresh_messages, local_key, join_messages, m_security, key_bits)
    verdicts = None if batch.header_only else _ctx(ctx).verify_collect(batch)
    err = batch.first_error(verdicts)
    if err.variant == 0:
        return None, err.keys_applied, batch
    name, fields = _VARIANTS[err.variant]
    vals = {f: (bool(err.f[k]) if f in _BOOL_FIELDS else int(err.f[k])) for k, f in enumerate(fields)}
    if err.panic:
        return FsDkrPanic(f"reference panics at {name}"), err.keys_applied, batch
    return FsDkrError(name, **vals), err.keys_applied, batch


def collect(refresh_messages, local_key, new_dk, join_messages, ctx=None, m_security=256, key_bits=2048):
    """RefreshMessage::collect (refresh_message.rs:321-467)."""
    ctx = _ctx(ctx)
    msgs, joins = list(refresh_messages), list(join_messages)
    err, applied, batch = verify(msgs, local_key, joins, ctx, m_security, key_bits)
    # paillier_key_vec is written message by message before a later check fails (:394, :436)
    for k, m in enumerate(msgs + joins):
        if k >= applied:
            break
        local_key.paillier_key_vec[m.party_index - 1] = m.ek
    if err is not None:
        raise err
    # ---- share recovery (:367-373, :439-464)
    t = local_key.vss_scheme.threshold
    indices = [msgs[j].old_party_index - 1 for j in range(t + 1)]
    li = [_lagrange(indices[j], indices) for j in range(t + 1)]
    nl = batch.nl
    cts = [msgs[j].points_encrypted_vec[local_key.i - 1] for j in range(t + 1)]
    dk = local_key.paillier_dk
    sig = ctx.paillier_decrypt(cts, dk.p, dk.q, nl)
    # Dec(prod c_j^l_j * Enc(0)) = sum l_j Dec(c_j) mod N  (the Enc(0) factor only re-randomises)
    new_share = sum(l * s for l, s in zip(li, sig)) % (dk.p * dk.q) % Q
    local_key.paillier_dk = new_dk
    local_key.x_i = new_share
    n_new = len(msgs) + len(joins)
    pts = [[(GX, GY)]] + [[msgs[j].points_committed_vec[i] for j in range(t + 1)] for i in range(n_new)]
    scs = [[new_share]] + [li[:] for _ in range(n_new)]
    # one MSM launch: y = G*x, then pk_vec[i] = sum_j P_j,i * l_j  (rows padded to t+1 terms)
    width = t + 1
    pts = [row + [None] * (width - len(row)) for row in pts]
    scs = [row + [0] * (width - len(row)) for row in scs]
    res = ctx.ec_msm(pts, scs)
    local_key.y = res[0]
    for i in range(n_new):
        local_key.pk_vec.insert(i, res[1 + i])
