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
    n_new = len(msgs) + len(joins)
    new_share, y, pk = recover_share(ctx, msgs, local_key.i, t, local_key.paillier_dk, batch.nl, n_new)
    local_key.paillier_dk = new_dk
    local_key.x_i = new_share
    local_key.y = y
    for i in range(n_new):
        local_key.pk_vec.insert(i, pk[i])


def recover_share(ctx, msgs, party_index, t, dk, nl, n_new):
    """get_ciphertext_sum + Paillier::decrypt + the pk_vec loop
    (refresh_message.rs:193-237, :439-464; add_party_message.rs:186-213):
    (new share, G * share, [pk_vec entry for each of the n_new parties]).

    Lagrange weights use the first t+1 messages in slice order.  The GPU
    decrypts each c_j and combines sum_j l_j * Dec(c_j) mod N: decryption is a
    homomorphism on units of Z_{N^2}, so this equals the reference's decryption
    of prod_j c_j^l_j * Enc(0) (the Enc(0) factor only re-randomises)."""
    indices = [msgs[j].old_party_index - 1 for j in range(t + 1)]
    li = [_lagrange(indices[j], indices) for j in range(t + 1)]
    cts = [msgs[j].points_encrypted_vec[party_index - 1] for j in range(t + 1)]
    sig = ctx.paillier_decrypt(cts, dk.p, dk.q, nl)
    new_share = sum(l * s for l, s in zip(li, sig)) % (dk.p * dk.q) % Q
    pts = [[(GX, GY)]] + [[msgs[j].points_committed_vec[i] for j in range(t + 1)] for i in range(n_new)]
    scs = [[new_share]] + [li[:] for _ in range(n_new)]
    # one MSM launch: y = G*x, then pk_vec[i] = sum_j P_j,i * l_j  (rows padded to t+1 terms)
    width = t + 1
    pts = [row + [None] * (width - len(row)) for row in pts]
    scs = [row + [0] * (width - len(row)) for row in scs]
    res = ctx.ec_msm(pts, scs)
    return new_share, res[0], res[1:]
