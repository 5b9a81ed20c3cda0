"""Host-side mirror of JoinMessage::collect (/root/reference/src/add_party_message.rs:136-294)
over the MI355X C ABI.

A joining party checks only what the reference checks there: validate_collect
(threshold, sizes, Feldman shares -- fsdkr_feldman_check) and every
ring-Pedersen proof (fsdkr_ring_pedersen_verify, one batched launch for all
refresh and join messages); then it recovers its share (GPU decryption + MSM)
and assembles the new LocalKey.  Errors are the reference's FsDkrError variant
and payload for the first failing check, in the reference's order.  There is no
CPU fallback."""
import secrets

from .batch import UnsupportedInput
from .refresh import GX, GY, Q, FsDkrError, FsDkrPanic, _ctx, recover_share
from .types import DLogStatement, EncryptionKey, LocalKey, VerifiableSS


def _nl_for(bits):
    if bits <= 2048:
        return 64
    if bits <= 3072:
        return 96
    raise UnsupportedInput(f"{bits}-bit modulus")


def validate_collect(ctx, refresh_messages, t, n):
    """RefreshMessage::validate_collect (refresh_message.rs:147-191), Feldman on the GPU."""
    msgs = list(refresh_messages)
    if len(msgs) <= t:
        raise FsDkrError("PartiesThresholdViolation", threshold=t, refreshed_keys=len(msgs))
    ref = len(msgs[0].pdl_proof_vec)
    for k, m in enumerate(msgs):
        a, b, c = len(m.pdl_proof_vec), len(m.points_committed_vec), len(m.points_encrypted_vec)
        if not (a == ref and b == ref and c == ref):
            raise FsDkrError("SizeMismatchError", refresh_message_index=k, pdl_proof_len=a,
                             points_commited_len=b, points_encrypted_len=c)
    # validate_share_public reads points_committed_vec[i] for i < n: message 0's first
    # `ref` shares are checked, then the index past the end panics
    rows = min(ref, n)
    groups = {}
    for k, m in enumerate(msgs):
        groups.setdefault(len(m.coefficients_committed_vec.commitments), []).append(k)
    ok = {}
    for ncoef, ks in groups.items():
        if ncoef == 0:       # curv get_point_commitment: head.unwrap() on an empty vector panics
            continue
        v = ctx.feldman_check([list(msgs[k].coefficients_committed_vec.commitments) for k in ks],
                              [msgs[k].points_committed_vec[i] for k in ks for i in range(rows)], rows, ncoef - 1)
        for q, k in enumerate(ks):
            ok[k] = v[q * rows:(q + 1) * rows]
    for k, m in enumerate(msgs):   # reference order: message by message, share by share
        if rows == 0 and ref < n:
            raise FsDkrPanic("validate_collect: points_committed_vec[i] out of bounds")
        if k not in ok:
            raise FsDkrPanic("validate_share_public: empty commitment vector (unwrap)")
        if not ok[k].all():
            raise FsDkrError("PublicShareValidationError")
        if ref < n:
            raise FsDkrPanic("validate_collect: points_committed_vec[i] out of bounds")


def verify_ring_pedersen(ctx, messages, m_security=256):
    """RingPedersenProof::verify for each message (statement, proof), in order:
    list of per-message outcomes 'ok' | 'err' | 'panic' (ring_pedersen_proof.rs:126-157)."""
    res = [None] * len(messages)
    good = []
    for k, m in enumerate(messages):
        p = m.ring_pedersen_proof
        if len(p.A) < m_security or len(p.Z) < m_security:
            res[k] = "panic"        # A[i] / Z[i] index panic
        else:
            good.append(k)
    if good:
        bits = max(max(messages[k].ring_pedersen_statement.N.bit_length() for k in good), 1)
        v = ctx.ring_pedersen_verify([messages[k].ring_pedersen_statement for k in good],
                                     [messages[k].ring_pedersen_proof for k in good], m_security, _nl_for(bits))
        for k, b in zip(good, v.tolist()):
            res[k] = "ok" if b & 1 else "panic" if b & 2 else "err"
    return res


def vss_share(ctx, t, n, secret, sample_below=None):
    """VerifiableSS::share(t, n, secret) commitments (curv feldman_vss [dep]): a
    random degree-t polynomial with constant term `secret` and a non-zero top
    coefficient; commitments G*a_k via one GPU MSM launch."""
    draw = sample_below or secrets.randbelow
    coeffs = [secret % Q] + [draw(Q) for _ in range(t)]
    while t > 0 and coeffs[-1] == 0:
        coeffs[-1] = draw(Q)
    com = ctx.ec_msm([[(GX, GY)] for _ in coeffs], [[a] for a in coeffs])
    return VerifiableSS(threshold=t, share_count=n, commitments=com)


def collect(self_msg, refresh_messages, paillier_key, join_messages, t, n, ctx=None, m_security=256,
            missing_dlog_statement=None, sample_below=None, key_bits=2048, rng=None):
    """JoinMessage::collect (add_party_message.rs:136-294) -> LocalKey.

    A party index with no message gets a freshly generated DLogStatement, as
    the reference does (:257-266 -> generate_dlog_statement_proofs().0, a new
    PAILLIER_KEY_SIZE keypair with h2 = h1^xhi, :50-66): by default on the GPU
    (fsdkr.distribute.generate_h1_h2_n_tilde: batched prime search + modexp;
    the two composite proofs the reference computes and discards are skipped).
    `missing_dlog_statement(party)` overrides it (injected statements);
    `rng` (sample_below(upper)) injects the generator's randomness and
    `sample_below` that of the new VSS polynomial (:279)."""
    ctx = _ctx(ctx)
    msgs, joins = list(refresh_messages), list(join_messages)
    validate_collect(ctx, msgs, t, n)
    outcome = verify_ring_pedersen(ctx, msgs + joins, m_security)
    for k, m in enumerate(msgs):                                       # :146-154
        if outcome[k] == "panic":
            raise FsDkrPanic("RingPedersenProof::verify panics (short challenge or proof vector)")
        if outcome[k] == "err":
            raise FsDkrError("RingPedersenProofValidation", party_index=m.party_index)
    for j, jm in enumerate(joins):                                     # :156-167
        o = outcome[len(msgs) + j]
        if o == "panic":
            raise FsDkrPanic("RingPedersenProof::verify panics (short challenge or proof vector)")
        if o == "err":
            if jm.party_index is not None:
                raise FsDkrError("RingPedersenProofValidation", party_index=jm.party_index)
            raise FsDkrError("RingPedersenProofError")
    party_index = self_msg.party_index                                 # :170
    if party_index is None:
        raise FsDkrError("NewPartyUnassignedIndexError")
    for jm in joins:                                                   # :174-176
        if jm.party_index is None:
            raise FsDkrError("NewPartyUnassignedIndexError")
    if len(msgs) < t + 1:
        raise FsDkrPanic("get_ciphertext_sum: refresh_messages[i] out of bounds")
    nl = _nl_for(max(paillier_key.ek.n.bit_length(), 1))
    new_share, y, pk_vec = recover_share(ctx, msgs, party_index, t, paillier_key.dk, nl, n)   # :183-213
    # party -> ek / DLogStatement; later entries of the chain win, as in HashMap::collect (:217-241)
    eks, sts = {}, {}
    for m in msgs:
        eks[m.party_index] = m.ek
        sts[m.party_index] = m.dlog_statement
    eks[party_index] = paillier_key.ek
    sts[party_index] = self_msg.dlog_statement
    for jm in joins:
        eks[jm.party_index] = jm.ek
        sts[jm.party_index] = jm.dlog_statement
    paillier_key_vec = [eks.get(p, EncryptionKey(0, 0)) for p in range(1, n + 1)]         # :244-256
    h1_h2 = []
    for p in range(1, n + 1):                                          # :258-267
        if p in sts:
            h1_h2.append(sts[p])
        elif missing_dlog_statement is not None:
            h1_h2.append(missing_dlog_statement(p))
        else:
            from .distribute import SystemRng, generate_h1_h2_n_tilde
            n_tilde, h1, h2, _, _ = generate_h1_h2_n_tilde(ctx, rng or SystemRng(), key_bits)
            h1_h2.append(DLogStatement(n_tilde, h1, h2))
    for m in msgs:                                                     # :271-275
        if m.public_key != msgs[0].public_key:
            raise FsDkrError("BroadcastedPublicKeyError")
    vss = vss_share(ctx, t, n, new_share, sample_below)                # :278-279
    return LocalKey(paillier_dk=paillier_key.dk, pk_vec=list(pk_vec), x_i=new_share, y=y,
                    paillier_key_vec=paillier_key_vec, y_sum_s=msgs[0].public_key, h1_h2_n_tilde_vec=h1_h2,
                    vss_scheme=vss, i=party_index, t=t, n=n)


__all__ = ["collect", "validate_collect", "verify_ring_pedersen", "vss_share", "DLogStatement"]
