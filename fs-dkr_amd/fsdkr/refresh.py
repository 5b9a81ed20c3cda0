"""Host-side mirror of RefreshMessage::collect (/root/reference/src/refresh_message.rs:321-467)
over the MI355X C ABI.

Same argument meaning and error behaviour as the reference: returns None on
success after mutating `local_key` exactly as collect() does, raises
FsDkrError with the reference's variant name and payload for the FIRST failing
check (or FsDkrPanic where the reference panics).  All proof verification runs
in one batched GPU pass (fsdkr_collect_launch/finish); the share recovery
(decryption + pk_vec MSM) by default runs speculatively on the context's
recovery stream WHILE the proofs are verified and is discarded if a check
fails (its result is deterministic, so running it early changes nothing but
the latency).  This departs from the reference, which decrypts with the old
secret key only after every check has passed (:439); `recovery="after"`
restores that order (decrypt once the verdicts are in; same LocalKey and
outcome, tests/test_reference_scenarios_gpu.py), at the cost of the overlap.
The share recovery's own panics keep the reference's place in the error order:
get_ciphertext_sum (:367-373) panics before the correct-key / moduli / DLog
checks and before any paillier_key_vec write; decryption and the pk_vec loop
(:439-464) after them.
collect_many() verifies many independent sessions in one device pass
(BASELINE configs[4]).  There is no CPU fallback."""
from ._native import RECOVER_NO_DECRYPT, Context
from .batch import CollectBatch, SessionSet

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


class _DecryptPanic(FsDkrPanic):
    """Paillier::decrypt panics on a degenerate decryption key (p or q even or 1,
    p == q): after every check (refresh_message.rs:439)."""


class _SumPanic(FsDkrPanic):
    """get_ciphertext_sum panics (refresh_message.rs:367-373: the old ek, a
    message's ciphertext for this party, the first t+1 old indices, a repeated
    index in the Lagrange set): after the ring-Pedersen checks, before the
    correct-key / moduli / DLog checks and before any paillier_key_vec write."""


# first_error variants the reference reaches only after get_ciphertext_sum (:375-437)
_AFTER_SUM = (7, 8, 9, 11)
RECOVERY_MODES = ("speculative", "after")


def _lagrange(index, s):
    """curv VerifiableSS::map_share_to_new_params: Lagrange coefficient at 0."""
    xi = index + 1
    num, den = 1, 1
    for j in s:
        if j == index:
            continue
        num = num * (j + 1) % Q
        den = den * ((j + 1) - xi) % Q
    if den == 0:
        raise FsDkrPanic("map_share_to_new_params: repeated party index (zero inverse)")
    return num * pow(den, -1, Q) % Q


_default_ctx = None


def _ctx(ctx):
    global _default_ctx
    if ctx is not None:
        return ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx


def _whole_chip(ctx):
    """A single-GPU collect uses every CU: undo a shard slice's GA split
    (fsdkr_ctx_set_cu_split returns at once when nothing changes)."""
    if hasattr(ctx, "set_cu_split"):
        ctx.set_cu_split(0)


def _error_of(err):
    """fsdkr_error -> None | FsDkrError | FsDkrPanic."""
    if err.variant == 0:
        return None
    name, fields = _VARIANTS[err.variant]
    vals = {f: (bool(err.f[k]) if f in _BOOL_FIELDS else int(err.f[k])) for k, f in enumerate(fields)}
    e = FsDkrPanic(f"reference panics at {name}") if err.panic else FsDkrError(name, **vals)
    e.code = err.variant
    return e


def _short_share_check(ctx, batch, msgs):
    """validate_collect with points_committed_vec shorter than new_n (:177-188):
    message 0's first `ref` shares are checked, then index `ref` panics."""
    m = msgs[0]
    com = list(m.coefficients_committed_vec.commitments)
    ref = batch.ref_len
    if ref and com:
        ok = ctx.feldman_check([com], list(m.points_committed_vec[:ref]), ref, len(com) - 1)
        if not ok.all():
            return FsDkrError("PublicShareValidationError")
    return FsDkrPanic("validate_collect: points_committed_vec[i] out of bounds")


def _mapped(ctx, batch, msgs, verdicts):
    """(error or None, keys_applied) of one session."""
    err = batch.first_error(verdicts)
    e = _error_of(err)
    if isinstance(e, FsDkrPanic) and err.variant == 2 and batch.size_fail and not batch.c.n_recv and \
            batch.R > batch.c.t and batch.ref_len < batch.n:
        e = _short_share_check(ctx, batch, msgs)
    return e, err.keys_applied


def verify(refresh_messages, local_key, join_messages, ctx=None, m_security=256, key_bits=2048):
    """Verification half of collect(): (error or None, keys_applied, batch)."""
    ctx = _ctx(ctx)
    msgs = list(refresh_messages)
    batch = CollectBatch(msgs, local_key, join_messages, m_security, key_bits)
    verdicts = None if batch.header_only else ctx.verify_collect(batch)
    err, applied = _mapped(ctx, batch, msgs, verdicts)
    return err, applied, batch


def _apply_keys(local_key, msgs, joins, applied):
    # paillier_key_vec is written message by message before a later check fails (:394, :436)
    for k, m in enumerate(msgs + joins):
        if k >= applied:
            break
        local_key.paillier_key_vec[m.party_index - 1] = m.ek


def _apply_share(local_key, new_dk, rec):
    new_share, y, pk, t_ok = rec
    local_key.paillier_dk = new_dk
    local_key.x_i = new_share
    local_key.y = y
    for i in range(len(pk)):
        local_key.pk_vec.insert(i, pk[i])
    if not t_ok:   # li_vec[j] for j <= local_key.t past the vss threshold (:460-462)
        raise FsDkrPanic("collect: li_vec index out of bounds (local_key.t > vss threshold)")


def _settle(err, applied, spec):
    """The reference's order between the verification outcome (err, keys
    applied) and the share recovery's (spec: the recovery tuple or the panic it
    hits): a get_ciphertext_sum panic wins over every later check and precedes
    every key write; a decryption / pk_vec panic comes after all checks."""
    if isinstance(spec, _SumPanic) and (err is None or getattr(err, "code", None) in _AFTER_SUM):
        return spec, 0
    if err is None and isinstance(spec, Exception):
        return spec, applied
    return err, applied


def _conclude(local_key, new_dk, msgs, joins, err, applied, spec):
    """collect()'s side effects for one outcome; returns the error collect() raises (or None)."""
    err, applied = _settle(err, applied, spec)
    _apply_keys(local_key, msgs, joins, applied)
    if err is None:
        try:
            _apply_share(local_key, new_dk, spec)
        except FsDkrPanic as e:
            err = e
    return err


def _needs_recovery(err):
    return err is None or getattr(err, "code", None) in _AFTER_SUM


def _recover_after(ctx, jobs, errs):
    """recovery="after": decrypt only for the jobs whose checks all passed (the
    reference's :439); jobs stopped by a later check still get their
    get_ciphertext_sum panic, which the reference hits first."""
    out = [None] * len(jobs)
    live = []
    for k, (job, err) in enumerate(zip(jobs, errs)):
        if not _needs_recovery(err):
            continue
        if err is None:
            live.append(k)
            continue
        try:
            _recovery_plan(*job)
        except _SumPanic as e:
            out[k] = e
        except Exception:   # a later (decryption / pk_vec) panic: the check's error comes first
            pass
    if live:
        for k, r in zip(live, _speculative(ctx, [jobs[k] for k in live])):
            out[k] = r
    return out


def _check_mode(recovery):
    if recovery not in RECOVERY_MODES:
        raise ValueError(f"recovery must be one of {RECOVERY_MODES}")


def prestart(ctx, batch):
    """The staged starts of a CollectBatch(..., staged=True) before complete():
    stage 1 (GA's fields) -> fsdkr_collect_prestart starts GA; stage 1b (the
    tables' bases and exponents) -> the table chains and comb tables start beside
    it.  Each call finds GA running and starts what the newly packed fields allow."""
    if not batch.ga_ready or not hasattr(ctx, "collect_prestart"):
        return
    ctx.collect_prestart(batch)
    if batch.stage1b():
        ctx.collect_prestart(batch)


def collect(refresh_messages, local_key, new_dk, join_messages, ctx=None, m_security=256, key_bits=2048,
            recovery="speculative"):
    """RefreshMessage::collect (refresh_message.rs:321-467).  `recovery`:
    "speculative" (default) decrypts the new share while the proofs are verified;
    "after" decrypts once every check has passed, as the reference does (:439)."""
    _check_mode(recovery)
    ctx = _ctx(ctx)
    _whole_chip(ctx)
    msgs, joins = list(refresh_messages), list(join_messages)
    job = (msgs, local_key, len(msgs) + len(joins))
    # stage 1 packs what the pipeline's longest job reads and starts it on the GPU;
    # the rest of the batch is packed while those chains run
    batch = CollectBatch(msgs, local_key, joins, m_security, key_bits, staged=True)
    prestart(ctx, batch)
    spec, verdicts, pend = None, None, None
    batch.complete()
    if not batch.header_only:
        ctx.collect_prepare(batch)
        ctx.collect_launch()
        try:   # the share recovery's host pre-pass and GPU work overlap the pipeline
            if recovery == "speculative":
                pend = _speculative_launch(ctx, [job])
        finally:   # neither the batch nor the recovery stays in flight
            verdicts, specs = _finish_both(ctx, lambda: ctx.collect_finish(batch), pend)
            if specs is not None:
                spec = specs[0]
    err, applied = _mapped(ctx, batch, msgs, verdicts)
    if recovery == "after" or batch.header_only:
        spec = _recover_after(ctx, [job], [err])[0]
    err = _conclude(local_key, new_dk, msgs, joins, err, applied, spec)
    if err is not None:
        raise err


def collect_many(sessions, ctx=None, m_security=256, key_bits=2048, recovery="speculative"):
    """Many independent RefreshMessage::collect calls verified in ONE device pass
    (fsdkr_collect_prepare_multi; BASELINE configs[4]).  `sessions`: list of
    (refresh_messages, local_key, new_dk, join_messages).  Each session gets the
    reference's outcome on its own: returns a list with None (local_key
    updated as collect() does) or the FsDkrError / FsDkrPanic collect() would
    raise (local_key partially updated as collect() leaves it)."""
    _check_mode(recovery)
    ctx = _ctx(ctx)
    _whole_chip(ctx)
    sess = [(list(r), lk, dk, list(j)) for r, lk, dk, j in sessions]
    jobs = [(msgs, lk, len(msgs) + len(joins)) for msgs, lk, dk, joins in sess]
    # one gather across the sessions (SessionSet); sessions of another shape keep
    # their own batch, header-only ones are mapped without a device pass
    sset = SessionSet([(r, lk, j) for r, lk, dk, j in sess], m_security, key_bits, staged=True)
    if sset.n_prestart:   # every session's s2^N, s^N mod N^2 chains start while the rest is packed
        ctx.collect_prestart_set(sset)
        if sset.stage1b():   # the table bases and correct-key inputs: those jobs start beside GA
            ctx.collect_prestart_set(sset)
        if sset.stage_z():   # then the ring-Pedersen T^Z exponents behind the T tables
            ctx.collect_prestart_rp_set(sset)
    sset.complete()
    live = sset.live
    specs = [None] * len(sess)
    verdicts, pend = None, None
    if live:
        ctx.collect_prepare_set(sset)
        ctx.collect_launch()
        try:   # the share recovery's host pre-pass and GPU work overlap the pipeline
            if recovery == "speculative":
                pend = _speculative_launch(ctx, [jobs[i] for i in live])
        finally:   # neither the batch nor the recovery stays in flight
            verdicts, rs = _finish_both(ctx, lambda: ctx.collect_finish_set(sset), pend)
            for i, r in zip(live, rs or ()):
                specs[i] = r
    errs = []
    fe = sset.first_errors(verdicts) if sset.row else {}
    for i, (msgs, lk, dk, joins) in enumerate(sess):
        if i in fe:
            e = fe[i]
            errs.append((_error_of(e), e.keys_applied))
        else:
            errs.append(_mapped(ctx, sset.batches[i], msgs, None))
    late = [i for i in range(len(sess)) if recovery == "after" or i not in sset.row]
    for i, r in zip(late, _recover_after(ctx, [jobs[i] for i in late], [errs[i][0] for i in late])):
        specs[i] = r
    return [_conclude(lk, dk, msgs, joins, errs[i][0], errs[i][1], specs[i])
            for i, (msgs, lk, dk, joins) in enumerate(sess)]


def _public_view(lk):
    """What verification reads from a LocalKey: the receivers' keys and statements."""
    return (lk.t, tuple(e.n for e in lk.paillier_key_vec),
            tuple((s.N, s.g, s.ni) for s in lk.h1_h2_n_tilde_vec))


def collect_all(refresh_messages, parties, join_messages, ctx=None, m_security=256, key_bits=2048,
                recovery="speculative"):
    """Every party's RefreshMessage::collect over the same broadcast messages,
    with the proofs verified ONCE.  In the reference each
    party runs collect() and re-verifies the same n^2 proofs (test.rs:328-331);
    verification reads only public LocalKey data (paillier_key_vec,
    h1_h2_n_tilde_vec, t), so parties whose public view agrees share one device
    pass, one first-error mapping and one batched share recovery (each party
    decrypts its own ciphertexts).  `parties`: list of (local_key, new_dk).
    Returns one outcome per party, as collect_many does: None (local_key
    updated) or the FsDkrError / FsDkrPanic collect() would raise."""
    _check_mode(recovery)
    ctx = _ctx(ctx)
    _whole_chip(ctx)
    msgs, joins = list(refresh_messages), list(join_messages)
    groups = {}
    for p, (lk, dk) in enumerate(parties):
        groups.setdefault(_public_view(lk), []).append(p)
    out = [None] * len(parties)
    for members in groups.values():
        lk0 = parties[members[0]][0]
        batch = CollectBatch(msgs, lk0, joins, m_security, key_bits, staged=True)
        prestart(ctx, batch)
        jobs = [(msgs, parties[p][0], len(msgs) + len(joins)) for p in members]
        specs = [None] * len(members)
        verdicts, pend = None, None
        batch.complete()
        if not batch.header_only:
            ctx.collect_prepare(batch)
            ctx.collect_launch()
            try:   # the share recovery's host pre-pass and GPU work overlap the pipeline
                if recovery == "speculative":
                    pend = _speculative_launch(ctx, jobs)
            finally:   # neither the batch nor the recovery stays in flight
                verdicts, rs = _finish_both(ctx, lambda: ctx.collect_finish(batch), pend)
                if rs is not None:
                    specs = rs
        err, applied = _mapped(ctx, batch, msgs, verdicts)
        if recovery == "after" or batch.header_only:
            specs = _recover_after(ctx, jobs, [err] * len(jobs))
        for p, spec in zip(members, specs):
            lk, dk = parties[p]
            out[p] = _conclude(lk, dk, msgs, joins, err, applied, spec)
    return out


def _dk_limbs(dk):
    """Limb width holding N = p q of a decryption key (and p^2, q^2)."""
    bits = max((dk.p * dk.q).bit_length(), 2 * dk.p.bit_length(), 2 * dk.q.bit_length())
    for w in (64, 96, 128, 192):
        if bits <= 32 * w:
            return w
    return None


def _speculative(ctx, jobs):
    """Share recovery of every job (msgs, local_key, n_new) in one
    fsdkr_collect_recover call on the recovery stream (GPU decryptions + one MSM
    launch).  Per job: the 4-tuple (share, y, pk_vec, t_ok) or the exception the
    reference raises there."""
    return _speculative_finish(ctx, _speculative_launch(ctx, jobs))


def _speculative_launch(ctx, jobs):
    """The host pre-pass of _speculative and the launch of its GPU work
    (fsdkr_collect_recover_launch); _speculative_finish collects the results.
    collect() launches it right after its pipeline, so the host pre-pass (the
    Lagrange weights: O(t^2) products at n = 256) overlaps the device work.
    A job is (msgs, local_key, n_new) or (msgs, local_key, n_new, (lo, hi),
    decrypt): a multi-GPU rank's part (fsdkr/shard.py), the pk_vec rows
    [lo, hi) and the decryption only if `decrypt`; the inputs of every row are
    still checked here, so every rank raises the same panic."""
    out = [None] * len(jobs)
    todo, cj = [], []
    for k, job in enumerate(jobs):
        msgs, lk, n_new = job[:3]
        lo, hi = job[3] if len(job) > 3 else (0, n_new)
        decrypt = job[4] if len(job) > 4 else True
        try:
            plan = _recovery_plan(msgs, lk, n_new)
            # the key's width and shape are checked on EVERY rank of a sharded call
            # (before the decrypt / no-decrypt split), so a key the decrypting rank
            # refuses makes every rank raise the same panic (fsdkr/shard.py)
            nl = _dk_limbs(lk.paillier_dk)
            if nl is None:
                raise FsDkrPanic("share recovery: decryption key wider than 6144 bits")
            # Paillier::mul / add / decrypt reduce their operands mod N^2 (powm and
            # mulm mod NN), so a ciphertext c + k N^2 -- or a negative one --
            # recovers like its residue: reduce here, the C ABI takes ciphertexts in
            # [0, 2^(64 nl)) (fsdkr.h)
            nn_ = (lk.paillier_dk.p * lk.paillier_dk.q) ** 2
            cts = [c % nn_ if nn_ and (c >= nn_ or c < 0) else abs(c) for c in plan["cts"]]   # p or q = 0: the GPU reports it
            if not decrypt:
                todo.append(k)
                cj.append(dict(nl=64, t_vss=plan["t_vss"], t_key=lk.t, old_index=plan["index"], cts=[0] *
                               (plan["t_vss"] + 1), p=1, q=1, points=plan["pts"][lo:hi], flags=RECOVER_NO_DECRYPT))
                continue
        except (FsDkrPanic, IndexError, AttributeError, TypeError) as e:
            out[k] = e if isinstance(e, FsDkrPanic) else FsDkrPanic(f"share recovery: {e!r}")
            continue
        todo.append(k)
        cj.append(dict(nl=nl, t_vss=plan["t_vss"], t_key=lk.t, old_index=plan["index"], cts=cts,
                       p=lk.paillier_dk.p, q=lk.paillier_dk.q, points=plan["pts"][lo:hi]))
    return out, todo, (ctx.collect_recover_launch(cj) if cj else None)


def _finish_both(ctx, finish, pend):
    """Finish the launched share recovery (pend, or None), then finish() the
    launched verification batch, each even when the other raises: neither stays
    in flight (a recovery left in flight would refuse every later
    fsdkr_collect_recover_launch on the context).  The recovery goes first: its
    GPU work ends well before the pipeline's, so its host combination overlaps
    the pipeline instead of following it (configs[4]: ~25 ms of 1024 sessions).
    Returns (finish()'s verdicts, the recovery results or None)."""
    specs = None
    try:
        if pend is not None:
            specs = _speculative_finish(ctx, pend)
    finally:
        verdicts = finish()
    return verdicts, specs


def _speculative_finish(ctx, pending):
    out, todo, handle = pending
    if handle is not None:
        for k, (status, share, y, pk) in zip(todo, ctx.collect_recover_finish(handle)):
            if status == 2:   # FSDKR_RECOVER_PANIC_DECRYPT
                out[k] = _DecryptPanic("share recovery: Paillier::decrypt (degenerate decryption key)")
            else:
                out[k] = (share, y, pk, status != 1)   # 1: FSDKR_RECOVER_PANIC_LI
    return out


def _recovery_plan(msgs, local_key, n_new):
    """get_ciphertext_sum (:193-237) + the pk_vec loop inputs (:455-464).

    Lagrange weights use the first t+1 messages in slice order, t = the vss
    threshold (local_key.vss_scheme.parameters); the pk_vec sum runs j over
    0..=local_key.t (:460).  The GPU decrypts each c_j and the host combines
    sum_j l_j * Dec(c_j) mod N: decryption is a homomorphism on units of
    Z_{N^2}, so this equals the reference's decryption of prod_j c_j^l_j *
    Enc(0) (the Enc(0) factor only re-randomises)."""
    try:   # get_ciphertext_sum (:367-373)
        i = local_key.i
        if i < 1:
            raise IndexError("party index 0")
        pkv = getattr(local_key, "paillier_key_vec", None)   # JoinMessage::collect passes its own ek
        if pkv is not None:
            pkv[i - 1]                                           # old_ek (:367)
        cts_all = [m.points_encrypted_vec[i - 1] for m in msgs]  # every message's ciphertext (:202-204)
        t_vss = local_key.vss_scheme.threshold
        indices = [msgs[j].old_party_index - 1 for j in range(t_vss + 1)]
        li = [_lagrange(indices[j], indices) for j in range(t_vss + 1)]
    except (IndexError, AttributeError, TypeError, FsDkrPanic) as e:
        raise _SumPanic(f"get_ciphertext_sum: {e}") from None
    cts = cts_all[:t_vss + 1]
    t_key = local_key.t
    terms = min(t_key, t_vss) + 1
    pts = [[msgs[j].points_committed_vec[i] for j in range(terms)] for i in range(n_new)]
    return {"t_vss": t_vss, "index": [msgs[j].old_party_index for j in range(t_vss + 1)], "cts": cts, "pts": pts}


def recover_share(ctx, msgs, party_index, t, dk, nl, n_new):
    """get_ciphertext_sum + Paillier::decrypt + the pk_vec loop
    (refresh_message.rs:193-237, :439-464; add_party_message.rs:186-213):
    (new share, G * share, [pk_vec entry for each of the n_new parties]),
    t = the threshold of both the Lagrange set and the pk_vec sum."""
    class _K:
        pass
    lk = _K()
    lk.vss_scheme = type("V", (), {"threshold": t})()
    lk.t, lk.i, lk.paillier_dk = t, party_index, dk
    r = _speculative(ctx, [(msgs, lk, n_new)])[0]
    if isinstance(r, Exception):
        raise r
    return r[0], r[1], r[2]
