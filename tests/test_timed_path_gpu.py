"""Full-size tamper tests of the TIMED path: refresh.collect() -- bench.py's step,
with its staged prestart (GA's split chains and their joint tail, the h1 / h2 / T
table chains and comb tables) -- at BASELINE configs[2] (60 refresh + 4 join
messages, n = 64, t = 32) and configs[3] (n = 256, t = 128, 256 distinct
messages), 2048-bit keys.

Tampers go into the inputs of the prestarted and joined jobs: PDL s2 and Alice s
(GA's chains), the ciphertext c (the joint tail's c^-1 and both proofs), PDL z
(z^e), PDL s1 / s3 and ring-Pedersen Z (the comb exponents), a ring-Pedersen A
(the challenge hash), a share commitment (Feldman), a correct-key sigma and a
join's DLog proof.  The raised FsDkrError must be the oracle's first error in
the reference order (refresh_message.rs:321-437, tests/tamper.expected: the
oracle verifies every tampered instance), paillier_key_vec must carry exactly
the writes the reference makes before that check (:394, :436), and the clean
batch must update the LocalKey.  A second variant prestarts the CLEAN batch and
prepares the tampered one: every prestarted part the tamper touches must be
recomputed (fsdkr_collect_reuse_mask), so the verdicts still equal the oracle's
(this fails if prepare trusted a stale prestart)."""
import copy
import dataclasses
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import tamper  # noqa: E402

pytestmark = pytest.mark.gpu


def _collect(ctx, msgs, joins, lk, dk):
    from fsdkr import refresh
    key = copy.deepcopy(lk)
    try:
        refresh.collect(msgs, key, dk, joins, ctx=ctx, key_bits=2048)
        out = None
    except refresh.FsDkrError as e:
        out = (e.variant, e.fields)
    return out, key


def _keys_written(msgs, joins, first):
    """messages whose ek the reference writes into paillier_key_vec before `first`"""
    allm = list(msgs) + list(joins)
    if first is None:
        return len(allm)
    variant, fields = first
    if variant in ("PaillierVerificationError", "DLogProofValidation", "ModuliTooSmall"):
        pi = fields["party_index"]
        return next(k for k, m in enumerate(allm) if m.party_index == pi)
    return 0


def _check_side_effects(lk, key, msgs, joins, first):
    applied = _keys_written(msgs, joins, first)
    want = [e.n for e in lk.paillier_key_vec]
    for m in (list(msgs) + list(joins))[:applied]:
        want[m.party_index - 1] = m.ek.n
    assert [e.n for e in key.paillier_key_vec] == want
    if first is not None:   # no share recovery applied
        assert (key.x_i, key.y, key.pk_vec) == (lk.x_i, lk.y, lk.pk_vec)


def _timed_cases(ctx, msgs, joins, lk, dk, cases):
    """refresh.collect on each tampered batch: the oracle's first error, the
    reference's key writes; the clean batch updates the LocalKey."""
    got, key = _collect(ctx, msgs, joins, lk, dk)
    assert got is None, got
    assert key.x_i != lk.x_i and len(key.pk_vec) == len(msgs) + len(joins)
    for spec in cases:
        m2, j2 = tamper.inject(msgs, joins, spec)
        first = tamper.expected(m2, j2, lk, spec, 2048)[3]
        assert first is not None, spec
        got, key = _collect(ctx, m2, j2, lk, dk)
        assert got == first, (spec, got, first)
        _check_side_effects(lk, key, m2, j2, first)


def _stale_prestart(ctx, msgs, joins, lk, spec, must_miss):
    """prestart the clean batch, prepare the tampered one: the parts that read a
    tampered field are recomputed and the verdicts equal the oracle's"""
    from fsdkr.batch import CollectBatch
    from fsdkr.refresh import prestart
    R, J = len(msgs), len(joins)
    m2, j2 = tamper.inject(msgs, joins, spec)
    pairs, mres, jres, first = tamper.expected(m2, j2, lk, spec, 2048)
    prestart(ctx, CollectBatch(msgs, lk, joins, 256, 2048, staged=True))
    b = CollectBatch(m2, lk, j2, 256, 2048)
    ctx.collect_prepare(b)
    assert not (ctx.collect_reuse() & must_miss), (spec, ctx.collect_reuse())
    v = ctx.collect_run(b)
    tamper.check_verdicts(v, R, J, R + J, pairs, mres, jres)


def _local(lk):
    return lk.i - 1


# ------------------------------------------------------------------ configs[2]
@pytest.fixture(scope="module")
def timed2(gpu_ctx):
    from fsdkr import synth
    msgs, joins, lk = synth.synth_collect(gpu_ctx, 60, 4, 32, 5151, key_bits=2048)
    return msgs, joins, lk, lk.paillier_dk


def test_timed_path_config2_tampers(gpu_ctx, timed2):
    msgs, joins, lk, dk = timed2
    o = (_local(lk) + 1) % 64   # a receiver other than the local party (its c feeds the share recovery)
    cases = [[("pdl_s2", 3, o)], [("range_s", 11, 40)], [("enc", 20, o)], [("pdl_z", 25, 9)], [("pdl_s1", 31, 12)],
             [("pdl_s3", 36, 63)], [("rp_Z", 45, 128)], [("rp_A", 62, 7)], [("feldman", 50, 33)], [("ck", 57, 0)],
             [("dlog", 2, 0)], [("range_e", 8, 1), ("rp_A", 3, 0)]]
    _timed_cases(gpu_ctx, msgs, joins, lk, dk, cases)


@pytest.mark.parametrize("spec,must_miss", [
    ([("pdl_s2", 14, 5)], {"ga"}),
    ([("range_s", 40, 2)], {"ga"}),
    ([("enc", 7, 3)], set()),          # GA's head is reused; its joint tail reads c in prepare
    ([("pdl_s3", 22, 17)], set()),     # the tables are sized by bounds; the exponents are prepare's
])
def test_timed_path_config2_stale_prestart(gpu_ctx, timed2, spec, must_miss):
    msgs, joins, lk, dk = timed2
    _stale_prestart(gpu_ctx, msgs, joins, lk, spec, must_miss)


def test_timed_path_config2_negative_operands(gpu_ctx, timed2):
    """VERDICT r4 item 8 at full size: one sender's negative PDL s1 -> that pair's
    panic (zk_pdl_with_slack.rs:139), no key written (the PDL loop precedes every
    write); s2 - N^2 in another pair (GA's base: the same residue) -> Ok, with the
    LocalKey the clean batch gives; a negative s3 -> that pair's u3 fails."""
    from fsdkr import refresh
    msgs, joins, lk, dk = timed2
    m2 = list(msgs)
    m = tamper._own(m2, 17)
    p = m.pdl_proof_vec[9]
    m.pdl_proof_vec[9] = dataclasses.replace(p, s1=-p.s1)
    key = copy.deepcopy(lk)
    with pytest.raises(refresh.FsDkrPanic):
        refresh.collect(m2, key, dk, joins, ctx=gpu_ctx, key_bits=2048)
    _check_side_effects(lk, key, m2, joins, ("PDLwSlackProof", {}))
    m3 = list(msgs)
    m = tamper._own(m3, 40)
    p = m.pdl_proof_vec[5]
    m.pdl_proof_vec[5] = dataclasses.replace(p, s2=p.s2 - lk.paillier_key_vec[5].n ** 2)
    got, key3 = _collect(gpu_ctx, m3, joins, lk, dk)
    assert got is None, got
    ref, key0 = _collect(gpu_ctx, msgs, joins, lk, dk)
    assert (key3.x_i, key3.y, key3.pk_vec) == (key0.x_i, key0.y, key0.pk_vec)
    # a sign-flipped s3 is an h2^-1 exponent (zk_pdl_with_slack.rs:177-184): the
    # pair's u3 alone fails (pdl_s3_neg; |s3| into the prestarted comb tables)
    m4 = list(msgs)
    m = tamper._own(m4, 23)
    p = m.pdl_proof_vec[11]
    m.pdl_proof_vec[11] = dataclasses.replace(p, s3=-p.s3)
    got, _ = _collect(gpu_ctx, m4, joins, lk, dk)
    assert got == ("PDLwSlackProof", {"is_u1_eq": True, "is_u2_eq": True, "is_u3_eq": False}), got


# ------------------------------------------------------------------ configs[3]
def test_timed_path_config3_n256_tampers(gpu_ctx):
    from fsdkr import synth
    msgs, joins, lk = synth.synth_collect(gpu_ctx, 256, 0, 128, 6161, key_bits=2048)
    dk = lk.paillier_dk
    o = (_local(lk) + 5) % 256
    cases = [[("pdl_s2", 200, o)], [("enc", 13, o), ("range_s", 100, 250)], [("pdl_s3", 77, 1)], [("rp_Z", 255, 3)],
             [("ck", 129, 0)]]
    _timed_cases(gpu_ctx, msgs, joins, lk, dk, cases)
    _stale_prestart(gpu_ctx, msgs, joins, lk, [("pdl_s2", 90, 91)], {"ga"})
