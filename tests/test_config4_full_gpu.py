"""BASELINE configs[4] at its full size through the bench's exact call: 1 024
independent t=1 n=3 RefreshMessage::collect sessions (refresh_message.rs:321-467
per session) with 3072-bit keys, verified by ONE refresh.collect_many pass with
its staged prestart (GA chains, table chains and comb tables, the correct-key
job, the ring-Pedersen T^Z exponents behind the T tables).

At this size the launches take the throughput shapes the bench times
(4-lane 3072/6144-bit modexp and comb launches, the prestarted T^Z path), which
the 24-session test in test_configs_gpu.py does not reach.  Tampers of every
job family sit in a few sessions; each session's outcome must equal the
oracle's (tamper.expected), untampered neighbours must succeed, and sampled
untampered sessions must end with the oracle's LocalKey.  A stale T^Z prestart
(Z rows of one session changed after the prestart) must be recomputed, not
reused (fsdkr_collect_reuse_mask)."""
import copy
import dataclasses
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import tamper  # noqa: E402

pytestmark = pytest.mark.gpu

S = 1024
SEED = 2028          # bench.py's configs[4] workload (--seed 2024 + 4)
KB = 3072
# session -> tamper spec [(kind, k, i)]: GA's s2^N chain, the prestarted T^Z
# exponents, the correct-key job, the Alice challenge, Feldman, the ciphertext
# (GA's joint c^-e and the hashes), the h2 fixed base, the Alice z^e chain
TAMPERS = {5: [("pdl_s2", 1, 2)], 130: [("rp_Z", 2, 200)], 333: [("ck", 0, 0)], 512: [("range_e", 2, 1)],
           700: [("feldman", 1, 0)], 901: [("enc", 0, 2)], 1000: [("pdl_s3", 2, 0)], 1023: [("range_z", 1, 1)]}
SAMPLED = (0, 257, 640, 1022)


@pytest.fixture(scope="module")
def sessions(gpu_ctx):
    from fsdkr import synth
    return synth.synth_sessions(gpu_ctx, S, n=3, t=1, seed=SEED, key_bits=KB)


def _work(sessions):
    work, expect = [], {}
    for s, (msgs, joins, lk, dk) in enumerate(sessions):
        if s in TAMPERS:
            msgs, joins = tamper.inject(msgs, joins, TAMPERS[s])
            first = tamper.expected(msgs, joins, lk, TAMPERS[s], KB)[3]
            assert first is not None, s
            expect[s] = first
        work.append((msgs, copy.deepcopy(lk), dk, joins))
    return work, expect


def _outcome(r):
    return None if r is None else (r.variant, r.fields)


def test_config4_1024_sessions_tampers_vs_oracle(gpu_ctx, sessions):
    from fsdkr import refresh
    from oracle import protocol
    from oracle.rng import Rng
    work, expect = _work(sessions)
    res = refresh.collect_many(work, ctx=gpu_ctx, key_bits=KB)
    assert {"ga", "tables", "tz"} <= gpu_ctx.collect_reuse()   # the prestarted path was the one that ran
    bad = [(s, _outcome(r), expect.get(s)) for s, r in enumerate(res) if _outcome(r) != expect.get(s)]
    assert not bad, bad[:8]
    for s in SAMPLED:
        msgs, joins, lk, dk = sessions[s]
        ko = copy.deepcopy(lk)
        protocol.collect(tamper.to_oracle(msgs), ko, dk, [], Rng("a8"), KB)
        got = work[s][1]
        assert (ko.x_i, ko.y, ko.pk_vec) == (got.x_i, got.y, got.pk_vec), s
        assert [k.n for k in ko.paillier_key_vec] == [k.n for k in got.paillier_key_vec], s


def test_config4_1024_sessions_stale_tz_prestart(gpu_ctx, sessions):
    """The T^Z prestart of a set whose Z rows differ in one session (another
    message than the tampered one) must not be reused for the real set: the
    prepare recomputes T^Z, the rp_Z tamper is still caught in its own session,
    and every other session's first error equals the oracle's."""
    from fsdkr.batch import SessionSet
    from fsdkr.refresh import _error_of
    work, expect = _work(sessions)
    target = [(m, lk, j) for m, lk, dk, j in work]
    other = list(target)
    m0, lk0, j0 = other[77]
    msgs = list(m0)
    rp = msgs[1].ring_pedersen_proof
    msgs[1] = copy.copy(msgs[1])
    msgs[1].ring_pedersen_proof = dataclasses.replace(rp, Z=tuple(z + (j == 3) for j, z in enumerate(rp.Z)))
    other[77] = (msgs, lk0, j0)
    pre = SessionSet(other, 256, KB, staged=True)
    assert pre.n_prestart == S
    gpu_ctx.collect_prestart_set(pre)
    assert pre.stage1b()
    gpu_ctx.collect_prestart_set(pre)
    assert pre.stage_z()
    gpu_ctx.collect_prestart_rp_set(pre)
    sset = SessionSet(target, 256, KB)
    gpu_ctx.collect_prepare_set(sset)
    reused = gpu_ctx.collect_reuse()
    assert "tz" not in reused and "tables" in reused
    gpu_ctx.collect_launch()
    v = gpu_ctx.collect_finish_set(sset)
    got = [_outcome(_error_of(sset.first_error(s, v))) for s in range(S)]
    bad = [(s, got[s], expect.get(s)) for s in range(S) if got[s] != expect.get(s)]
    assert not bad, bad[:8]
    # and a prestart of exactly this set is consumed with the same verdicts
    pre = SessionSet(target, 256, KB, staged=True)
    gpu_ctx.collect_prestart_set(pre)
    assert pre.stage1b()
    gpu_ctx.collect_prestart_set(pre)
    assert pre.stage_z()
    gpu_ctx.collect_prestart_rp_set(pre)
    sset2 = SessionSet(target, 256, KB)
    gpu_ctx.collect_prepare_set(sset2)
    assert "tz" in gpu_ctx.collect_reuse()
    gpu_ctx.collect_launch()
    v2 = gpu_ctx.collect_finish_set(sset2)
    for s in range(S):
        assert sset2.first_error(s, v2).variant == sset.first_error(s, v).variant, s
