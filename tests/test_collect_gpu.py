"""GPU parity of RefreshMessage::collect (fs-dkr_amd, HIP via the C ABI)
against the oracle (CPU restatement of refresh_message.rs:321-467).

For every scenario both sides run on the same seeded messages; the outcome
(Ok, or the FsDkrError variant + payload), the side effects on
paillier_key_vec and, on success, the whole updated LocalKey must be equal."""
import copy
import dataclasses

import pytest

from oracle import paillier, protocol
from oracle import secp256k1 as ec
from oracle import zk_pdl_with_slack as pdl
from oracle import range_proofs
from oracle.rng import Rng

pytestmark = pytest.mark.gpu

KB = 1024          # flows are size-independent; one test below runs 2048-bit keys


def _dkr(t, n, seed, key_bits=KB):
    rng = Rng(seed)
    keys = protocol.simulate_keygen(t, n, rng, key_bits)
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.distribute(key.i, key, n, rng, key_bits)
        msgs.append(m)
        dks.append(dk)
    return keys, msgs, dks, rng


def _both(msgs, key, dk, joins, key_bits=KB, ctx=None):
    """Run oracle and GPU collect on copies; return (oracle_result, gpu_result, oracle_key, gpu_key)."""
    from fsdkr import refresh
    ko, kg = key.clone(), key.clone()
    ro = rg = None
    try:
        protocol.collect(copy.deepcopy(msgs), ko, dk, copy.deepcopy(joins), Rng("a8"), key_bits)
    except protocol.FsDkrError as e:
        ro = (e.variant, e.fields)
    except Exception as e:  # PanicError
        ro = ("panic", type(e).__name__)
    try:
        refresh.collect(copy.deepcopy(msgs), kg, dk, copy.deepcopy(joins), ctx=ctx, key_bits=key_bits)
    except refresh.FsDkrError as e:
        rg = (e.variant, e.fields)
    except refresh.FsDkrPanic:
        rg = ("panic", "PanicError")
    return ro, rg, ko, kg


def _same_key(a, b):
    assert a.x_i == b.x_i
    assert a.y == b.y
    assert a.pk_vec == b.pk_vec
    assert [k.n for k in a.paillier_key_vec] == [k.n for k in b.paillier_key_vec]
    assert (a.paillier_dk.p, a.paillier_dk.q) == (b.paillier_dk.p, b.paillier_dk.q)


@pytest.fixture(scope="module")
def dkr5():
    return _dkr(2, 5, "collect-gpu-t2n5")


def test_collect_valid_t2_n5(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    for party in (0, 3):
        ro, rg, ko, kg = _both(msgs, keys[party], dks[party], [], ctx=gpu_ctx)
        assert ro is None and rg is None
        _same_key(ko, kg)


def test_collect_valid_2048(gpu_ctx):
    keys, msgs, dks, _ = _dkr(1, 3, "collect-gpu-2048", key_bits=2048)
    ro, rg, ko, kg = _both(msgs, keys[1], dks[1], [], key_bits=2048, ctx=gpu_ctx)
    assert ro is None and rg is None
    _same_key(ko, kg)


def test_collect_valid_3072(gpu_ctx):
    """BASELINE configs[4] shape: t=1, n=3 with PAILLIER_KEY_SIZE = 3072 (96-limb N,
    192-limb N^2), plus one tampered range proof."""
    keys, msgs, dks, _ = _dkr(1, 3, "collect-gpu-3072", key_bits=3072)
    ro, rg, ko, kg = _both(msgs, keys[2], dks[2], [], key_bits=3072, ctx=gpu_ctx)
    assert ro is None and rg is None
    _same_key(ko, kg)
    m2 = _tampered(msgs, lambda m: _bump_range(m, 1, 2, s=m[1].range_proofs[2].s + 1))
    ro, rg, _, _ = _both(m2, keys[0], dks[0], [], key_bits=3072, ctx=gpu_ctx)
    assert ro == ("RangeProof", {"party_index": 2}) and rg == ro


def _tampered(msgs, fn):
    m2 = copy.deepcopy(msgs)
    fn(m2)
    return m2


def _bump_pdl(m, k, i, **kw):
    p = m[k].pdl_proof_vec[i]
    m[k].pdl_proof_vec[i] = pdl.PDLwSlackProof(**{**p.__dict__, **kw})


def _bump_range(m, k, i, **kw):
    a = m[k].range_proofs[i]
    m[k].range_proofs[i] = range_proofs.AliceProof(**{**a.__dict__, **kw})


TAMPERS = {
    "feldman": lambda m: m[1].points_committed_vec.__setitem__(2, ec.mul(ec.G, 12345)),
    "pdl_u2": lambda m: _bump_pdl(m, 2, 1, u2=m[2].pdl_proof_vec[1].u2 + 1),
    "pdl_u3": lambda m: _bump_pdl(m, 0, 4, s3=m[0].pdl_proof_vec[4].s3 + 1),
    "pdl_u1": lambda m: _bump_pdl(m, 3, 0, s1=m[3].pdl_proof_vec[0].s1 + 1),
    "range_s2": lambda m: _bump_range(m, 1, 3, s2=m[1].range_proofs[3].s2 + 1),
    "range_s1_bound": lambda m: _bump_range(m, 4, 2, s1=ec.Q ** 3 + 1),
    "range_e": lambda m: _bump_range(m, 2, 2, e=m[2].range_proofs[2].e ^ 1),
    "ped_Z": lambda m: setattr(m[3], "ring_pedersen_proof", type(m[3].ring_pedersen_proof)(
        m[3].ring_pedersen_proof.A, tuple(z + (j == 7) for j, z in enumerate(m[3].ring_pedersen_proof.Z)))),
    "ck_sigma": lambda m: setattr(m[2], "dk_correctness_proof", type(m[2].dk_correctness_proof)(
        (m[2].dk_correctness_proof.sigma_vec[0] + 1,) + tuple(m[2].dk_correctness_proof.sigma_vec[1:]))),
}


@pytest.mark.parametrize("name", sorted(TAMPERS))
def test_collect_tampered(gpu_ctx, dkr5, name):
    keys, msgs, dks, _ = dkr5
    m2 = _tampered(msgs, TAMPERS[name])
    ro, rg, ko, kg = _both(m2, keys[0], dks[0], [], ctx=gpu_ctx)
    assert ro is not None, "tamper did not break the oracle"
    assert rg == ro
    # side effects before the failure (paillier_key_vec written per passing message)
    assert [k.n for k in ko.paillier_key_vec] == [k.n for k in kg.paillier_key_vec]


def test_pdl_soundness_vector(gpu_ctx, dkr5):
    """zk_pdl_with_slack.rs:268-331: encrypting x+1 with an honest-looking proof."""
    keys, msgs, dks, rng = dkr5
    m2 = copy.deepcopy(msgs)
    k, i = 1, 2
    ek = keys[0].paillier_key_vec[i]
    st0 = keys[0].h1_h2_n_tilde_vec[i]
    x = paillier.decrypt(keys[i].paillier_dk, msgs[k].points_encrypted_vec[i])   # the honest share
    r = rng.sample_below(ek.n)
    c = paillier.encrypt_with_chosen_randomness(ek, x + 1, r)                      # here we encrypt x + 1
    st = pdl.PDLwSlackStatement(c, ek, msgs[k].points_committed_vec[i], ec.G, st0.g, st0.ni, st0.N)
    m2[k].points_encrypted_vec[i] = c
    m2[k].pdl_proof_vec[i] = pdl.prove(x, r, st, rng)
    ro, rg, _, _ = _both(m2, keys[0], dks[0], [], ctx=gpu_ctx)
    assert ro == ("PDLwSlackProof", {"is_u1_eq": True, "is_u2_eq": False, "is_u3_eq": True})
    assert rg == ro


def test_threshold_and_size(gpu_ctx, dkr5):
    keys, msgs, dks, _ = dkr5
    ro, rg, _, _ = _both(msgs[:2], keys[0], dks[0], [], ctx=gpu_ctx)
    assert ro == ("PartiesThresholdViolation", {"threshold": 2, "refreshed_keys": 2}) and rg == ro
    m2 = copy.deepcopy(msgs)
    m2[3].pdl_proof_vec.pop()
    ro, rg, _, _ = _both(m2, keys[0], dks[0], [], ctx=gpu_ctx)
    assert ro[0] == "SizeMismatchError" and rg == ro


def test_moduli_too_small(gpu_ctx, dkr5):
    keys, msgs, dks, rng = dkr5
    m2 = copy.deepcopy(msgs)
    ek, dk = paillier.keypair_with_modulus_size(KB - 128, rng)
    m2[3].ek = ek
    m2[3].dk_correctness_proof = protocol.NiCorrectKeyProof.proof(dk.p, dk.q)
    ro, rg, ko, kg = _both(m2, keys[2], dks[2], [], ctx=gpu_ctx)
    assert ro[0] == "ModuliTooSmall" and rg == ro
    assert [k.n for k in ko.paillier_key_vec] == [k.n for k in kg.paillier_key_vec]


def test_collect_with_joins(gpu_ctx):
    """replace + JoinMessage path (test.rs:95-224 shape, t=1, n=4: 3 refresh + 1 join)."""
    rng = Rng("joins")
    t, n = 1, 4
    all_keys = protocol.simulate_keygen(t, n, rng, KB)
    keys = [k.clone() for k in all_keys[:3]]
    jm, kk = protocol.join_distribute(rng, KB)
    jm.set_party_index(4)
    old_to_new = {1: 1, 2: 2, 3: 3}
    msgs, dks = [], []
    for key in keys:
        m, dk = protocol.replace([jm], key, old_to_new, 4, rng, KB)
        msgs.append(m)
        dks.append(dk)
    ro, rg, ko, kg = _both(msgs, keys[1], dks[1], [jm], ctx=gpu_ctx)
    assert ro is None and rg is None
    _same_key(ko, kg)
    # tampered DLog proof of the joiner
    j2 = copy.deepcopy(jm)
    j2.composite_dlog_proof_base_h2 = type(jm.composite_dlog_proof_base_h2)(jm.composite_dlog_proof_base_h2.x + 1,
                                                                            jm.composite_dlog_proof_base_h2.y)
    ro, rg, _, _ = _both(msgs, keys[1], dks[1], [j2], ctx=gpu_ctx)
    assert ro == ("DLogProofValidation", {"party_index": 4}) and rg == ro
    # unassigned joiner index
    j3 = copy.deepcopy(jm)
    j3.party_index = None
    ro, rg, _, _ = _both(msgs, keys[1], dks[1], [j3], ctx=gpu_ctx)
    assert rg == ro


def test_paillier_encrypt_job1(gpu_ctx):
    """Job 1: encrypt_with_chosen_randomness (refresh_message.rs:72-84) on the GPU."""
    rng = Rng("job1")
    keys = [paillier.keypair_with_modulus_size(2048, rng)[0] for _ in range(3)]
    ms = [rng.sample_below(ec.Q) for _ in range(24)]
    idx = [k % 3 for k in range(24)]
    rs = [rng.sample_below(keys[i].n) for i in idx]
    got = gpu_ctx.paillier_encrypt(ms, rs, [k.n for k in keys], idx, 64)
    want = [paillier.encrypt_with_chosen_randomness(keys[i], m, r) for m, r, i in zip(ms, rs, idx)]
    assert got == want


@pytest.mark.parametrize("bits", [2048, 3072])
def test_paillier_encrypt_ragged_keys(gpu_ctx, bits):
    """Job 1 with the shares of many keys in shuffled order and ragged counts per
    key (one key with a single share, one with 70, one unused): at 2048 bits the
    r^N chains are regrouped by key into sliding-window waves (pads rewrite their
    own row), at 3072 bits fixed windows; every ciphertext equals
    encrypt_with_chosen_randomness in the caller's order."""
    import random
    rng = Rng(f"job1-ragged-{bits}")
    keys = [paillier.keypair_with_modulus_size(bits, rng)[0] for _ in range(5)]
    idx = [0] * 1 + [1] * 70 + [2] * 9 + [4] * 33   # key 3 unused
    random.Random(bits).shuffle(idx)
    ms = [rng.sample_below(ec.Q) for _ in idx]
    rs = [rng.sample_below(keys[i].n) for i in idx]
    rs[5] = 1                                        # r = 1: c = 1 + mN
    got = gpu_ctx.paillier_encrypt(ms, rs, [k.n for k in keys], idx, bits // 32)
    want = [paillier.encrypt_with_chosen_randomness(keys[i], m, r) for m, r, i in zip(ms, rs, idx)]
    assert got == want


def test_prestart_hit_and_miss(gpu_ctx):
    """fsdkr_collect_prestart: a prepare of the batch it was started for reuses
    the s^N mod N^2 rows (every proof verifies); a prepare of a DIFFERENT batch
    (one PDL s2 changed after the prestart) recomputes them, so the changed pair
    fails u2 and nothing else does; a prestart while a batch is in flight is
    refused."""
    from fsdkr.batch import CollectBatch
    keys, msgs, dks, _ = _dkr(1, 3, "prestart")
    lk = keys[0]
    st = CollectBatch(msgs, lk, [], 256, KB, staged=True)
    assert st.ga_ready
    gpu_ctx.collect_prestart(st)
    st.complete()
    gpu_ctx.collect_prepare(st)
    v = gpu_ctx.collect_run(st)
    assert (v.pdl & 7 == 7).all() and (v.range & 1).all()
    # prestart for the original, prepare a tampered copy: must not reuse the rows
    gpu_ctx.collect_prestart(CollectBatch(msgs, lk, [], 256, KB, staged=True))
    bad = copy.deepcopy(msgs)
    p = bad[1].pdl_proof_vec[2]
    bad[1].pdl_proof_vec[2] = dataclasses.replace(p, s2=p.s2 + 1)
    b2 = CollectBatch(bad, lk, [], 256, KB)
    gpu_ctx.collect_prepare(b2)
    v2 = gpu_ctx.collect_run(b2)
    want = [7] * 9
    want[1 * 3 + 2] = 7 & ~2   # u2 of pair (message 1, receiver 2)
    assert [int(x) & 7 for x in v2.pdl] == want
    assert (v2.range & 1).all()
    # GA rows reusable, h1/h2 tables not: an s3 far wider than the prestart sized
    # the h2 tables for (u3 of that pair fails; everything else still verifies)
    gpu_ctx.collect_prestart(CollectBatch(msgs, lk, [], 256, KB, staged=True))
    wide = copy.deepcopy(msgs)
    p = wide[2].pdl_proof_vec[0]
    wide[2].pdl_proof_vec[0] = dataclasses.replace(p, s3=p.s3 << 40)
    b4 = CollectBatch(wide, lk, [], 256, KB)
    gpu_ctx.collect_prepare(b4)
    v4 = gpu_ctx.collect_run(b4)
    want = [7] * 9
    want[2 * 3 + 0] = 7 & ~4
    assert [int(x) & 7 for x in v4.pdl] == want
    assert (v4.range & 1).all()
    # in flight: refused
    b3 = CollectBatch(msgs, lk, [], 256, KB, staged=True)
    gpu_ctx.collect_prepare(CollectBatch(msgs, lk, [], 256, KB))
    gpu_ctx.collect_launch()
    with pytest.raises(RuntimeError):
        gpu_ctx.collect_prestart(b3)
    gpu_ctx.collect_finish(b3.complete())


def test_prestart_drops_a_plan_that_reads_it(gpu_ctx):
    """A prepared batch that consumed a prestart reads its s^N rows and fixed-base
    tables in place; a later prestart (of another batch) overwrites those buffers,
    so it drops that plan: running it again is refused instead of reading the other
    batch's rows."""
    from fsdkr.batch import CollectBatch
    keys, msgs, dks, _ = _dkr(1, 3, "prestart-drop")
    lk = keys[0]
    a = CollectBatch(msgs, lk, [], 256, KB, staged=True)
    gpu_ctx.collect_prestart(a)
    a.complete()
    gpu_ctx.collect_prepare(a)
    v = gpu_ctx.collect_run(a)
    assert (v.pdl & 7 == 7).all()
    bad = copy.deepcopy(msgs)
    p = bad[0].pdl_proof_vec[1]
    bad[0].pdl_proof_vec[1] = dataclasses.replace(p, s2=p.s2 + 1)
    gpu_ctx.collect_prestart(CollectBatch(bad, lk, [], 256, KB, staged=True))
    with pytest.raises(RuntimeError):
        gpu_ctx.collect_run(a)
    # the prestart itself is intact: a prepare of its batch consumes it
    b = CollectBatch(bad, lk, [], 256, KB)
    gpu_ctx.collect_prepare(b)
    v2 = gpu_ctx.collect_run(b)
    want = [7] * 9
    want[1] = 7 & ~2
    assert [int(x) & 7 for x in v2.pdl] == want


def test_collect_recover_entry(gpu_ctx, dkr5):
    """fsdkr_collect_recover (share recovery in one C-ABI call, refresh_message.rs:367-373,
    439-464) against the oracle's collect() for every party of a t=2 n=5 refresh, in one
    call with a degenerate-key job (p == q: Paillier::decrypt panics) and a job whose
    local_key.t exceeds the VSS threshold (li_vec index panic) beside them."""
    from fsdkr.refresh import _dk_limbs
    keys, msgs, dks, _ = dkr5
    jobs, want = [], []
    for party in range(5):
        lk = keys[party]
        t = lk.vss_scheme.threshold
        jobs.append(dict(nl=_dk_limbs(lk.paillier_dk), t_vss=t, t_key=lk.t,
                         old_index=[m.old_party_index for m in msgs[:t + 1]],
                         cts=[m.points_encrypted_vec[lk.i - 1] for m in msgs[:t + 1]],
                         p=lk.paillier_dk.p, q=lk.paillier_dk.q,
                         points=[[m.points_committed_vec[i] for m in msgs[:t + 1]] for i in range(5)]))
        ko = lk.clone()
        protocol.collect(copy.deepcopy(msgs), ko, dks[party], [], Rng("a8"), KB)
        want.append((0, ko.x_i, ko.y, ko.pk_vec[:5]))
    bad = dict(jobs[1], q=jobs[1]["p"])
    over = dict(jobs[2], t_key=jobs[2]["t_vss"] + 1)
    got = gpu_ctx.collect_recover(jobs + [bad, over])
    assert got[:5] == want
    assert got[5][0] == 2                       # FSDKR_RECOVER_PANIC_DECRYPT
    assert got[6][0] == 1 and got[6][1:3] == want[2][1:3]   # FSDKR_RECOVER_PANIC_LI, share still recovered


def test_collect_recover_launch_finish(gpu_ctx, dkr5):
    """fsdkr_collect_recover_launch / _finish: the same results as the one-call
    form while a collect batch runs beside it, inputs copied at launch (the
    caller's arrays may go away), one recovery in flight per context, and a
    finish without a launch refused."""
    from fsdkr._native import FsdkrError
    from fsdkr.batch import CollectBatch
    from fsdkr.refresh import _dk_limbs
    keys, msgs, dks, _ = dkr5
    jobs = []
    for party in range(5):
        lk = keys[party]
        t = lk.vss_scheme.threshold
        jobs.append(dict(nl=_dk_limbs(lk.paillier_dk), t_vss=t, t_key=lk.t,
                         old_index=[m.old_party_index for m in msgs[:t + 1]],
                         cts=[m.points_encrypted_vec[lk.i - 1] for m in msgs[:t + 1]],
                         p=lk.paillier_dk.p, q=lk.paillier_dk.q,
                         points=[[m.points_committed_vec[i] for m in msgs[:t + 1]] for i in range(5)]))
    want = gpu_ctx.collect_recover(jobs)
    b = CollectBatch(msgs, keys[0], [], 256, KB)
    gpu_ctx.collect_prepare(b)
    gpu_ctx.collect_launch()
    h = gpu_ctx.collect_recover_launch(jobs)
    with pytest.raises(FsdkrError):
        gpu_ctx.collect_recover_launch(jobs)     # one in flight
    v = gpu_ctx.collect_finish(b)
    assert gpu_ctx.collect_recover_finish(h) == want
    assert (v.pdl & 7 == 7).all()
    with pytest.raises(FsdkrError):
        gpu_ctx.collect_recover_finish(h)        # nothing launched any more
    assert gpu_ctx.collect_recover(jobs) == want  # the context is usable again


def _vt(v):
    return tuple(bytes(getattr(v, f)) for f in ("feldman", "pdl", "range", "ped", "ck", "dlog"))


