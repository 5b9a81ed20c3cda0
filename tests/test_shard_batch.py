"""Multi-GPU shards of one collect(): each rank packs a slice of
the refresh / join messages against the full receiver set.  A slice may hold
<= t messages (n = 64, t = 32 over 2+ GPUs): the threshold check belongs to the
whole message set, so a shard batch must still be packed for the GPU.

CPU part: packing of every slice.  GPU part: the verdicts of all slices,
scattered and max-merged exactly as shard.merge's all-reduce does, equal the
single-batch verdicts (valid and tampered inputs)."""
import copy
import dataclasses
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import codec  # noqa: E402


def _fixture(name="transcript_t2_n5_kb1024.json.gz"):
    raw = codec.load_raw(name)
    cls = codec.product_classes()
    return raw, cls, {k: codec.dec(raw[k], cls) for k in ("keys", "dks", "msgs", "joins")}


@pytest.mark.parametrize("name,world", [("transcript_t2_n5_kb1024.json.gz", 2),
                                        ("transcript_t2_n5_kb1024.json.gz", 3),
                                        ("transcript_t2_n5_kb1024.json.gz", 5),
                                        ("transcript_join_t1_n4_kb1024.json.gz", 2)])
def test_shard_slices_pack(name, world):
    from fsdkr.batch import CollectBatch
    from fsdkr.shard import shard_range
    raw, cls, d = _fixture(name)
    msgs, joins, key = d["msgs"], d["joins"], d["keys"][0]
    R, J = len(msgs), len(joins)
    n = R + J
    for rank in range(world):
        r0, r1 = shard_range(R, world, rank)
        j0, j1 = shard_range(J, world, rank)
        b = CollectBatch(msgs[r0:r1], key, joins[j0:j1], 256, raw["meta"]["key_bits"], n_recv=n)
        if r1 > r0:
            assert not b.header_only, (world, rank)
            assert (b.R, b.J, b.n, b.nl) == (r1 - r0, j1 - j0, n, 64)


def _sharded_verdicts(ctx, msgs, key, joins, world, kb):
    from fsdkr.batch import CollectBatch
    from fsdkr import shard
    R, J = len(msgs), len(joins)
    n = R + J
    acc = np.zeros(shard.global_len(R, J, n), np.uint8)
    for rank in range(world):
        r0, r1 = shard.shard_range(R, world, rank)
        j0, j1 = shard.shard_range(J, world, rank)
        b = CollectBatch(msgs[r0:r1], key, joins[j0:j1], 256, kb, n_recv=n)
        v = ctx.verify_collect(b)
        acc = np.maximum(acc, shard.scatter(v, R, J, n, world, rank))   # = all_reduce(MAX)
    return shard.MergedVerdicts(acc, R, J, n)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_verdicts_equal_single_batch(gpu_ctx, world):
    import dataclasses
    from fsdkr.batch import CollectBatch
    raw, cls, d = _fixture()
    kb = raw["meta"]["key_bits"]
    key = d["keys"][0]
    msgs = copy.deepcopy(d["msgs"])
    p = msgs[3].pdl_proof_vec[1]
    msgs[3].pdl_proof_vec[1] = dataclasses.replace(p, u2=p.u2 + 1)          # one bad PDL proof
    a = msgs[1].range_proofs[4]
    msgs[1].range_proofs[4] = dataclasses.replace(a, s2=a.s2 + 1)           # one bad range proof
    for m_in in (d["msgs"], msgs):
        whole = gpu_ctx.verify_collect(CollectBatch(m_in, key, [], 256, kb))
        merged = _sharded_verdicts(gpu_ctx, m_in, key, [], world, kb)
        for f in ("feldman", "pdl", "range", "ped", "ck"):
            assert np.array_equal(getattr(whole, f), getattr(merged, f)), f
    assert merged.pdl[3 * 5 + 1] != 7 and merged.range[1 * 5 + 4] == 0


class _Shared:
    def __init__(self, world):
        import threading
        self.world = world
        self.bar = threading.Barrier(world)
        self.buf = [None] * world


class _RankDist:
    """torch.distributed stand-in for ranks emulated as threads of one process
    (each with its own HIP context on the one GPU): all_reduce(MAX) over a barrier."""

    class ReduceOp:
        MAX = "max"

    def __init__(self, shared, rank):
        self.s, self.rank = shared, rank

    def get_rank(self):
        return self.rank

    def get_world_size(self):
        return self.s.world

    def all_reduce(self, t, op):
        import torch
        assert op == "max"
        self.s.buf[self.rank] = t.clone()
        self.s.bar.wait()
        m = self.s.buf[0]
        for x in self.s.buf[1:]:
            m = torch.maximum(m, x)
        t.copy_(m)
        self.s.bar.wait()


@pytest.mark.gpu
@pytest.mark.parametrize("tamper", [None, "pdl", "ck", "neg_s1", "neg_alice_e"])
def test_sharded_collect_two_emulated_ranks(gpu_ctx, tamper):
    """fsdkr.shard.collect with two ranks emulated as threads (one HIP context
    each, one GPU): every rank's outcome and LocalKey equal the single-process
    GPU collect() and the oracle's (negative operands: the panic of that
    sender's pair, found by the rank that holds it and merged to every rank)."""
    import threading
    from fsdkr import Context, refresh, shard
    from oracle import protocol
    from oracle.rng import Rng
    raw, cls, d = _fixture()
    kb = raw["meta"]["key_bits"]
    msgs, key, dk = copy.deepcopy(d["msgs"]), d["keys"][0], d["dks"][0]
    if tamper == "pdl":
        p = msgs[3].pdl_proof_vec[1]
        msgs[3].pdl_proof_vec[1] = dataclasses.replace(p, s3=p.s3 + 1)
    elif tamper == "neg_s1":
        p = msgs[3].pdl_proof_vec[1]
        msgs[3].pdl_proof_vec[1] = dataclasses.replace(p, s1=-p.s1)
    elif tamper == "neg_alice_e":
        a = msgs[4].range_proofs[0]
        msgs[4].range_proofs[0] = dataclasses.replace(a, e=-a.e)
    elif tamper == "ck":
        sv = msgs[4].dk_correctness_proof.sigma_vec
        msgs[4].dk_correctness_proof = dataclasses.replace(msgs[4].dk_correctness_proof,
                                                           sigma_vec=(sv[0] + 1,) + tuple(sv[1:]))

    def outcome(fn):
        try:
            fn()
            return None
        except Exception as e:
            return (getattr(e, "variant", "panic"), getattr(e, "fields", {}))

    def summary(k):
        return (k.x_i, k.y, list(k.pk_vec), [e.n for e in k.paillier_key_vec])
    single = copy.deepcopy(key)
    want = outcome(lambda: refresh.collect(copy.deepcopy(msgs), single, dk, [], ctx=gpu_ctx, key_bits=kb))
    ocls = codec.oracle_classes()
    od = {k: codec.dec(raw[k], ocls) for k in ("keys", "dks")}
    sys.path.insert(0, HERE)
    import tamper as tp
    ko = od["keys"][0].clone()
    ow = outcome(lambda: protocol.collect(tp.to_oracle(copy.deepcopy(msgs)), ko, od["dks"][0], [], Rng("a8"), kb))
    assert want == ow
    shared = _Shared(2)
    res = {}

    def rank_main(r):
        ctx = Context()
        k = copy.deepcopy(key)
        res[r] = (outcome(lambda: shard.collect(_RankDist(shared, r), msgs, k, dk, [], ctx, key_bits=kb)), summary(k))
        ctx.close()
    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    for r in range(2):
        assert res[r][0] == want, (r, res[r][0], want)
        assert res[r][1] == summary(single)


@pytest.mark.gpu
def test_cu_split_keeps_verdicts(gpu_ctx):
    """fsdkr_ctx_set_cu_split (GA chains on their own CUs, used by shard slices)
    is a performance setting: the same batch gives the same verdicts with and
    without it; bad CU counts are rejected."""
    from fsdkr._native import FsdkrError
    from fsdkr.batch import CollectBatch
    raw, cls, d = _fixture()
    kb = raw["meta"]["key_bits"]
    msgs = copy.deepcopy(d["msgs"])
    p = msgs[2].pdl_proof_vec[0]
    msgs[2].pdl_proof_vec[0] = dataclasses.replace(p, u3=p.u3 + 1)
    b = CollectBatch(msgs, d["keys"][0], [], 256, kb)
    base = gpu_ctx.verify_collect(b)
    try:
        for cus in (160, 64, 0):
            gpu_ctx.set_cu_split(cus)
            v = gpu_ctx.verify_collect(b)
            for f in ("feldman", "pdl", "range", "ped", "ck"):
                assert np.array_equal(getattr(base, f), getattr(v, f)), (cus, f)
        for bad in (12, 232):
            with pytest.raises(FsdkrError):
                gpu_ctx.set_cu_split(bad)
    finally:
        gpu_ctx.set_cu_split(0)
