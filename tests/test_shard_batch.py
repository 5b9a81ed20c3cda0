"""Multi-GPU shards of one collect(): each rank packs a slice of
the refresh / join messages against the full receiver set.  A slice may hold
<= t messages (n = 64, t = 32 over 2+ GPUs): the threshold check belongs to the
whole message set, so a shard batch must still be packed for the GPU.

CPU part: packing of every slice.  GPU part: the verdicts of all slices,
scattered and max-merged exactly as shard.merge's all-reduce does, equal the
single-batch verdicts (valid and tampered inputs)."""
import copy
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
