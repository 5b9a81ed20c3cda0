"""Multi-GPU sharding logic (fsdkr.shard) on CPU: world_size 2 (and 3) gloo
processes each hold the verdicts of their message slice; one all_reduce(MAX)
must rebuild exactly the single-process verdicts."""
import os
import socket
import sys
import types

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _truth(R, J, n, seed=3):
    rnd = np.random.default_rng(seed)
    P = R * n
    return types.SimpleNamespace(feldman=rnd.integers(0, 2, P, dtype=np.uint8),
                                 pdl=rnd.integers(0, 16, P, dtype=np.uint8),
                                 range=rnd.integers(0, 2, P, dtype=np.uint8),
                                 ped=rnd.integers(0, 4, R + J, dtype=np.uint8),
                                 ck=rnd.integers(0, 2, R + J, dtype=np.uint8),
                                 dlog=rnd.integers(0, 4, J, dtype=np.uint8))


def _local(truth, R, J, n, world, rank):
    from fsdkr.shard import shard_range
    r0, r1 = shard_range(R, world, rank)
    j0, j1 = shard_range(J, world, rank)
    return types.SimpleNamespace(
        feldman=truth.feldman[r0 * n:r1 * n], pdl=truth.pdl[r0 * n:r1 * n], range=truth.range[r0 * n:r1 * n],
        ped=np.concatenate([truth.ped[r0:r1], truth.ped[R + j0:R + j1]]),
        ck=np.concatenate([truth.ck[r0:r1], truth.ck[R + j0:R + j1]]), dlog=truth.dlog[j0:j1])


def _worker(rank, world, port, R, J, n, q):
    sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
    import torch.distributed as dist
    from fsdkr import shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    truth = _truth(R, J, n)
    vec = shard.merge(dist, shard.scatter(_local(truth, R, J, n, world, rank), R, J, n, world, rank))
    m = shard.MergedVerdicts(vec, R, J, n)
    ok = all(np.array_equal(getattr(m, f), getattr(truth, f)) for f in ("feldman", "pdl", "range", "ped", "ck", "dlog"))
    dist.destroy_process_group()
    q.put((rank, ok))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,R,J,n", [(2, 60, 4, 64), (3, 7, 2, 9)])
def test_sharded_verdicts_merge(world, R, J, n):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, R, J, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert sorted(res) == [(r, True) for r in range(world)]


def test_shard_ranges_cover():
    from fsdkr.shard import shard_range
    for count in (0, 1, 5, 60, 61):
        for world in (1, 2, 3, 8):
            got = [shard_range(count, world, r) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == count
            assert all(got[k][1] == got[k + 1][0] for k in range(world - 1))
