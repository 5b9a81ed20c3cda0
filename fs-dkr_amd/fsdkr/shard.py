"""Multi-GPU sharding of one collect() verification.

Rank r of W verifies a contiguous slice of the refresh messages and of the
join messages' proofs against the FULL receiver set (fsdkr_collect_batch
n_recv = n); the verdicts of all ranks are merged with ONE all-reduce(MAX) of a
zero-filled byte vector laid out as

    [feldman R*n | pdl R*n | range R*n | ped R+J | ck R+J | dlog J]

No other data crosses the interconnect."""
import numpy as np


def shard_range(count, world, rank):
    """Contiguous [lo, hi) slice of `count` units for `rank` of `world`."""
    return rank * count // world, (rank + 1) * count // world


def global_len(R, J, n):
    return 3 * R * n + 2 * (R + J) + J


def scatter(v, R, J, n, world, rank):
    """Place this rank's Verdicts (of its slice) into a zero-filled global vector."""
    r0, r1 = shard_range(R, world, rank)
    j0, j1 = shard_range(J, world, rank)
    P = R * n
    out = np.zeros(global_len(R, J, n), np.uint8)
    lo, cnt = r0 * n, (r1 - r0) * n
    out[lo:lo + cnt] = v.feldman[:cnt]
    out[P + lo:P + lo + cnt] = v.pdl[:cnt]
    out[2 * P + lo:2 * P + lo + cnt] = v.range[:cnt]
    base_ped, base_ck, base_dl = 3 * P, 3 * P + (R + J), 3 * P + 2 * (R + J)
    nr = r1 - r0
    for q in range(nr):
        out[base_ped + r0 + q] = v.ped[q]
        out[base_ck + r0 + q] = v.ck[q]
    for q in range(j1 - j0):
        out[base_ped + R + j0 + q] = v.ped[nr + q]
        out[base_ck + R + j0 + q] = v.ck[nr + q]
        out[base_dl + j0 + q] = v.dlog[q]
    return out


class MergedVerdicts:
    """Global verdicts rebuilt from the all-reduced vector (same fields as batch.Verdicts)."""

    def __init__(self, vec, R, J, n):
        P = R * n
        self.feldman = vec[:P]
        self.pdl = vec[P:2 * P]
        self.range = vec[2 * P:3 * P]
        self.ped = vec[3 * P:3 * P + R + J]
        self.ck = vec[3 * P + R + J:3 * P + 2 * (R + J)]
        self.dlog = vec[3 * P + 2 * (R + J):3 * P + 2 * (R + J) + J]


def merge(dist, local_vec, device=None):
    """all_reduce(MAX) of the scattered verdict vector over the default group
    (RCCL on GPU tensors, gloo on CPU tensors); returns a numpy uint8 vector."""
    import torch
    t = torch.from_numpy(local_vec)
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu().numpy()
