"""Multi-GPU sharding of one collect().

Rank r of W verifies a contiguous slice of the refresh messages and of the
join messages' proofs against the FULL receiver set (fsdkr_collect_batch
n_recv = n); the verdicts of all ranks are merged with ONE all-reduce(MAX) of a
zero-filled byte vector laid out as

    [feldman R*n | pdl R*n | range R*n | ped R+J | ck R+J | dlog J]

The share recovery (refresh_message.rs:439-464) is split the same way: rank r
rebuilds the pk_vec rows of its slice of the new parties (one MSM row per
party) and rank 0 alone decrypts the new share; their results ride in the same
all-reduce, in a region appended to the verdict bytes (each rank writes only
its own part, the others are zero, so MAX is the union):

    [status 1 | share 32 | y 64 | pk_vec n*64]      (little-endian limbs)

No other data crosses the interconnect.  collect() then maps the merged
verdicts to the reference's first error on a header-only batch of the whole
message set (threshold, sizes, party indices, ek.n) and applies collect()'s
side effects and the merged share recovery on every rank."""
import os
import time

import numpy as np

from .batch import CollectBatch, Verdicts


# GA split of a small slice (measured: profiles/r02zd_ga_lanes_cus_ab.jsonl, r02zn_ga_split_size_ab.jsonl)
GA_SPLIT_CUS = 160
GA_SPLIT_MAX_CHAINS = 1024


def shard_range(count, world, rank):
    """Contiguous [lo, hi) slice of `count` units for `rank` of `world`."""
    return rank * count // world, (rank + 1) * count // world


def global_len(R, J, n):
    return 3 * R * n + 2 * (R + J) + J


DEC_RANK = 0   # the rank that decrypts the new share


def recovery_len(n):
    return 1 + 32 + 64 + 64 * n


def _pt_bytes(pt):
    return bytes(64) if pt is None else pt[0].to_bytes(32, "little") + pt[1].to_bytes(32, "little")


def _bytes_pt(b):
    v = int.from_bytes(bytes(b), "little")
    return None if v == 0 else (v & ((1 << 256) - 1), v >> 256)


def encode_recovery(spec, n, rows, decrypt):
    """This rank's part of the share recovery as bytes of the exchange region:
    its pk_vec rows, and (the decrypting rank) status, share and y.  Status: 1 ok,
    2 ok but li_vec out of bounds, 3 Paillier::decrypt panic, 4 another panic of
    the decrypting rank (the plan's and the key checks run on every rank from the
    same inputs, refresh._speculative_launch, so every rank normally raises it
    itself; 4 makes the ranks agree whatever happens), 0 never written."""
    from .refresh import _DecryptPanic
    out = np.zeros(recovery_len(n), np.uint8)
    if spec is None or isinstance(spec, Exception):
        if decrypt and isinstance(spec, _DecryptPanic):   # Paillier::decrypt on a degenerate key
            out[0] = 3
        elif decrypt:   # any other panic (or no result) of the decrypting rank: every rank raises
            out[0] = 4
        return out
    share, y, pk, t_ok = spec
    lo, hi = rows
    if decrypt:
        out[0] = 1 if t_ok else 2
        out[1:33] = np.frombuffer(int(share).to_bytes(32, "little"), np.uint8)
        out[33:97] = np.frombuffer(_pt_bytes(y), np.uint8)
    for i, pt in zip(range(lo, hi), pk):
        out[97 + 64 * i:97 + 64 * (i + 1)] = np.frombuffer(_pt_bytes(pt), np.uint8)
    return out


def decode_recovery(region, local_spec, n):
    """The merged recovery (the tuple refresh._conclude takes, or the panic).
    A status other than 1 / 2 / 3 from the decrypting rank is a panic on every
    rank: a share 0 applied by some ranks while the decrypting rank panics would
    leave the ranks' LocalKeys diverged."""
    from .refresh import _DecryptPanic
    if isinstance(local_spec, Exception) and not isinstance(local_spec, _DecryptPanic):
        return local_spec
    st = int(region[0])
    if st == 3:
        return _DecryptPanic("share recovery: Paillier::decrypt (degenerate decryption key)")
    if st not in (1, 2):   # 0: the decrypting rank wrote nothing; 4: it hit a panic this rank did not
        from .refresh import FsDkrPanic
        return FsDkrPanic(f"share recovery: no result from the decrypting rank (status {st})")
    share = int.from_bytes(bytes(region[1:33]), "little")
    y = _bytes_pt(region[33:97])
    pk = [_bytes_pt(region[97 + 64 * i:97 + 64 * (i + 1)]) for i in range(n)]
    return (share, y, pk, st != 2)


def scatter(v, R, J, n, world, rank):
    """Place this rank's Verdicts (of its slice) into a zero-filled global vector."""
    r0, r1 = shard_range(R, world, rank)
    j0, j1 = shard_range(J, world, rank)
    P = R * n
    out = np.zeros(global_len(R, J, n), np.uint8)
    if v is None:
        return out
    lo, cnt = r0 * n, (r1 - r0) * n
    out[lo:lo + cnt] = v.feldman[:cnt]
    out[P + lo:P + lo + cnt] = v.pdl[:cnt]
    out[2 * P + lo:2 * P + lo + cnt] = v.range[:cnt]
    base_ped, base_ck, base_dl = 3 * P, 3 * P + (R + J), 3 * P + 2 * (R + J)
    nr = r1 - r0
    out[base_ped + r0:base_ped + r1] = v.ped[:nr]
    out[base_ck + r0:base_ck + r1] = v.ck[:nr]
    nj = j1 - j0
    out[base_ped + R + j0:base_ped + R + j1] = v.ped[nr:nr + nj]
    out[base_ck + R + j0:base_ck + R + j1] = v.ck[nr:nr + nj]
    out[base_dl + j0:base_dl + j1] = v.dlog[:nj]
    return out


class MergedVerdicts(Verdicts):
    """Global verdicts rebuilt from the all-reduced vector (same fields and C view as batch.Verdicts)."""

    def __init__(self, vec, R, J, n):
        P = R * n
        vec = np.ascontiguousarray(vec, dtype=np.uint8)
        self.feldman = vec[:P]
        self.pdl = vec[P:2 * P]
        self.range = vec[2 * P:3 * P]
        self.ped = vec[3 * P:3 * P + R + J]
        self.ck = vec[3 * P + R + J:3 * P + 2 * (R + J)]
        self.dlog = vec[3 * P + 2 * (R + J):3 * P + 2 * (R + J) + J] if J else np.zeros(1, np.uint8)
        self._vec = vec
        self._bind(P, R + J, J)


def merge(dist, local_vec, device=None):
    """all_reduce(MAX) of the scattered verdict vector over the default group
    (RCCL on GPU tensors, gloo on CPU tensors); returns a numpy uint8 vector."""
    import torch
    t = torch.from_numpy(local_vec)
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu().numpy()


class _Clock:
    """phase durations (ms) of one rank's call into `out` (None: no timing)"""

    def __init__(self, out):
        self.out = out
        self.t = time.perf_counter()

    def __call__(self, name):
        if self.out is not None:
            now = time.perf_counter()
            self.out[name] = self.out.get(name, 0.0) + (now - self.t) * 1e3
            self.t = now


def verify_slice(ctx, msgs, lk, joins, world, rank, m_security=256, key_bits=2048, launch_only=False, clock=None):
    """This rank's slice as a CollectBatch (n_recv = n); launched on the GPU.
    Returns (batch or None, verdicts or None); with launch_only the caller
    finishes it (ctx.collect_finish) after overlapping host work."""
    clock = clock or _Clock(None)
    R, J = len(msgs), len(joins)
    n = R + J
    r0, r1 = shard_range(R, world, rank)
    j0, j1 = shard_range(J, world, rank)
    if r1 == r0 and j1 == j0:
        return None, None
    # a slice whose s^N mod N^2 chains (2 per pair) leave most of the chip idle is
    # latency-bound on them: they get 160 CUs of their own, every other stream the
    # remaining 96 (8-way shard of n=64: 29.4 -> 22.5 ms per rank; no gain at 2-
    # and 4-way shards, profiles/r02zd_ga_lanes_cus_ab.jsonl)
    if hasattr(ctx, "set_cu_split"):
        ctx.set_cu_split(GA_SPLIT_CUS if 2 * (r1 - r0) * n <= GA_SPLIT_MAX_CHAINS else 0)
    b = CollectBatch(msgs[r0:r1], lk, joins[j0:j1], m_security, key_bits, n_recv=n, staged=True)
    clock("slice_stage1_ms")
    if b.header_only:   # an empty refresh slice (joins only) or a size failure the header batch reports
        return None, None
    from .refresh import prestart
    prestart(ctx, b)   # the long chains start while stage 2 packs
    clock("prestart_ms")
    b.complete()
    clock("slice_stage2_ms")
    ctx.collect_prepare(b)
    clock("prepare_ms")
    ctx.collect_launch()
    clock("launch_ms")
    if launch_only:
        return b, None
    return b, ctx.collect_finish(b)


def collect(dist, refresh_messages, local_key, new_dk, join_messages, ctx, device=None, m_security=256,
            key_bits=2048, recovery="speculative", timings=None):
    """RefreshMessage::collect (refresh_message.rs:321-467) sharded over the ranks of
    `dist` (torch.distributed, initialised): every rank holds every message (the
    broadcast channel of README.md:19) and the same LocalKey; each verifies its
    slice, the verdict bytes are all-reduced once, and every rank returns the
    reference's outcome: None after updating `local_key` as collect() does, or
    raises the FsDkrError / FsDkrPanic collect() raises (with its partial
    paillier_key_vec updates).  `recovery` as in refresh.collect.  `timings`
    (a dict) receives this rank's host phases in ms (bench.py --emulate-shard)."""
    from .refresh import _check_mode, _conclude, _finish_both, _mapped, _recover_after, _speculative_launch
    clock = _Clock(timings)
    _check_mode(recovery)
    world, rank = dist.get_world_size(), dist.get_rank()
    msgs, joins = list(refresh_messages), list(join_messages)
    R, J = len(msgs), len(joins)
    n = R + J
    header = CollectBatch(msgs, local_key, joins, m_security, key_bits, header_only=True)
    clock("header_ms")
    job = (msgs, local_key, n)
    spec = None
    if header.size_fail:
        merged = None
    else:
        b, _ = verify_slice(ctx, msgs, local_key, joins, world, rank, m_security, key_bits, launch_only=True,
                            clock=clock)
        rows, decrypt = shard_range(n, world, rank), rank == DEC_RANK
        pend = None
        try:   # this rank's part of the share recovery overlaps its pipeline on the recovery stream
            if recovery == "speculative":
                pend = _speculative_launch(ctx, [job + (rows, decrypt)])
            clock("recovery_launch_ms")
        finally:   # neither the slice nor the recovery stays in flight
            v, specs = _finish_both(ctx, (lambda: ctx.collect_finish(b)) if b is not None else (lambda: None), pend)
        clock("finish_wait_ms")
        vec = scatter(v, R, J, n, world, rank)
        if recovery == "speculative":
            vec = np.concatenate([vec, encode_recovery(specs[0], n, rows, decrypt)])
        mvec = merge(dist, vec, device)
        clock("merge_ms")
        G = global_len(R, J, n)
        merged = MergedVerdicts(mvec[:G], R, J, n)
        if recovery == "speculative":
            spec = decode_recovery(mvec[G:], specs[0], n)
    err, applied = _mapped(ctx, header, msgs, merged)
    if recovery == "after" or header.size_fail:
        spec = _recover_after(ctx, [job], [err])[0]
    err = _conclude(local_key, new_dk, msgs, joins, err, applied, spec)
    clock("conclude_ms")
    if err is not None:
        raise err
