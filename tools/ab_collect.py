#!/usr/bin/env python3
"""Interleaved A/B of collect() tuning knobs (environment variables read per
collect_run call, csrc/collect.cpp) over ONE generated n = 64 workload: box-to-box
noise (+-15 % between gpurun boxes) swamps single bench runs, so every config is
timed in each of --rounds rounds, configs alternating, and the median is kept.
Usage: python tools/ab_collect.py "-" "FSDKR_GA_FIRST=3" "FSDKR_GA_FIRST=3+FSDKR_PRIO=2,3,2,1" ..."""
import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
# FSDKR_HWQ=<q> sets the hardware queue count exactly (A/B across processes)
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("FSDKR_HWQ") or \
    str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--t", type=int, default=32)
    ap.add_argument("--joins", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--shard", type=int, default=1, help="time rank 0's slice of a W-way shard")
    ap.add_argument("--timing", action="store_true", help="context with per-kernel HIP-event timing")
    a = ap.parse_args()
    import torch
    from fsdkr import Context, synth, shard
    from fsdkr.batch import CollectBatch
    ctx = Context(timing=a.timing)
    R, J = a.n - a.joins, a.joins
    msgs, joins, lk = synth.synth_collect(ctx, R, J, a.t, 2024)
    r0, r1 = shard.shard_range(R, a.shard, 0)
    j0, j1 = shard.shard_range(J, a.shard, 0)
    batch = CollectBatch(msgs[r0:r1], lk, joins[j0:j1], 256, 2048, n_recv=a.n)
    ctx.collect_prepare(batch)
    P = (r1 - r0) * a.n
    knobs = sorted({kv.split("=", 1)[0] for c in a.configs if c != "-" for kv in c.split("+")})

    def apply(cfg):
        for k in knobs:
            os.environ.pop(k, None)
        if cfg != "-":
            for kv in cfg.split("+"):
                k, v = kv.split("=", 1)
                os.environ[k] = v

    times = {c: [] for c in a.configs}
    for cfg in a.configs:   # warm-up + correctness gate per config
        apply(cfg)
        v = ctx.collect_run(batch)
        assert v.feldman[:P].all() and (v.pdl[:P] == 7).all() and v.range[:P].all(), cfg
    for r in range(a.rounds):
        for cfg in a.configs:
            apply(cfg)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                ctx.collect_run(batch)
            torch.cuda.synchronize()
            times[cfg].append((time.perf_counter() - t0) / a.steps * 1e3)
        print(f"round {r}: " + "  ".join(f"{c}={times[c][-1]:.1f}" for c in a.configs), flush=True)
    for c in a.configs:
        print(json.dumps({"config": c, "shard": a.shard, "timing": a.timing, "median_ms": statistics.median(times[c]),
                          "min_ms": min(times[c]), "ms": times[c]}), flush=True)


if __name__ == "__main__":
    main()
