#!/usr/bin/env python3
"""Interleaved A/B of tuning knobs over WHOLE refresh.collect() calls (bench.py's
step: staged pack, prestart, prepare, pipeline, recovery, first error), one
generated n = 64 workload, configs alternating step by step, median per config.
Knobs are environment variables the library reads per call (FSDKR_PRE_GA_PRIO,
FSDKR_FB_SPLIT, FSDKR_PRE_FB, FSDKR_GC_STREAM, ...).
Usage: python tools/ab_full.py "-" "FSDKR_FB_SPLIT=0" "FSDKR_PRE_GA_PRIO=3+FSDKR_FB_SPLIT=0" ..."""
import argparse
import copy
import gc
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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--gc-freeze", action="store_true", help="gc.freeze() after the workload is built")
    a = ap.parse_args()
    import torch  # noqa: F401
    from fsdkr import Context, refresh, synth
    ctx = Context()
    msgs, joins, lk = synth.synth_collect(ctx, 60, 4, 32, 2024)
    knobs = sorted({kv.split("=", 1)[0] for c in a.configs if c != "-" for kv in c.split("+")})
    keys = [copy.deepcopy(lk) for _ in range((a.rounds + 1) * len(a.configs))]
    if a.gc_freeze:
        gc.collect()
        gc.freeze()

    def apply(cfg):
        for k in knobs:
            os.environ.pop(k, None)
        if cfg != "-":
            for kv in cfg.split("+"):
                k, v = kv.split("=", 1)
                os.environ[k] = v
    ki = 0
    for cfg in a.configs:   # warm every path once
        apply(cfg)
        refresh.collect(msgs, keys[ki], lk.paillier_dk, joins, ctx=ctx)
        ki += 1
    res = {c: [] for c in a.configs}
    for r in range(a.rounds):
        for cfg in a.configs:
            apply(cfg)
            time.sleep(0.01)
            t0 = time.perf_counter()
            refresh.collect(msgs, keys[ki], lk.paillier_dk, joins, ctx=ctx)
            res[cfg].append((time.perf_counter() - t0) * 1e3)
            ki += 1
    for cfg in a.configs:
        v = res[cfg]
        print(json.dumps({"config": cfg, "gc_freeze": a.gc_freeze, "median_ms": statistics.median(v),
                          "min_ms": min(v), "ms": [round(x, 1) for x in v]}), flush=True)


if __name__ == "__main__":
    main()
