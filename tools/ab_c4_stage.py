#!/usr/bin/env python3
"""Interleaved A/B of configs[4]'s staging on one box (same sessions, one process):
v0 = the default split stage 1 (GA's fields, prestart, then the table bases and
a second prestart), v1 = one stage 1 with GA's fields and the table bases, so the
T / h1 / h2 table chains are enqueued with GA in one prestart call.  Prints one
JSON line per step.  Diagnostics for DESIGN.md."""
import argparse
import copy
import functools
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
os.environ["GPU_MAX_HW_QUEUES"] = str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    from fsdkr import Context, refresh, synth
    from fsdkr import batch as B
    ctx = Context()
    sess = synth.synth_sessions(ctx, a.sessions, n=3, t=1, seed=2028, key_bits=3072)
    orig = B.SessionSet.__init__

    def run(split):
        B.SessionSet.__init__ = functools.partialmethod(orig, split_stage1=split)
        try:
            work = [(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in sess]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = refresh.collect_many(work, ctx=ctx, key_bits=3072)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
        finally:
            B.SessionSet.__init__ = orig
        assert all(r is None for r in res)
        return ms, ctx.collect_last_span_ms()
    run(True)
    run(False)
    for r in range(a.rounds):
        for v, split in ((0, True), (1, False)):
            ms, span = run(split)
            print(json.dumps({"round": r, "variant": v, "split_stage1": split, "ms": ms, "span_ms": span}), flush=True)


if __name__ == "__main__":
    main()
