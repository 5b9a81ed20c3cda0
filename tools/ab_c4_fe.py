#!/usr/bin/env python3
"""Interleaved A/B of configs[4]'s per-session error mapping on one box (same
sessions, one process): v0 = one fsdkr_collect_first_error call per session
(round 5), v1 = one fsdkr_collect_first_error_multi call for the set.  Prints one
JSON line per step.  Diagnostics for DESIGN.md."""
import argparse
import copy
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
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    import torch
    from fsdkr import Context, refresh, synth
    from fsdkr import batch as B
    ctx = Context()
    sess = synth.synth_sessions(ctx, a.sessions, n=3, t=1, seed=2028, key_bits=3072)
    multi = B.SessionSet.first_errors

    def per_session(self, verdicts):
        return {s: self.first_error(s, verdicts) for s in self.row}

    def run(v):
        B.SessionSet.first_errors = multi if v else per_session
        try:
            work = [(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in sess]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = refresh.collect_many(work, ctx=ctx, key_bits=3072)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
        finally:
            B.SessionSet.first_errors = multi
        assert all(r is None for r in res)
        return ms, ctx.collect_last_span_ms()
    run(0)
    run(1)
    for r in range(a.rounds):
        for v in (0, 1):
            ms, span = run(v)
            print(json.dumps({"round": r, "variant": v, "ms": ms, "span_ms": span}), flush=True)


if __name__ == "__main__":
    main()
