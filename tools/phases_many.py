#!/usr/bin/env python3
"""Phase times of refresh.collect_many over BASELINE configs[4] (S independent
t=1 n=3 sessions, 3072-bit keys): per-session packing, the multi-session
prepare, launch, overlapped share recovery, finish, per-session first error +
key updates; plus the device pipeline alone.  Diagnostics for DESIGN.md."""
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
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch  # noqa: F401
    from fsdkr import Context, synth
    from fsdkr.refresh import _apply_keys, _apply_share, _speculative, collect_many
    ctx = Context()
    sess = synth.synth_sessions(ctx, a.sessions, n=3, t=1, seed=9, key_bits=3072)
    from fsdkr.batch import SessionSet
    for rep in range(a.reps):
        work = [(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in sess]
        t0 = time.perf_counter()
        sset = SessionSet([(m, lk, j) for m, lk, dk, j in work], 256, 3072)
        t1 = time.perf_counter()
        ctx.collect_prepare_set(sset)
        t2 = time.perf_counter()
        ctx.collect_launch()
        t3 = time.perf_counter()
        specs = _speculative(ctx, [(m, lk, len(m) + len(j)) for m, lk, dk, j in work])
        t4 = time.perf_counter()
        v = ctx.collect_finish_set(sset)
        t5 = time.perf_counter()
        for s, ((m, lk, dk, j), sp) in enumerate(zip(work, specs)):
            e = sset.first_error(s, v)
            _apply_keys(lk, m, j, e.keys_applied)
            assert e.variant == 0 and not isinstance(sp, Exception)
            _apply_share(lk, dk, sp)
        t6 = time.perf_counter()
        work2 = [(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in sess]
        t7 = time.perf_counter()
        collect_many(work2, ctx=ctx, key_bits=3072)
        t8 = time.perf_counter()
        print(json.dumps({"sessions": a.sessions, "pack_ms": (t1 - t0) * 1e3, "prepare_ms": (t2 - t1) * 1e3,
                          "launch_ms": (t3 - t2) * 1e3, "recovery_overlapped_ms": (t4 - t3) * 1e3,
                          "finish_wait_ms": (t5 - t4) * 1e3, "map_apply_ms": (t6 - t5) * 1e3,
                          "collect_many_ms": (t8 - t7) * 1e3}), flush=True)
    runs = []
    for _ in range(2):
        t0 = time.perf_counter()
        ctx.collect_launch()
        ctx.collect_finish_set(sset)
        runs.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"device_pipeline_ms": min(runs)}), flush=True)


if __name__ == "__main__":
    main()
