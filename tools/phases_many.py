#!/usr/bin/env python3
"""Phase times of refresh.collect_many over BASELINE configs[4] (S independent
t=1 n=3 sessions, 3072-bit keys), in collect_many's own order: stage-1 gather,
GA prestart, stage 1b (Z) + the T^Z prestart, stage-2 gather, multi-session prepare, launch, share-recovery
launch, finish wait, recovery finish, per-session first error + key updates;
then the whole collect_many call and the device pipeline alone.  With
--gap-ms each instrumented call is preceded by an idle gap, so a rocprofv3
kernel trace can be cut per call (tools/prof_summary.py --gap).  Diagnostics
for DESIGN.md."""
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
    ap.add_argument("--gap-ms", type=float, default=0.0)
    a = ap.parse_args()
    import torch
    from fsdkr import Context, synth
    from fsdkr.batch import SessionSet
    from fsdkr.refresh import _apply_keys, _apply_share, _speculative_finish, _speculative_launch, collect_many
    ctx = Context()
    sess = synth.synth_sessions(ctx, a.sessions, n=3, t=1, seed=9, key_bits=3072)
    for rep in range(a.reps):
        work = [(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in sess]
        torch.cuda.synchronize()
        if a.gap_ms:
            time.sleep(a.gap_ms * 1e-3)
        t = [time.perf_counter()]
        sset = SessionSet([(m, lk, j) for m, lk, dk, j in work], 256, 3072, staged=True)
        t.append(time.perf_counter())
        ctx.collect_prestart_set(sset)
        t.append(time.perf_counter())
        if sset.stage1b():   # the table bases and correct-key inputs, a second prestart call
            ctx.collect_prestart_set(sset)
        if sset.stage_z():   # stage 1b (the ring-Pedersen Z rows), then the T^Z combs
            ctx.collect_prestart_rp_set(sset)
        t.append(time.perf_counter())
        sset.complete()
        t.append(time.perf_counter())
        ctx.collect_prepare_set(sset)
        t.append(time.perf_counter())
        ctx.collect_launch()
        t.append(time.perf_counter())
        pend = _speculative_launch(ctx, [(m, lk, len(m) + len(j)) for m, lk, dk, j in work])
        t.append(time.perf_counter())
        v = ctx.collect_finish_set(sset)
        t.append(time.perf_counter())
        specs = _speculative_finish(ctx, pend)
        t.append(time.perf_counter())
        for s, ((m, lk, dk, j), sp) in enumerate(zip(work, specs)):
            e = sset.first_error(s, v)
            _apply_keys(lk, m, j, e.keys_applied)
            assert e.variant == 0 and not isinstance(sp, Exception)
            _apply_share(lk, dk, sp)
        t.append(time.perf_counter())
        names = ["stage1_ms", "prestart_ms", "stage1b_z_prestart_rp_ms", "stage2_ms", "prepare_ms", "launch_ms", "recovery_launch_ms",
                 "finish_wait_ms", "recovery_finish_ms", "map_apply_ms"]
        out = {"sessions": a.sessions}
        out.update({k: (t[i + 1] - t[i]) * 1e3 for i, k in enumerate(names)})
        out["total_ms"] = (t[-1] - t[0]) * 1e3
        work2 = [(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in sess]
        torch.cuda.synchronize()
        t7 = time.perf_counter()
        collect_many(work2, ctx=ctx, key_bits=3072)
        out["collect_many_ms"] = (time.perf_counter() - t7) * 1e3
        print(json.dumps(out), flush=True)
    sset = SessionSet([(m, lk, j) for (m, j, lk, dk) in sess], 256, 3072)
    ctx.collect_prepare_set(sset)
    runs = []
    for _ in range(2):
        t0 = time.perf_counter()
        ctx.collect_launch()
        ctx.collect_finish_set(sset)
        runs.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"device_pipeline_ms": min(runs)}), flush=True)


if __name__ == "__main__":
    main()
