#!/usr/bin/env python3
"""Phase times of one RefreshMessage::collect() at a BASELINE config (default
n = 64, t = 32, 60 refresh + 4 joins, 2048-bit): host-mirror packing
(CollectBatch), collect_prepare (host pre-pass + H2D), collect_run (kernels +
verdict readback), first_error, share recovery.  Diagnostics for DESIGN.md;
FSDKR_PREP_PROFILE=1 adds the pre-pass breakdown on stderr."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
os.environ["GPU_MAX_HW_QUEUES"] = str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--t", type=int, default=32)
    ap.add_argument("--joins", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch  # noqa: F401  (device init like bench.py)
    from fsdkr import Context, synth
    from fsdkr.batch import CollectBatch
    ctx = Context()
    R, J = a.n - a.joins, a.joins
    msgs, joins, lk = synth.synth_collect(ctx, R, J, a.t, 2024)
    import copy
    from fsdkr.refresh import collect, _speculative
    for rep in range(a.reps):
        t0 = time.perf_counter()
        b = CollectBatch(msgs, lk, joins, 256, 2048)
        t1 = time.perf_counter()
        ctx.collect_prepare(b)
        t2 = time.perf_counter()
        ctx.collect_launch()
        t3 = time.perf_counter()
        spec = _speculative(ctx, [(msgs, lk, a.n)])[0]
        t4 = time.perf_counter()
        v = ctx.collect_finish(b)
        t5 = time.perf_counter()
        e = b.first_error(v)
        t6 = time.perf_counter()
        assert e.variant == 0 and not isinstance(spec, Exception)
        k2 = copy.deepcopy(lk)
        t7 = time.perf_counter()
        collect(msgs, k2, lk.paillier_dk, joins, ctx=ctx)
        t8 = time.perf_counter()
        print(json.dumps({"pack_ms": (t1 - t0) * 1e3, "prepare_ms": (t2 - t1) * 1e3, "launch_ms": (t3 - t2) * 1e3,
                          "recovery_overlapped_ms": (t4 - t3) * 1e3, "finish_wait_ms": (t5 - t4) * 1e3,
                          "first_error_ms": (t6 - t5) * 1e3, "collect_full_ms": (t8 - t7) * 1e3}), flush=True)
    # device pipeline alone, for reference
    ctx.collect_prepare(b)
    for _ in range(2):
        t0 = time.perf_counter()
        ctx.collect_run(b)
        print(json.dumps({"run_ms": (time.perf_counter() - t0) * 1e3}), flush=True)


if __name__ == "__main__":
    main()
