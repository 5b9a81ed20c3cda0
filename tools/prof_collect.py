#!/usr/bin/env python3
"""Device-pipeline profile target: K collect_run calls (no host work between
launches beyond the verdict readback, 20 ms idle gaps so tools/prof_summary.py
--gap can cut the steps) on BASELINE configs[2] (n=64 + 4 joins) or, with
--sessions S, on S independent t=1 n=3 3072-bit sessions (configs[4])."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
# --hwq N sets the hardware queue count exactly (1 serialises every stream: each
# kernel's standalone full-chip duration); default: at least 12 like bench.py
_hwq = next((sys.argv[i + 1] for i, x in enumerate(sys.argv[:-1]) if x == "--hwq"), None)
os.environ["GPU_MAX_HW_QUEUES"] = _hwq or str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--sessions", type=int, default=0)
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--joins", type=int, default=4)
    ap.add_argument("--t", type=int, default=32)
    ap.add_argument("--hwq", type=int, default=0)
    ap.add_argument("--full", action="store_true",
                    help="time whole refresh.collect() calls (bench.py's step) instead of collect_run")
    a = ap.parse_args()
    import torch  # noqa: F401
    from fsdkr import Context, synth
    from fsdkr.batch import CollectBatch
    ctx = Context()
    if a.sessions:
        sess = synth.synth_sessions(ctx, a.sessions, n=3, t=1, seed=5, key_bits=3072)
        if a.full:   # whole refresh.collect_many() calls (bench.py's configs[4] step)
            import copy
            from fsdkr import refresh
            for k in range(a.steps + 1):
                work = [(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in sess]
                time.sleep(0.02)
                t0 = time.perf_counter()
                refresh.collect_many(work, ctx=ctx, key_bits=3072)
                print(f"collect_many {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
            return
        batches = [CollectBatch(m, lk, j, 256, 3072) for (m, j, lk, dk) in sess]
        ctx.collect_prepare_many(batches)
        for _ in range(a.steps):
            time.sleep(0.02)
            t0 = time.perf_counter()
            ctx.collect_launch()
            ctx.collect_finish_many(batches)
            print(f"multi-session run {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
        return
    msgs, joins, lk = synth.synth_collect(ctx, a.n - a.joins, a.joins, a.t, 2024)
    if a.full:
        import copy
        from fsdkr import refresh
        keys = [copy.deepcopy(lk) for _ in range(a.steps + 1)]
        refresh.collect(msgs, keys[-1], lk.paillier_dk, joins, ctx=ctx)
        for k in range(a.steps):
            time.sleep(0.02)
            t0 = time.perf_counter()
            refresh.collect(msgs, keys[k], lk.paillier_dk, joins, ctx=ctx)
            print(f"collect {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
        return
    b = CollectBatch(msgs, lk, joins, 256, 2048)
    ctx.collect_prepare(b)
    for _ in range(a.steps):
        time.sleep(0.02)
        t0 = time.perf_counter()
        ctx.collect_run(b)
        print(f"collect_run {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
