#!/usr/bin/env python3
"""PMC target for whole collect() calls (bench.py's step) with no other kernels
in the process: the synthetic workload is generated once (--gen-only, outside
the profiler) and pickled to --cache; a profiled run loads it and makes
1 + --steps refresh.collect() calls (with --sessions S: refresh.collect_many()
calls over S independent t=1 n=3 3072-bit sessions, bench.py's configs[4]
step), so every dispatch rocprofv3 records belongs to one of those calls
(tools/pmc_summary_step.py divides the counter totals by the call count)."""
import argparse
import copy
import os
import pickle
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
os.environ["GPU_MAX_HW_QUEUES"] = str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--joins", type=int, default=4)
    ap.add_argument("--t", type=int, default=32)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--sessions", type=int, default=0)
    ap.add_argument("--shard", type=int, default=0,
                    help="W: rank 0's shard.collect() of a W-way shard (the all-reduce replaced by the other "
                         "ranks' all-valid verdicts, as bench.py --emulate-shard)")
    ap.add_argument("--cache", required=True)
    ap.add_argument("--gen-only", action="store_true")
    a = ap.parse_args()
    import torch  # noqa: F401
    from fsdkr import Context, refresh, synth
    ctx = Context()
    if a.gen_only:
        if a.sessions:
            data = synth.synth_sessions(ctx, a.sessions, n=3, t=1, seed=a.seed, key_bits=3072)
        else:
            data = synth.synth_collect(ctx, a.n - a.joins, a.joins, a.t, a.seed)
        with open(a.cache, "wb") as f:
            pickle.dump(data, f)
        print(f"workload cached: {a.cache}", flush=True)
        return
    with open(a.cache, "rb") as f:   # written by this script (--gen-only) in the same session
        data = pickle.load(f)
    if a.sessions:
        for k in range(a.steps + 1):
            work = [(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in data]
            t0 = time.perf_counter()
            res = refresh.collect_many(work, ctx=ctx, key_bits=3072)
            assert all(r is None for r in res)
            print(f"collect_many {k} {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
        print(f"calls {a.steps + 1}", flush=True)
        return
    msgs, joins, lk = data
    keys = [copy.deepcopy(lk) for _ in range(a.steps + 1)]
    if a.shard:
        from fsdkr import shard
        R, J, n = len(msgs), len(joins), a.n

        class Rank0:   # bench.py --emulate-shard's stand-in for the process group
            class ReduceOp:
                MAX = None

            def get_world_size(self):
                return a.shard

            def get_rank(self):
                return 0

            def all_reduce(self, t, op=None):
                P, M = R * n, R + J
                for lo, hi, ok in ((0, P, 1), (P, 2 * P, 7), (2 * P, 3 * P, 1), (3 * P, 3 * P + 2 * M, 1),
                                   (3 * P + 2 * M, 3 * P + 2 * M + J, 3)):
                    t[lo:hi] = ok
        for k in range(a.steps + 1):
            t0 = time.perf_counter()
            shard.collect(Rank0(), msgs, keys[k], lk.paillier_dk, joins, ctx)
            print(f"shard collect {k} {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
        print(f"calls {a.steps + 1}", flush=True)
        return
    for k in range(a.steps + 1):
        t0 = time.perf_counter()
        refresh.collect(msgs, keys[k], lk.paillier_dk, joins, ctx=ctx)
        print(f"collect {k} {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    print(f"calls {a.steps + 1}", flush=True)


if __name__ == "__main__":
    main()
