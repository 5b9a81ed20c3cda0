#!/usr/bin/env python3
"""Per-rank latency of a W-way shard of the n=64 collect (rank 0's whole
shard.collect() call with the all-reduce replaced by the other ranks' all-valid
verdicts, as bench.py --emulate-shard) under several context settings, on one
synthetic workload: `--env "FSDKR_GA_CUS=0" "FSDKR_GA_CUS=128" ...`, each run
in a fresh Context (the knobs are read at context creation), interleaved."""
import argparse
import copy
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
os.environ["GPU_MAX_HW_QUEUES"] = str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))


class Rank0:
    class ReduceOp:
        MAX = None

    def __init__(self, W, R, J, n):
        self.W, self.R, self.J, self.n = W, R, J, n

    def get_world_size(self):
        return self.W

    def get_rank(self):
        return 0

    def all_reduce(self, t, op=None):
        P, M, J = self.R * self.n, self.R + self.J, self.J
        for lo, hi, ok in ((0, P, 1), (P, 2 * P, 7), (2 * P, 3 * P, 1), (3 * P, 3 * P + 2 * M, 1),
                           (3 * P + 2 * M, 3 * P + 2 * M + J, 3)):
            t[lo:hi] = ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[8])
    ap.add_argument("--env", nargs="+", default=["FSDKR_GA_CUS=0"])
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch
    from fsdkr import Context, shard, synth
    torch.cuda.set_device(0)
    gen = Context()
    msgs, joins, lk = synth.synth_collect(gen, 60, 4, 32, 2024, key_bits=2048)
    gen.close()
    R, J = len(msgs), len(joins)
    n = R + J
    res = {}
    for rnd in range(a.rounds):
        for W in a.world:
            for env in a.env:
                kvs = [kv.split("=", 1) for kv in env.split("+")]   # K=V[+K2=V2...]
                saved = {k: os.environ.get(k) for k, _ in kvs}
                for k, v in kvs:
                    os.environ[k] = v
                ctx = Context()
                dist = Rank0(W, R, J, n)
                keys = [copy.deepcopy(lk) for _ in range(a.steps + 2)]
                for s in range(2):
                    shard.collect(dist, msgs, keys[s], lk.paillier_dk, joins, ctx)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for s in range(a.steps):
                    shard.collect(dist, msgs, keys[2 + s], lk.paillier_dk, joins, ctx)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / a.steps * 1e3
                ctx.close()
                for k, v in saved.items():
                    if v is None:
                        del os.environ[k]
                    else:
                        os.environ[k] = v
                res.setdefault((W, env), []).append(ms)
                print(json.dumps({"world": W, "env": env, "round": rnd, "rank0_collect_ms": ms}), flush=True)
    for (W, env), v in sorted(res.items()):
        print(json.dumps({"world": W, "env": env, "min_ms": min(v), "runs": v}), flush=True)


if __name__ == "__main__":
    main()
