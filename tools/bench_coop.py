"""Latency-shape comparison for shard-sized launches: 4096-bit s^N mod N^2
chains (GA's shape; 64 receivers, exponent N) at the counts of an 8 / 4 / 2-way
n = 64 rank, on the 16-lane CIOS shape (fixed windows through
fsdkr_modexp_batch) and on the one-wave cooperative shape (coop.hip, group
256).  Kernel time from the context's HIP events; every result checked against
pow on a sample."""
import argparse
import json
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fs-dkr_amd"))

from fsdkr._native import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--counts", default="1024,2048")
    ap.add_argument("--groups", default="16,256")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--limbs", type=int, default=128)
    a = ap.parse_args()
    ctx = Context()
    ctx.set_timing(True)
    rnd = random.Random(5)
    half = 16 * a.limbs
    ns = [rnd.getrandbits(half) | 1 | (1 << (half - 1)) for _ in range(64)]
    mods = [n * n for n in ns]
    for count in [int(x) for x in a.counts.split(",")]:
        idx = [i * 64 // count for i in range(count)]
        bases = [rnd.getrandbits(32 * a.limbs - 1) for _ in range(count)]
        exps = [ns[k] for k in idx]
        for g in [int(x) for x in a.groups.split(",")]:
            ctx.set_modexp_group(g)
            ctx.modexp_batch(bases[:64], exps[:64], mods, idx[:64], a.limbs)   # warm
            ctx.kernel_time_reset()
            for _ in range(a.reps):
                out = ctx.modexp_batch(bases, exps, mods, idx, a.limbs)
            ms, n = ctx.kernel_time("modexp")
            ok = all(out[i] == pow(bases[i], exps[i], mods[idx[i]]) for i in range(0, count, max(1, count // 16)))
            print(json.dumps({"count": count, "group": g, "kernel_ms": ms / max(n, 1), "launches": n, "ok": ok}),
                  flush=True)
    ctx.set_modexp_group(0)


if __name__ == "__main__":
    main()
