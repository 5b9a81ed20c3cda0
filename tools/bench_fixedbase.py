"""Fixed-base engine timing: table chain latency (fb_table) and exponent phase
(fb_exp) for `bases` bases with `per_base` exponents of `bits` bits each
(h2_i with 2816-bit s3 / s2, ring-Pedersen T with 2048-bit Z)."""
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
    ap.add_argument("--bases", type=int, default=136)
    ap.add_argument("--per-base", type=int, default=14)
    ap.add_argument("--bits", type=int, default=2816)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    rnd = random.Random(5)
    mods = [rnd.getrandbits(2048) | 1 | (1 << 2047) for _ in range(a.bases)]
    bases = [rnd.getrandbits(2047) for _ in range(a.bases)]
    bidx = [k // a.per_base for k in range(a.bases * a.per_base)]
    exps = [rnd.getrandbits(a.bits) for _ in bidx]
    ctx = Context(timing=True)
    out = ctx.fixed_base_modexp(bases, list(range(a.bases)), mods, bidx, exps, 64)
    assert out[0] == pow(bases[0], exps[0], mods[0])
    ctx.kernel_time_reset()
    for _ in range(a.reps):
        ctx.fixed_base_modexp(bases, list(range(a.bases)), mods, bidx, exps, 64)
    tt, nt = ctx.kernel_time("fb_table")
    te, ne = ctx.kernel_time("fb_exp")
    tc, nc = ctx.kernel_time("comb_exp")
    print(json.dumps({"bases": a.bases, "per_base": a.per_base, "bits": a.bits, "fb_table_ms": tt / max(nt, 1),
                      "fb_exp_ms": te / max(ne, 1), "comb_exp_ms": tc / max(nc, 1), "comb_launches": nc,
                      "table_us_per_square": tt / max(nt, 1) * 1e3 / a.bits}))


if __name__ == "__main__":
    main()
