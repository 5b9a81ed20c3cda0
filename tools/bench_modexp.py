"""Metric-2 microbench: 4096-bit modexp/s (base U[0,N^2), exponent N, modulus
N^2 of seeded 2048-bit N) with operands resident in HBM, plus 2048/2048."""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fs-dkr_amd"))
import torch  # noqa: E402

from fsdkr._native import Context, ints_to_limbs  # noqa: E402

PEAK_MAC = 3.40e13   # measured v_mad_u64_u32 lane-ops/s, profiles/r01_intrates.jsonl


def mmacs(k32, ebits):
    return (ebits + (ebits + 4) // 5) * (2 * k32 * k32 + k32)


def run(ctx, k32, count, nmod, reps, seed, keyed=False):
    rng = np.random.default_rng(seed)
    import random
    rnd = random.Random(seed)
    half = 16 * k32
    Ns = [rnd.getrandbits(half) | 1 | (1 << (half - 1)) for _ in range(nmod)]
    if k32 in (128, 192):
        mods = [n * n for n in Ns]
        ebits_nominal = half
        exps_int = Ns
    else:
        mods = [rnd.getrandbits(32 * k32) | 1 | (1 << (32 * k32 - 1)) for _ in range(nmod)]
        exps_int = [rnd.getrandbits(32 * k32) for _ in range(nmod)]
        ebits_nominal = 32 * k32
    idx = (np.arange(count) % nmod).astype(np.uint32)
    base = rng.integers(0, 2**32, size=(count, k32), dtype=np.uint64).astype(np.uint32)
    base[:, -1] >>= 1  # < 2^(32k-1) <= N^2 for top-bit-set moduli (uniform below that bound)
    # keyed: one exponent row per modulus (fsdkr_modexp_keyed_device, sliding windows)
    E = ints_to_limbs(exps_int if keyed else [exps_int[i] for i in idx], (ebits_nominal + 31) // 32)
    M = ints_to_limbs(mods, k32)
    dev = torch.device("cuda")
    d_base = torch.from_numpy(base.view(np.int32)).to(dev)
    d_exp = torch.from_numpy(E.view(np.int32)).to(dev)
    d_idx = torch.from_numpy(idx.view(np.int32)).to(dev)
    d_mod = torch.from_numpy(M.view(np.int32)).to(dev)
    d_out = torch.empty((count, k32), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    L = ctx._lib
    fn = L.fsdkr_modexp_keyed_device if keyed else L.fsdkr_modexp_batch_device

    def once():
        ctx.check(fn(ctx.handle, k32, count, d_base.data_ptr(), d_exp.data_ptr(),
                                              E.shape[1], ebits_nominal, d_idx.data_ptr(), d_mod.data_ptr(),
                                              nmod, d_out.data_ptr()))
    once()
    ctx.kernel_time_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    kms, kn = ctx.kernel_time("modexp")
    kms /= max(kn, 1)
    # spot check 8 results against pow
    out = d_out.cpu().numpy().view(np.uint32)
    for i in range(0, count, max(1, count // 8)):
        b = int.from_bytes(base[i].tobytes(), "little")
        r = int.from_bytes(out[i].tobytes(), "little")
        assert r == pow(b, exps_int[idx[i]], mods[idx[i]]), f"mismatch at {i}"
    W = mmacs(k32, ebits_nominal)
    rate = count / (kms * 1e-3)
    return {"mod_bits": 32 * k32, "exp_bits": ebits_nominal, "count": count, "wall_ms": wall * 1e3,
            "kernel_ms": kms, "modexp_per_s": rate, "wall_modexp_per_s": count / wall,
            "achieved_mac_per_s": rate * W, "frac_of_peak": rate * W / PEAK_MAC}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--count", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--widths", default="128,64")
    ap.add_argument("--groups", default="0", help="lanes per instance to force (0 = automatic), comma list")
    ap.add_argument("--keyed", action="store_true", help="fsdkr_modexp_keyed_device (exponent per modulus)")
    a = ap.parse_args()
    ctx = Context(timing=True)
    for k in [int(x) for x in a.widths.split(",")]:
        for g in [int(x) for x in a.groups.split(",")]:
            ctx.set_modexp_group(g)
            r = run(ctx, k, a.count, 16, a.reps, 1234 + k, a.keyed)
            r["group"] = g
            r["keyed"] = a.keyed
            print(json.dumps(r), flush=True)
    ctx.set_modexp_group(0)
