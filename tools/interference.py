"""Latency of a small serial chain while a large modexp launch occupies the
chip (two contexts = two HIP streams, two host threads).  Separates
co-residency effects (shared SIMDs / instruction cache / clocks) from the
chain's own latency: `python tools/interference.py [--bg-count N]`."""
import argparse
import json
import os
import random
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fs-dkr_amd"))

from fsdkr._native import Context  # noqa: E402


def fb_case(ctx, bases=136, per_base=14, bits=2816):
    rnd = random.Random(5)
    mods = [rnd.getrandbits(2048) | 1 | (1 << 2047) for _ in range(bases)]
    bs = [rnd.getrandbits(2047) for _ in range(bases)]
    bidx = [k // per_base for k in range(bases * per_base)]
    exps = [rnd.getrandbits(bits) for _ in bidx]
    ctx.kernel_time_reset()
    ctx.fixed_base_modexp(bs, list(range(bases)), mods, bidx, exps, 64)
    return ctx.kernel_time("fb_table")[0]


def chain_case(ctx, count=64, bits=2816):
    """variable-base 2048-bit modexp chains (the GD / CK shape)"""
    rnd = random.Random(6)
    mods = [rnd.getrandbits(2048) | 1 | (1 << 2047) for _ in range(count)]
    ctx.kernel_time_reset()
    ctx.modexp_batch([rnd.getrandbits(2047) for _ in range(count)], [rnd.getrandbits(bits) for _ in range(count)],
                     mods, list(range(count)), 64)
    return ctx.kernel_time("modexp")[0]


def background_prepare(ctx, count):
    """device-resident operands of a metric-2 launch (base^N mod N^2)"""
    import numpy as np
    import torch
    from fsdkr._native import ints_to_limbs
    rnd = random.Random(7)
    Ns = [rnd.getrandbits(2048) | 1 | (1 << 2047) for _ in range(16)]
    mods = [n * n for n in Ns]
    idx = (np.arange(count) % 16).astype(np.uint32)
    base = np.random.default_rng(7).integers(0, 2 ** 32, size=(count, 128), dtype=np.uint64).astype(np.uint32)
    base[:, -1] >>= 1
    dev = torch.device("cuda")
    t = dict(b=torch.from_numpy(base.view(np.int32)).to(dev),
             e=torch.from_numpy(ints_to_limbs([Ns[i] for i in idx], 64).view(np.int32)).to(dev),
             i=torch.from_numpy(idx.view(np.int32)).to(dev),
             m=torch.from_numpy(ints_to_limbs(mods, 128).view(np.int32)).to(dev),
             o=torch.empty((count, 128), dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    return t


def background(ctx, count, t, out):
    t0 = time.perf_counter()
    ctx.check(ctx._lib.fsdkr_modexp_batch_device(ctx.handle, 128, count, t["b"].data_ptr(), t["e"].data_ptr(), 64,
                                                 2048, t["i"].data_ptr(), t["m"].data_ptr(), 16, t["o"].data_ptr()))
    out["bg_s"] = time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bg-count", type=int, default=65536)
    a = ap.parse_args()
    import torch
    torch.cuda.init()        # torch initialises HIP first (as in bench.py), then the contexts
    c1, c2 = Context(timing=True), Context(timing=True)
    res = {"alone_fb_table_ms": fb_case(c2), "alone_chain_ms": chain_case(c2)}
    t = background_prepare(c1, a.bg_count)
    for name, fn in (("fb_table", fb_case), ("chain", chain_case)):
        out = {}
        th = threading.Thread(target=background, args=(c1, a.bg_count, t, out))
        th.start()
        time.sleep(0.03)         # the background kernel is resident and running
        res[f"loaded_{name}_ms"] = fn(c2)
        th.join()
        res[f"bg_{name}_s"] = out["bg_s"]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
