"""Co-residency probe: the GA-shaped launch of the n = 64 call (7 680 keyed
4096-bit chains, 16 lanes, sliding windows) timed alone and while a background
launch of equal wave count but different code runs on a second context/stream:

  same   the GA kernel itself (modexp_slide<144,16,128>, ~15 KB of code)
  m2048  2048-bit chains at 8 lanes (modexp_kernel<72,8,64>, ~14 KB)
  big    4096-bit fixed-window chains at 4 lanes (modexp_kernel<144,4,128>, ~105 KB)
  m2048s the m2048 shape at 60 waves (the wave count of the call's Feldman launch)
  feldman  the n = 64 call's Feldman launch (3 840 checks, 60 waves; a ~107 KB hot loop)
  pdl_u1   the n = 64 call's pdl_u1 launch (3 840 pairs, 240 waves; a ~96 KB hot loop)

The modexp backgrounds run 0.5 waves per SIMD, looped so it covers the whole
foreground launch.  If the large-code background stretches GA much more than
the small ones (at equal waves and similar instruction mix), the per-CU
instruction cache, not issue slots alone, is what the concurrent streams share.
One JSON line per (round, variant): foreground kernel ms, background launches
completed and their mean wall ms.
Usage: python tools/cobg_probe.py [--rounds 2] [--reps 3]"""
import argparse
import json
import os
import random
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fs-dkr_amd"))
import torch  # noqa: E402

from fsdkr._native import Context, ints_to_limbs  # noqa: E402


class Launch:
    """device-resident operands of one modexp launch and a call that runs it"""

    def __init__(self, ctx, k32, count, keyed, group, seed, nmod=16):
        rnd = random.Random(seed)
        rng = np.random.default_rng(seed)
        half = 16 * k32
        if k32 == 128:
            Ns = [rnd.getrandbits(half) | 1 | (1 << (half - 1)) for _ in range(nmod)]
            mods, exps, ebits = [n * n for n in Ns], Ns, half
        else:
            mods = [rnd.getrandbits(32 * k32) | 1 | (1 << (32 * k32 - 1)) for _ in range(nmod)]
            exps, ebits = [rnd.getrandbits(32 * k32) for _ in range(nmod)], 32 * k32
        idx = (np.arange(count) % nmod).astype(np.uint32)
        base = rng.integers(0, 2**32, size=(count, k32), dtype=np.uint64).astype(np.uint32)
        base[:, -1] >>= 1
        E = ints_to_limbs(exps if keyed else [exps[i] for i in idx], (ebits + 31) // 32)
        dev = torch.device("cuda")
        self.t = [torch.from_numpy(x.view(np.int32)).to(dev) for x in (base, E, idx, ints_to_limbs(mods, k32))]
        self.out = torch.empty((count, k32), dtype=torch.int32, device=dev)
        self.args = (k32, count, E.shape[1], ebits, nmod)
        self.fn = ctx._lib.fsdkr_modexp_keyed_device if keyed else ctx._lib.fsdkr_modexp_batch_device
        self.ctx, self.group = ctx, group
        self.check = (base, exps, idx, mods)
        torch.cuda.synchronize()

    def __call__(self):
        k32, count, ew, ebits, nmod = self.args
        b, e, i, m = self.t
        self.ctx.check(self.fn(self.ctx.handle, k32, count, b.data_ptr(), e.data_ptr(), ew, ebits, i.data_ptr(),
                               m.data_ptr(), nmod, self.out.data_ptr()))

    def verify(self, n=4):
        base, exps, idx, mods = self.check
        out = self.out.cpu().numpy().view(np.uint32)
        for i in range(0, len(idx), max(1, len(idx) // n)):
            b = int.from_bytes(base[i].tobytes(), "little")
            assert int.from_bytes(out[i].tobytes(), "little") == pow(b, exps[idx[i]], mods[idx[i]]), i


P256 = 2**256 - 2**32 - 977
N256 = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


def ec_points(count):
    """G, 2G, 3G, ... (affine secp256k1)"""
    lam = 3 * GX * GX * pow(2 * GY, -1, P256) % P256   # 2G
    x = (lam * lam - 2 * GX) % P256
    y = (lam * (GX - x) - GY) % P256
    out = [(GX, GY), (x, y)]
    for _ in range(count - 2):
        lam = (y - GY) * pow(x - GX, -1, P256) % P256
        x3 = (lam * lam - x - GX) % P256
        y = (lam * (x - x3) - y) % P256
        x = x3
        out.append((x, y))
    return out


class Feldman:
    def __init__(self, ctx, n_msgs=60, n=64, t=32):
        pts = ec_points(n_msgs * (t + 1) + n_msgs * n)
        self.vss = [pts[i * (t + 1):(i + 1) * (t + 1)] for i in range(n_msgs)]
        self.commit = pts[n_msgs * (t + 1):]
        self.ctx, self.n, self.t = ctx, n, t

    def __call__(self):
        self.ctx.feldman_check(self.vss, self.commit, self.n, self.t)

    def verify(self, n=0):
        pass


class PdlU1:
    def __init__(self, ctx, count=3840):
        rnd = random.Random(3)
        pts = ec_points(2 * count)
        self.args = ([rnd.getrandbits(768) for _ in range(count)], [rnd.getrandbits(256) for _ in range(count)],
                     pts[:count], pts[count:])
        self.ctx = ctx

    def __call__(self):
        self.ctx.pdl_u1_check(*self.args)

    def verify(self, n=0):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--fg-count", type=int, default=7680)
    ap.add_argument("--bg-waves", type=int, default=512)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    fg_ctx, bg_ctx = Context(device=0, timing=True), Context(device=0, timing=True)
    fg_ctx.set_modexp_group(16)
    fg = Launch(fg_ctx, 128, a.fg_count, True, 16, 11)
    W = a.bg_waves
    bgs = {"same": (128, W * 4, True, 16), "m2048": (2048 // 32, W * 8, False, 8), "big": (128, W * 16, False, 4),
           "m2048s": (2048 // 32, 60 * 8, False, 8), "feldman": (0, 0, False, 0), "pdl_u1": (0, 0, False, 0)}
    bg = {}
    for name, (k32, count, keyed, group) in bgs.items():
        if name == "feldman":
            bg[name] = Feldman(bg_ctx)
        elif name == "pdl_u1":
            bg[name] = PdlU1(bg_ctx)
        else:
            bg[name] = Launch(bg_ctx, k32, count, keyed, group, 20 + len(bg))
    fg()
    fg.verify()
    for r in range(a.rounds):
        for name in ["none"] + list(bgs):
            stop, done = threading.Event(), []
            th = None
            if name != "none":
                bg_ctx.set_modexp_group(bgs[name][3])
                bg_ctx.kernel_time_reset()
                L = bg[name]

                def loop():
                    while not stop.is_set():
                        t0 = time.perf_counter()
                        L()
                        done.append(time.perf_counter() - t0)
                th = threading.Thread(target=loop)
                th.start()
                time.sleep(0.15)   # the background launch is resident
            fg_ctx.kernel_time_reset()
            for _ in range(a.reps):
                fg()
            torch.cuda.synchronize()
            kms, kn = fg_ctx.kernel_time("modexp")
            n_during = len(done)
            stop.set()
            if th is not None:
                th.join()
                bg[name].verify(2)
            fg.verify(2)
            bk = sum(bg_ctx.kernel_time(k)[0] for k in ("modexp", "feldman", "pdl_u1")) if th is not None else 0.0
            print(json.dumps({"round": r, "background": name, "fg_kernel_ms": kms / max(kn, 1), "fg_launches": kn,
                              "bg_kernel_ms_total": bk,
                              "bg_launches_done": n_during,
                              "bg_wall_ms_mean": (1e3 * sum(done) / len(done)) if done else None}), flush=True)
    # each background alone (its own duration at this wave count)
    for name, (k32, count, keyed, group) in bgs.items():
        bg_ctx.set_modexp_group(group)
        bg_ctx.kernel_time_reset()
        t0 = time.perf_counter()
        for _ in range(2):
            bg[name]()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 2
        res = {k: bg_ctx.kernel_time(k) for k in ("modexp", "feldman", "pdl_u1")}
        print(json.dumps({"background_alone": name, "wall_ms": wall * 1e3,
                          "kernels": {k: v[0] / max(v[1], 1) for k, v in res.items() if v[1]}}), flush=True)
    fg_ctx.close()
    bg_ctx.close()


if __name__ == "__main__":
    main()
