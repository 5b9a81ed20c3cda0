#!/usr/bin/env python3
"""Host-only timing of the configs[4] SessionSet pack (stage 1 + stage 2) over
1024 shape-correct t=1 n=3 sessions with random 3072-bit field values (no GPU,
no valid proofs: the pack only reads shapes and integers).  Diagnostics for
DESIGN.md; the phase split of the real call is tools/phases_many.py."""
import argparse
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]

from fsdkr import types as T   # noqa: E402
from fsdkr.batch import SessionSet   # noqa: E402


def fake_sessions(S, n=3, t=1, bits=3072, M=256, seed=1):
    rnd = random.Random(seed)

    def r(b=bits):
        return rnd.getrandbits(b) | 1

    def pt():
        return (r(256), r(256))
    # share the expensive-to-build big vectors between messages (the pack reads them per message)
    A = tuple(r() for _ in range(M))
    Z = tuple(r() for _ in range(M))
    sig = tuple(r() for _ in range(11))
    out = []
    for s in range(S):
        keys = [T.EncryptionKey(r(), 0) for _ in range(n)]
        sts = [T.DLogStatement(r(), r(), r()) for _ in range(n)]
        lk = T.LocalKey(None, [], 0, None, keys, None, sts, T.VerifiableSS(t, n, []), 1, t, n)
        msgs = []
        for k in range(n):
            pdl = [T.PDLwSlackProof(r(), pt(), r(2 * bits - 8), r(), r(770), r(), r(770 + bits)) for _ in range(n)]
            rng = [T.AliceProof(r(), r(256), r(), r(770), r(770 + bits)) for _ in range(n)]
            rps = T.RingPedersenStatement(r(), r(), r(), 0, keys[k])
            msgs.append(T.RefreshMessage(k + 1, k + 1, pdl, rng, T.VerifiableSS(t, n, [pt() for _ in range(t + 1)]),
                                         [pt() for _ in range(n)], [r(2 * bits - 8) for _ in range(n)],
                                         T.NiCorrectKeyProof(sig), sts[k], keys[k], [], None, rps,
                                         T.RingPedersenProof(A, Z)))
        out.append((msgs, lk, []))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--split", action="store_true", help="time gather / convert / points separately")
    a = ap.parse_args()
    sess = fake_sessions(a.sessions)
    acc = {}
    if a.split:
        from fsdkr import batch as B

        def wrap(name):
            f = getattr(B, name)

            def g(*x, **k):
                t = time.perf_counter()
                r = f(*x, **k)
                acc[name] = acc.get(name, 0.0) + (time.perf_counter() - t) * 1e3
                return r
            setattr(B, name, g)
        for name in ("_gather", "_convert", "pack_points"):
            wrap(name)
    for _ in range(a.reps):
        acc.clear()
        t0 = time.perf_counter()
        sset = SessionSet(sess, 256, 3072, staged=True)
        t1 = time.perf_counter()
        sset.stage1b()
        tb = time.perf_counter()
        sset.stage_z()
        tz = time.perf_counter()
        sset.complete()
        t2 = time.perf_counter()
        out = {"sessions": a.sessions, "stage1_ms": (t1 - t0) * 1e3, "stage1b_ms": (tb - t1) * 1e3,
               "stage_z_ms": (tz - tb) * 1e3, "stage2_ms": (t2 - tz) * 1e3}
        out.update({k.strip("_") + "_ms": v for k, v in acc.items()})
        print(json.dumps(out), flush=True)
        del sset


if __name__ == "__main__":
    main()
