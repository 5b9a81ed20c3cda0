"""ctypes driver of the C++ CPU baseline (oracle/cpu_baseline.cpp) -- TEST
INFRASTRUCTURE ONLY: bench.py's `cpu_baseline` leg and a second checker of the
GPU verdicts.  It runs the reference's verification algorithms with GMP (the
reference's bignum engine) over the same packed batch the product's C ABI
takes, on 1 thread and on many threads, on a bounded sample of the workload."""
import ctypes
import os
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libcpubase.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise ImportError(f"{LIB} missing (make -C oracle)")
        L = ctypes.CDLL(LIB)
        u8 = ctypes.POINTER(ctypes.c_uint8)
        L.cpubase_available.restype = ctypes.c_int
        L.cpubase_verify.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 5 + [u8] * 6 + \
            [ctypes.POINTER(ctypes.c_double)]
        L.cpubase_verify.restype = ctypes.c_int
        if not L.cpubase_available():
            raise OSError("libgmp.so.10 not loadable")
        _lib = L
    return _lib


def verify(batch, n_pairs, n_msgs, n_joins, n_fel, threads):
    """Verdicts of the first units of a packed fsdkr.batch.CollectBatch; returns
    (dict of uint8 arrays, seconds per phase)."""
    L = lib()
    u8 = ctypes.POINTER(ctypes.c_uint8)
    out = {k: np.zeros(max(c, 1), np.uint8) for k, c in (("pdl", n_pairs), ("range", n_pairs), ("ped", n_msgs),
                                                          ("ck", n_msgs), ("dlog", n_joins), ("feldman", n_fel))}
    secs = (ctypes.c_double * 5)()
    rc = L.cpubase_verify(ctypes.addressof(batch.c), n_pairs, n_msgs, n_joins, n_fel, threads,
                          *[out[k].ctypes.data_as(u8) for k in ("pdl", "range", "ped", "ck", "dlog", "feldman")],
                          secs)
    if rc != 0:
        raise RuntimeError("cpubase_verify failed")
    return out, list(secs)


def measure(batch, ref, threads=16, budget_s=12.0):
    """Time the CPU restatement on a bounded sample on 1 and on `threads` threads
    and extrapolate to the whole collect() (every pair, every message's
    ring-Pedersen + correct-key proof, every join's DLog proofs, every Feldman
    check).  `ref`: GPU Verdicts of the same batch; the sample must agree."""
    R, J, n = batch.R, batch.J, batch.n
    P, Mt = R * n, R + J
    t0 = time.perf_counter()
    # 1 thread: a small sample of each unit
    s1 = {"pairs": min(P, 12), "msgs": min(Mt, 1), "joins": min(J, 1), "fel": min(P, 32)}
    v1, sec1 = verify(batch, s1["pairs"], s1["msgs"], s1["joins"], s1["fel"], 1)
    # `threads` threads: enough units to keep every thread busy a few rounds
    sT = {"pairs": min(P, 4 * threads), "msgs": min(Mt, threads), "joins": min(J, threads),
          "fel": min(P, 64 * threads)}
    vT, secT = verify(batch, sT["pairs"], sT["msgs"], sT["joins"], sT["fel"], threads)
    wall = time.perf_counter() - t0
    agree = True
    for v, s in ((v1, s1), (vT, sT)):
        agree &= bool(np.array_equal(v["pdl"][:s["pairs"]], ref.pdl[:s["pairs"]] & 15))
        agree &= bool(np.array_equal(v["range"][:s["pairs"]], ref.range[:s["pairs"]]))
        agree &= bool(np.array_equal(v["ped"][:s["msgs"]], ref.ped[:s["msgs"]]))
        agree &= bool(np.array_equal(v["ck"][:s["msgs"]], ref.ck[:s["msgs"]]))
        agree &= bool(np.array_equal(v["feldman"][:s["fel"]], ref.feldman[:s["fel"]]))
        if J:
            agree &= bool(np.array_equal(v["dlog"][:s["joins"]], ref.dlog[:s["joins"]]))

    def extrapolate(sec, s):
        per = [sec[0] / max(s["pairs"], 1), sec[1] / max(s["msgs"], 1), sec[2] / max(s["msgs"], 1),
               sec[3] / max(s["joins"], 1), sec[4] / max(s["fel"], 1)]
        return P * per[0] + Mt * (per[1] + per[2]) + J * per[3] + P * per[4], per

    c1, per1 = extrapolate(sec1, s1)
    cT, perT = extrapolate(secT, sT)
    return {"cores": threads, "collect_s": cT, "single_thread_collect_s": c1,
            "per_pair_ms_1t": per1[0] * 1e3, "per_ring_pedersen_ms_1t": per1[1] * 1e3,
            "per_correct_key_ms_1t": per1[2] * 1e3, "per_feldman_ms_1t": per1[4] * 1e3,
            "verdicts_match_gpu": agree,
            "sample": f"C++ restatement over GMP (oracle/cpu_baseline.cpp, dlopen libgmp.so.10): {s1['pairs']} "
                      f"PDL+Alice pairs, {s1['msgs']} ring-Pedersen + correct-key, {s1['joins']} DLog, "
                      f"{s1['fel']} Feldman on 1 thread; {sT['pairs']} pairs, {sT['msgs']} RP+CK, {sT['joins']} "
                      f"DLog, {sT['fel']} Feldman on {threads} threads ({wall:.1f} s); extrapolated to the "
                      f"n={n} proof mix ({P} pairs, {Mt} messages, {J} joins)"}
