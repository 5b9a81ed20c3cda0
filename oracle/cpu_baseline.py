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


def host_cores():
    """What the host offers this process: nproc (os.cpu_count: on a GPU box the
    whole machine's CPUs), the scheduler affinity set, the cgroup CPU quota, the
    job's CPU share (OMP_NUM_THREADS: 16 per GPU on the GPU boxes), and
    `available` = the smallest of those (the cores a run may actually use)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    share = os.environ.get("OMP_NUM_THREADS")
    share = int(share) if share and share.isdigit() and int(share) > 0 else None
    avail = min(nproc, aff, int(quota + 0.999) if quota else nproc, share or nproc)
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "job_cpu_share": share,
            "available": max(1, avail)}


def _agree(v, s, ref, J):
    ok = bool(np.array_equal(v["pdl"][:s["pairs"]], ref.pdl[:s["pairs"]] & 15))
    ok &= bool(np.array_equal(v["range"][:s["pairs"]], ref.range[:s["pairs"]]))
    ok &= bool(np.array_equal(v["ped"][:s["msgs"]], ref.ped[:s["msgs"]]))
    ok &= bool(np.array_equal(v["ck"][:s["msgs"]], ref.ck[:s["msgs"]]))
    ok &= bool(np.array_equal(v["feldman"][:s["fel"]], ref.feldman[:s["fel"]]))
    if J:
        ok &= bool(np.array_equal(v["dlog"][:s["joins"]], ref.dlog[:s["joins"]]))
    return ok


def measure(batch, ref, threads=16, budget_s=12.0):
    """Time the CPU restatement over the WHOLE collect() verification of the batch
    (every pair, every message's ring-Pedersen + correct-key proof, every join's
    DLog proofs, every Feldman check) on `threads` threads, wall clock, and
    compare every verdict with the GPU's (`ref`).  The single-thread figure is a
    bounded sample extrapolated to the same mix (the whole n = 64 call would take
    ~100 s on one core)."""
    R, J, n = batch.R, batch.J, batch.n
    P, Mt = R * n, R + J
    # `threads` threads: the whole verification, timed end to end
    t0 = time.perf_counter()
    vT, secT = verify(batch, P, Mt, J, P, threads)
    full_s = time.perf_counter() - t0
    # 1 thread: a small sample of each unit
    s1 = {"pairs": min(P, 12), "msgs": min(Mt, 1), "joins": min(J, 1), "fel": min(P, 32)}
    v1, sec1 = verify(batch, s1["pairs"], s1["msgs"], s1["joins"], s1["fel"], 1)
    sT = {"pairs": P, "msgs": Mt, "joins": J, "fel": P}
    agree = _agree(v1, s1, ref, J) and _agree(vT, sT, ref, J)
    hc = host_cores()
    all_cores = None
    if hc["available"] != threads:   # the same whole verification on every core the host gives this run
        t0 = time.perf_counter()
        vA, _ = verify(batch, P, Mt, J, P, hc["available"])
        a_s = time.perf_counter() - t0
        agree = agree and _agree(vA, sT, ref, J)
        all_cores = {"threads": hc["available"], "collect_s": a_s}
    per1 = [sec1[0] / max(s1["pairs"], 1), sec1[1] / max(s1["msgs"], 1), sec1[2] / max(s1["msgs"], 1),
            sec1[3] / max(s1["joins"], 1), sec1[4] / max(s1["fel"], 1)]
    c1 = P * per1[0] + Mt * (per1[1] + per1[2]) + J * per1[3] + P * per1[4]
    return {"cores": threads, "host_cores": hc, "all_cores": all_cores, "collect_s": full_s,
            "collect_phases_s": dict(zip(
                ("pairs", "ring_pedersen", "correct_key", "dlog", "feldman"), secT)),
            "single_thread_collect_s": c1,
            "per_pair_ms_1t": per1[0] * 1e3, "per_ring_pedersen_ms_1t": per1[1] * 1e3,
            "per_correct_key_ms_1t": per1[2] * 1e3, "per_feldman_ms_1t": per1[4] * 1e3,
            "verdicts_match_gpu": agree,
            "sample": f"C++ restatement over GMP (oracle/cpu_baseline.cpp, dlopen libgmp.so.10): the WHOLE n={n} "
                      f"verification ({P} PDL+Alice pairs, {Mt} ring-Pedersen + correct-key, {J} DLog, {P} Feldman) "
                      f"timed on {threads} threads ({full_s:.1f} s wall), every verdict compared with the GPU's; "
                      f"single-thread figure extrapolated from {s1['pairs']} pairs, {s1['msgs']} RP+CK, "
                      f"{s1['joins']} DLog, {s1['fel']} Feldman"}
