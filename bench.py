#!/usr/bin/env python3
"""Headline benchmark: RefreshMessage::collect() proofs verified per second at
n = 64 (60 refresh + 4 JoinMessage replacements, t = 32, 2048-bit Paillier N,
M = 256) — BASELINE.json configs[2], the configuration the metric is quoted
on; plus the metric's second half, 4096-bit modexp/s/GPU (exponent N,
modulus N^2), and BASELINE configs[4] (many independent t=1 n=3 sessions with
3072-bit keys in one device pass) as an extra object on the same line.

One step = ONE WHOLE collect() call (fsdkr.refresh.collect) on host-resident
messages: packing of the n x n proof instances into the C-ABI SoA buffers,
the host pre-pass + one upload (fsdkr_collect_prepare), the kernel pipeline
(every PDL, Alice range, ring-Pedersen, correct-key and composite-DLog proof
and every Feldman check), verdict readback, first-error mapping, the
paillier_key_vec updates and the share recovery (GPU decryption + pk_vec MSM,
overlapped with the pipeline), on a fresh copy of the LocalKey each step.
With --gpus N (torchrun) each rank verifies a slice of the messages and the
verdict bytes are all-reduced over RCCL (fsdkr.shard.collect).  Inputs are
synthetic, generated on the GPU with a seeded prover (fsdkr.synth)."""
import argparse
import copy
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
# collect() runs about twelve concurrent streams (csrc/collect.cpp stream plan; 12
# hardware queues measured 2-5 % faster than 16, profiles/r02p_hwq.txt); with
# HIP's default of 4 hardware queues per process (exported as 4 on the GPU
# boxes) several of them would share queues and serialise.  Raise it (never
# lower it) before the HIP runtime initialises.
os.environ["GPU_MAX_HW_QUEUES"] = str(max(12, int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)))

import numpy as np  # noqa: E402

METRIC = "collect() proofs verified/sec at n=64, 2048-bit N; 4096-bit modexp/s/GPU"
PEAK_MAC = 3.40e13   # measured v_mad_u64_u32 lane-ops/s, 4 waves/SIMD (profiles/r01_intrates.jsonl)


def w_modexp(k32, ebits):
    """SURVEY §8d algorithmic work: (L + ceil(L/5)) modmuls of 2k^2+k MACs."""
    return (ebits + (ebits + 4) // 5) * (2 * k32 * k32 + k32)


def kernel_issued(kd, g, ebits):
    """v_mad_u64_u32 lane-ops modexp_kernel actually issues for one instance
    (csrc/modexp.hip, mont29.hpp): 29-bit digits, KD x G lanes, 2^w - 1 table
    products + per window w squaring products and one multiply + the exit
    product; a plain product is KD rows x G lanes x 2L MACs, a squaring product
    KD x G x ((L+1)/2 or L/2+1 tournament slots + L reduction MACs)."""
    w = min(range(1, 7), key=lambda x: ebits + (ebits + x - 1) // x + (1 << x))
    nwin = (ebits + w - 1) // w
    L = kd // g
    mul = kd * g * 2 * L
    sqr = kd * g * ((L + 1) // 2 if L % 2 else L // 2 + 1) + kd * g * L
    return ((1 << w) - 1 + (nwin - 1) + 1) * mul + (nwin - 1) * w * sqr


def slide_window(ebits):
    """capi.cpp choose_slide_window: 2^(w-1) odd powers + ebits/(w+1) products, fewest."""
    return min(range(1, 8), key=lambda w: (1 << (w - 1)) + ebits / (w + 1))


def slide_products(e, w):
    """(squarings, multiplies) modexp_slide_kernel runs for exponent e: the odd-power
    table (x*R^2, x^2, 2^(w-1) - 1 products), the window scan from the top bit (the
    first window is a table load) and the exit product."""
    bits = bin(e)[2:][::-1]
    bit = lambda i: bits[i] == "1"
    sq, mul = 1, 1 + (1 << (w - 1)) - 1 + 1
    i = len(bits) - 1
    j = max(i - w + 1, 0)
    while not bit(j):
        j += 1
    i = j - 1
    while i >= 0:
        if not bit(i):
            sq, i = sq + 1, i - 1
            continue
        j = max(i - w + 1, 0)
        while not bit(j):
            j += 1
        sq, mul, i = sq + i - j + 1, mul + 1, j - 1
    return sq, mul


def slide_issued(kd, g, exps):
    """kernel_issued for modexp_slide_kernel, averaged over the launch's exponents."""
    w = slide_window(max(e.bit_length() for e in exps))
    L = kd // g
    mul = kd * g * 2 * L
    sqr = kd * g * ((L + 1) // 2 if L % 2 else L // 2 + 1) + kd * g * L
    tot = [slide_products(e, w) for e in exps]
    return sum(q * sqr + m * mul for q, m in tot) / len(tot)


def proofs_of(R, J, n):
    return 2 * R * n + (R + J) + (R + J) + 2 * J


def collect_work(R, J, n, M=256, k=64):
    """Algorithmic MACs of one collect (SURVEY §8d accounting); k = limbs of N."""
    kk = 2 * k
    b = 32 * k
    s1, s3 = 769, b + 768
    pair = (w_modexp(kk, b) * 2 + w_modexp(kk, 256) * 2 + w_modexp(k, s1) * 2 + w_modexp(k, s3) * 2 +
            w_modexp(k, 256) * 2 + 2 * (2 * kk * kk + kk))
    return R * n * pair + (R + J) * (M * w_modexp(k, b) + 11 * w_modexp(k, b)) + \
        J * 2 * (w_modexp(k, b + 512) + w_modexp(k, 256))


def fb_window(bits):
    """fixedbase.hip fb_window: the BGMW window minimising ceil(bits/w) + 2^w - 1."""
    return min(range(1, 9), key=lambda w: ((bits + w - 1) // w + (1 << w) - 1, w))


def comb_cost(bits, w, avail, per_base):
    """fixedbase_host.cpp comb_choose (no memory cap): products per exponent of
    the cheapest Lim-Lee comb (h, v, b) over a chain with entries every w
    squarings (avail of them per base) and the table products per base, or None
    when BGMW stays (the comb must beat it by 10 %)."""
    if bits < 64 or per_base < 8:
        return None
    wb = fb_window(bits)
    best, best_cost = None, 0.9 * ((bits + wb - 1) // wb + (1 << wb) - 1)
    for h in range(2, 13):
        for v in range(1, 9):
            hv = h * v
            b = -(-bits // hv)
            b = -(-b // w) * w
            if (hv * b + 31) // 32 > 256 or (hv - 1) * (b // w) >= avail:
                continue
            cost = (b - 1) + v * b + v * ((1 << h) - 1 - h) / per_base
            if cost < best_cost:
                best_cost, best = cost, ((b - 1) + v * b, v * ((1 << h) - 1 - h))
    return best


def collect_issued(R, J, n, M=256, k=64):
    """MACs the GPU actually issues per collect: collect_work with the bases
    shared across exponents (h1_i, h2_i per receiver, ring-Pedersen T per
    message) evaluated as fixed-base exponentiations: one squaring chain per base
    (entries every w bits), then per base class either a Lim-Lee comb (comb.hip:
    b - 1 + v b products per exponent plus v (2^h - 1 - h) table products per
    base) or BGMW windowing (ceil(L/w) + 2^w - 1 products per exponent), as
    FbJob::plan_comb / fsdkr_collect_prestart_rp choose.  Reported beside the
    algorithmic figure so the saving is not read as kernel efficiency (SURVEY
    §8d).  k = limbs of N (configs[4]'s prestarted T^Z exponents make the same
    choice: M per base)."""
    mm = 2 * k * k + k
    b = 32 * k
    s1, s3 = 769, b + 768
    w = fb_window(max(s1, s3, b))

    def fb(bits, exps, bases):
        """products of `exps` exponents of up to `bits` bits over `bases` bases"""
        c = comb_cost(bits, w, -(-bits // w), exps / max(bases, 1))
        if c is None:
            return exps * ((bits + w - 1) // w + (1 << w) - 1)
        return exps * c[0] + bases * c[1]

    var = collect_work(R, J, n, M, k)
    var -= R * n * 2 * (w_modexp(k, s1) + w_modexp(k, s3)) + (R + J) * M * w_modexp(k, b)
    fixed = (fb(s1, 2 * R * n, n) + fb(s3, 2 * R * n, n) + fb(b, (R + J) * M, R + J)) * mm
    tables = (n * (s1 + s3) + (R + J) * b) * mm
    return var + fixed + tables


def pmc_per_call(label):
    """SQ_INSTS_VALU_INT64 per whole collect() call from the committed rocprofv3
    --pmc pass (tools/pmc_step.py + tools/pmc_summary_step.py; PMC serialises the
    dispatches, so it cannot run inside the timed region): (count, source)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"*pmc_step_{label}.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    return d["per_call"]["SQ_INSTS_VALU_INT64"], os.path.relpath(files[-1], REPO), d.get("pmc_mac_per_call")


def efficiency(work, issued, seconds, world=1, pmc=None):
    """MAC accounting of a timed step.  algorithmic_mac_per_step is
    the SURVEY work (32-bit limbs, 2k^2+k per modmul, no fixed-base or squaring
    savings): a work count, not a rate against the peak.  issued_model_frac
    models the MACs the kernels issue (collect_issued).  Measured (one committed
    --pmc pass over whole calls at HEAD, tools/pmc_step.py): pmc_issued_frac =
    SQ_INSTS_VALU_INT64 x 64 lanes over the step time and the v_mad_u64_u32 peak
    -- every 64-bit integer VALU instruction, i.e. the MACs AND the rows' 64-bit
    carry shifts / adds; pmc_mac_frac counts only the v_mad_u64_u32 MACs: each
    kernel's INT64 count times its MAC share from the disassembly of the same
    build (tools/mac_share.py: the smallest share over its product cycle loops,
    rolling-normalisation folds excluded)."""
    out = {"algorithmic_mac_per_step": work,
           "issued_model_mac_per_step": issued, "issued_model_frac": issued / seconds / PEAK_MAC / world}
    if pmc:
        out["pmc_int64_lane_ops_per_step"] = pmc[0] * 64
        out["pmc_issued_frac"] = pmc[0] * 64 / seconds / PEAK_MAC / world
        if pmc[2]:
            out["pmc_mac_lane_ops_per_step"] = pmc[2] * 64
            out["pmc_mac_frac"] = pmc[2] * 64 / seconds / PEAK_MAC / world
        out["pmc_source"] = pmc[1]
    return out


def cpu_baseline(batch, verdict_ref, proofs, threads, seconds_budget=12.0):
    """The C++ restatement of collect()'s verification over GMP (oracle/cpu_baseline.cpp,
    dlopen libgmp.so.10: the reference's own bignum engine) on this host over the
    SAME packed workload: the whole verification timed on `threads` threads
    (about 7 s at n = 64), every verdict checked against the GPU's; the
    single-thread figure is extrapolated from a bounded sample."""
    from oracle import cpu_baseline as cb
    out = cb.measure(batch, verdict_ref, threads=threads, budget_s=seconds_budget)
    out["value"] = proofs / out["collect_s"]
    if out.get("all_cores"):
        out["all_cores"]["value"] = proofs / out["all_cores"]["collect_s"]
    out["single_thread_value"] = proofs / out["single_thread_collect_s"]
    out["unit"] = "proofs/s"
    out["kind"] = "port"
    return out


def cpu_baseline_python(msgs, joins, lk, n_pairs):
    """Fallback when the C++ baseline is not built: the Python oracle, 1 thread."""
    from oracle import range_proofs, ring_pedersen
    from oracle import secp256k1 as ec
    from oracle import zk_pdl_with_slack as pdl
    from oracle.zk_paillier import NiCorrectKeyProof
    R, J = len(msgs), len(joins)
    n = R + J
    t_pair = 0.0
    done = 0
    for k in range(R):
        for i in range(n):
            m = msgs[k]
            st = pdl.PDLwSlackStatement(m.points_encrypted_vec[i], lk.paillier_key_vec[i], m.points_committed_vec[i],
                                        ec.G, lk.h1_h2_n_tilde_vec[i].g, lk.h1_h2_n_tilde_vec[i].ni,
                                        lk.h1_h2_n_tilde_vec[i].N)
            a = time.perf_counter()
            pdl.verify(m.pdl_proof_vec[i], st)
            assert range_proofs.verify(m.range_proofs[i], st.ciphertext, st.ek, lk.h1_h2_n_tilde_vec[i])
            t_pair += time.perf_counter() - a
            done += 1
            if done >= n_pairs:
                break
        if done >= n_pairs:
            break
    m = msgs[0]
    a = time.perf_counter()
    assert ring_pedersen.verify(m.ring_pedersen_proof, m.ring_pedersen_statement, 256)
    t_rp = time.perf_counter() - a
    a = time.perf_counter()
    assert NiCorrectKeyProof(m.dk_correctness_proof.sigma_vec).verify(m.ek.n)
    t_ck = time.perf_counter() - a
    t_collect = R * n * t_pair / done + (R + J) * (t_rp + t_ck)
    return {"value": proofs_of(R, J, n) / t_collect, "unit": "proofs/s", "cores": 1, "kind": "port",
            "sample": f"Python oracle (GMP mpz_powm via ctypes), 1 thread: {done} PDL+Alice pairs, 1 ring-Pedersen, "
                      f"1 correct-key; extrapolated to the n={n} proof mix (C++ baseline not built)"}


def keygen_bench(ctx, count=64, bits=2048, seed=77):
    """`count` Paillier keypairs + NiCorrectKeyProof in one batched
    call (fsdkr.keygen.refresh_keys: GPU Miller-Rabin prime walks, one modexp
    launch for the proofs), and one keypair alone (the distribute() path)."""
    import random
    from fsdkr import keygen

    class _Seeded:   # synthetic draws (bench only); production uses the OS RNG
        def __init__(self, s):
            self.r = random.Random(s)

        def bits(self, k):
            return self.r.getrandbits(k)

    keygen.refresh_keys(ctx, _Seeded(seed), bits, 2)   # warm-up
    t0 = time.perf_counter()
    keys = keygen.refresh_keys(ctx, _Seeded(seed + 1), bits, count)
    batch_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    keygen.keypair_with_modulus_size(ctx, _Seeded(seed + 2), bits)
    single_s = time.perf_counter() - t0
    assert all(ek.n.bit_length() == bits for ek, _, _ in keys)
    return {"bits": bits, "keys": count, "keys_per_s": count / batch_s, "batch_ms": batch_s * 1e3,
            "single_keypair_ms": single_s * 1e3,
            "what": "keypairs + correct-key proofs per batched call; single = one keypair (distribute path)"}


def modexp_roofline(ctx, count, reps, seed=1234, keyed=True):
    """The dominant kernel on the metric-2 shape: base^N mod N^2, N 2048-bit.
    keyed: fsdkr_modexp_keyed_device (exponent N per key, waves regrouped by key,
    sliding windows: modexp_slide_kernel); else fsdkr_modexp_batch_device with a
    per-instance exponent row (fixed windows: modexp_kernel)."""
    import random
    import torch
    from fsdkr._native import ints_to_limbs
    rnd = random.Random(seed)
    nmod = 16
    Ns = [rnd.getrandbits(2048) | 1 | (1 << 2047) for _ in range(nmod)]
    mods = [x * x for x in Ns]
    idx = (np.arange(count) % nmod).astype(np.uint32)
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 2 ** 32, size=(count, 128), dtype=np.uint64).astype(np.uint32)
    base[:, -1] >>= 1
    E = ints_to_limbs(Ns if keyed else [Ns[i] for i in idx], 64)
    Mo = ints_to_limbs(mods, 128)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_b = torch.from_numpy(base.view(np.int32)).to(dev)
    d_e = torch.from_numpy(E.view(np.int32)).to(dev)
    d_i = torch.from_numpy(idx.view(np.int32)).to(dev)
    d_m = torch.from_numpy(Mo.view(np.int32)).to(dev)
    d_o = torch.empty((count, 128), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    L = ctx._lib

    fn = L.fsdkr_modexp_keyed_device if keyed else L.fsdkr_modexp_batch_device

    def once():
        ctx.check(fn(ctx.handle, 128, count, d_b.data_ptr(), d_e.data_ptr(), 64, 2048, d_i.data_ptr(), d_m.data_ptr(),
                     nmod, d_o.data_ptr()))
    once()
    ctx.set_timing(True)
    ctx.kernel_time_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    wall = (time.perf_counter() - t0) / reps
    ms, nl = ctx.kernel_time("modexp")
    ctx.set_timing(False)
    ms /= max(nl, 1)
    out = d_o.cpu().numpy().view(np.uint32)
    for i in range(0, count, count // 4):
        b = int.from_bytes(base[i].tobytes(), "little")
        assert int.from_bytes(out[i].tobytes(), "little") == pow(b, Ns[idx[i]], mods[idx[i]]), "modexp parity"
    W = count * w_modexp(128, 2048)
    cap = 256 * 4 * 3 * 64   # modexp.hip pick_group / capi.cpp run_modexp_keyed for 128 limbs
    g = 16 if count * 16 <= cap else 8 if count * 8 <= cap else 4
    issued = slide_issued(144, g, Ns) if keyed else kernel_issued(144, g, 2048)
    return {"count": count, "kernel_ms": ms, "wall_ms": wall * 1e3, "modexp_per_s": count / (ms * 1e-3),
            "achieved_mac_per_s": W / (ms * 1e-3), "group": g, "keyed": keyed,
            "issued_mac_per_s": count * issued / (ms * 1e-3)}


def pmc_traffic(count, pattern="r*_pmc_modexp4096_keyed.json"):
    """Bytes past L2 per launch of the roofline kernel from the committed rocprofv3
    --pmc passes (tools/pmc.sh + tools/pmc_summary.py: FETCH_SIZE x2 per the
    gfx950 correction + WRITE_SIZE, one pass each), scaled to `count`
    instances, and the pass's L2 hit rate.  FETCH_SIZE / WRITE_SIZE count the
    L2's fabric requests, Infinity-Cache (MALL) hits included
    (MI355X_MICROARCH.md, HBM section), so this bounds HBM traffic from above.
    The newest round's file wins.  PMC cannot be collected inside the timed run."""
    import glob
    import re
    files = glob.glob(os.path.join(REPO, "profiles", "**", pattern), recursive=True)
    if not files:
        return None, None, None
    rnd = lambda f: int(re.search(r"r(\d+)", os.path.basename(f)).group(1))   # noqa: E731
    f = max(files, key=lambda f: (rnd(f), os.path.basename(f)))
    d = json.load(open(f))
    inst = d.get("instances", 65536)   # tools/pmc.sh's --count (files before round 6 did not record it)
    return d["hbm_traffic_bytes"] * count / inst, os.path.relpath(f, REPO), d.get("l2_hit_rate")


def _phases_once(ctx, msgs, lk, joins, key_bits):
    """One instrumented collect, in refresh.collect's order: where the host time
    of a step goes (stage-1 pack, GA prestart, stage-2 pack overlapping the
    prestarted chains, prepare, pipeline launch, share-recovery launch (its host
    pre-pass overlaps the pipeline), finish wait, recovery finish, first error)."""
    from fsdkr.batch import CollectBatch
    from fsdkr.refresh import _speculative_finish, _speculative_launch, prestart
    t0 = time.perf_counter()
    b = CollectBatch(msgs, lk, joins, 256, key_bits, staged=True)
    ts = time.perf_counter()
    prestart(ctx, b)
    tp = time.perf_counter()
    b.complete()
    t1 = time.perf_counter()
    ctx.collect_prepare(b)
    t2 = time.perf_counter()
    ctx.collect_launch()
    t3 = time.perf_counter()
    pend = _speculative_launch(ctx, [(msgs, lk, len(msgs) + len(joins))])
    tr = time.perf_counter()
    v = ctx.collect_finish(b)
    t4 = time.perf_counter()
    span = ctx.collect_last_span_ms()
    _speculative_finish(ctx, pend)
    t45 = time.perf_counter()
    b.first_error(v)
    t5 = time.perf_counter()
    # the device pipeline alone on the prepared batch (no host work, and no
    # prestart: GA runs inside it from a cold start)
    ctx.collect_prepare(b)
    runs = []
    for _ in range(3):
        a = time.perf_counter()
        ctx.collect_run(b)
        runs.append((time.perf_counter() - a) * 1e3)
    return b, v, {"pack_stage1_ms": (ts - t0) * 1e3, "prestart_ms": (tp - ts) * 1e3,
                  "pack_stage2_ms": (t1 - tp) * 1e3, "prepare_ms": (t2 - t1) * 1e3, "launch_ms": (t3 - t2) * 1e3,
                  "recovery_launch_ms": (tr - t3) * 1e3, "finish_wait_ms": (t4 - tr) * 1e3,
                  "recovery_finish_ms": (t45 - t4) * 1e3, "first_error_ms": (t5 - t45) * 1e3,
                  "device_pipeline_ms": min(runs), "call_device_span_ms": span}


def phases(ctx, msgs, lk, joins, key_bits, reps=3):
    """_phases_once `reps` times (a fresh LocalKey each): the median of every
    phase (one instrumented call is one sample of a ~50 ms call)."""
    res = [_phases_once(ctx, msgs, copy.deepcopy(lk), joins, key_bits) for _ in range(reps)]
    ph = {k: float(np.median([r[2][k] for r in res])) for k in res[0][2]}
    ph["samples"] = reps
    return res[-1][0], res[-1][1], ph


def sessions_bench(ctx, count, steps, seed):
    """BASELINE configs[4]: `count` independent t=1 n=3 collect() sessions with
    3072-bit keys, verified in ONE device pass per step (refresh.collect_many:
    packing, one multi-session image, pipeline, per-session first error, key
    updates and share recovery)."""
    from fsdkr import refresh, synth
    tg = time.perf_counter()
    sess = synth.synth_sessions(ctx, count, n=3, t=1, seed=seed, key_bits=3072)
    gen_s = time.perf_counter() - tg
    work = [[(m, copy.deepcopy(lk), dk, j) for (m, j, lk, dk) in sess] for _ in range(steps + 1)]
    res = refresh.collect_many(work[0], ctx=ctx, key_bits=3072)
    assert all(r is None for r in res), "synthetic sessions failed verification"
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        refresh.collect_many(work[s + 1], ctx=ctx, key_bits=3072)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    proofs = count * proofs_of(3, 0, 3)
    return {"workload": f"{count} independent RefreshMessage::collect sessions, t=1 n=3, 3072-bit Paillier "
                        f"(BASELINE configs[4]), one device pass per step", "sessions": count,
            "proofs_per_step": proofs, "steps": steps, "ms_per_step": el * 1e3, "value": proofs / el,
            "unit": "proofs/s", "sessions_per_s": count / el, "workload_gen_s": gen_s,
            "collect_efficiency": efficiency(count * collect_work(3, 0, 3, k=96),
                                             count * collect_issued(3, 0, 3, k=96), el,
                                             pmc=pmc_per_call("c4") if count == 1024 else None),
            "data": "synthetic (seeded GPU prover; keys are distinct products of pairs from a shared prime pool)"}


def config3_bench(ctx, steps, seed, n=256, t=128, dist=None, dev=None):
    """BASELINE configs[3] (the north_star target): RefreshMessage::collect at n = 256,
    t = 128, 2048-bit keys, 65 536 PDL + 65 536 Alice proofs + 256 ring-Pedersen +
    256 correct-key proofs verified in ONE batched pass (the whole collect() call
    per step, as the headline), on n distinct refresh messages from the seeded GPU
    prover (synth.synth_collect).  With a process group (bench.py --gpus N) every
    rank runs shard.collect on its slice of the messages (one verdict all-reduce
    per call) and the step time is the max over ranks."""
    import torch
    from fsdkr import refresh, shard, synth
    world = dist.get_world_size() if dist is not None else 1
    tg = time.perf_counter()
    msgs, joins, lk = synth.synth_collect(ctx, n, 0, t, seed)
    gen_s = time.perf_counter() - tg
    keys = [copy.deepcopy(lk) for _ in range(steps + 1)]

    def call(key):
        if dist is not None:
            shard.collect(dist, msgs, key, lk.paillier_dk, joins, ctx, device=dev)
        else:
            refresh.collect(msgs, key, lk.paillier_dk, joins, ctx=ctx)
    call(keys[0])   # warm-up + correctness gate
    assert keys[0].x_i != lk.x_i and len(keys[0].pk_vec) == n, "collect() did not update the LocalKey"
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        call(keys[s + 1])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = (time.perf_counter() - t0) / steps
    if dist is not None:
        tt = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    proofs = proofs_of(n, 0, n)
    where = "on ONE GPU" if world == 1 else f"sharded by refresh message over {world} GPUs (max over ranks)"
    return {"workload": f"RefreshMessage::collect n={n} t={t}: {n} refresh messages, M=256, 2048-bit N "
                        f"(BASELINE configs[3], the north_star target) {where}; one step = the whole collect() "
                        f"call", "n": n, "t": t, "n_gpus": world, "proofs_per_step": proofs, "steps": steps,
            "ms_per_step": el * 1e3, "value": proofs / el, "unit": "proofs/s", "workload_gen_s": gen_s,
            "collect_efficiency": efficiency(collect_work(n, 0, n), collect_issued(n, 0, n), el, world,
                                             pmc=pmc_per_call("n256") if world == 1 else None),
            "data": f"synthetic (seeded GPU prover fs-dkr_amd/fsdkr/synth.py); {n} distinct refresh messages"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--t", type=int, default=32)
    ap.add_argument("--joins", type=int, default=4)
    ap.add_argument("--key-bits", type=int, default=2048)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--modexp-count", type=int, default=65536)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sessions", type=int, default=1024, help="configs[4] sessions (0: skip)")
    ap.add_argument("--session-steps", type=int, default=2)
    ap.add_argument("--config3-steps", type=int, default=2, help="configs[3] n=256 whole-call steps (0: skip)")
    ap.add_argument("--unique-msgs", type=int, default=0,
                    help="generate U distinct refresh messages and tile them to n (n = 256 run; the verifier "
                         "still checks every pair)")
    ap.add_argument("--emulate-shard", type=int, default=0,
                    help="analysis only: run rank 0's slice of a W-way shard on one GPU and report its step time")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="with --emulate-shard: idle gap before each timed whole-call step (profiling)")
    a = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the multi-rank path on a one-GPU box (FSDKR_BENCH_REHEARSE=1):
    # every rank on device 0, gloo instead of RCCL (which needs one GPU per rank)
    rehearse = os.environ.get("FSDKR_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from fsdkr import Context, refresh, shard, synth
    ctx = Context(device=local)
    R, J, t, n = a.n - a.joins, a.joins, a.t, a.n
    tg = time.perf_counter()
    if a.unique_msgs and a.unique_msgs < R:
        assert J == 0, "--unique-msgs tiles refresh-only batches"
        msgs, joins, lk = synth.synth_collect_tiled(ctx, R, t, a.seed, a.unique_msgs, key_bits=a.key_bits)
    else:
        msgs, joins, lk = synth.synth_collect(ctx, R, J, t, a.seed, key_bits=a.key_bits)
    gen_s = time.perf_counter() - tg
    new_dk = lk.paillier_dk
    dev = torch.device("cuda", local)
    if a.emulate_shard and world == 1:
        # analysis only: rank 0's slice of a W-way shard (verification of the slice)
        from fsdkr.batch import CollectBatch
        r0, r1 = shard.shard_range(R, a.emulate_shard, 0)
        j0, j1 = shard.shard_range(J, a.emulate_shard, 0)
        b = CollectBatch(msgs[r0:r1], lk, joins[j0:j1], 256, a.key_bits, n_recv=n)
        ctx.collect_prepare(b)
        for _ in range(a.warmup):
            ctx.collect_run(b)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ctx.collect_run(b)
        torch.cuda.synchronize()
        dev_ms = (time.perf_counter() - t0) / a.steps * 1e3
        # the whole rank-0 shard.collect() call; the all-reduce is replaced by the
        # all-valid merge of the other ranks (the RCCL exchange itself is one
        # all_reduce of 4n^2+3n bytes, not emulated)
        class _Rank0:
            class ReduceOp:
                MAX = None

            def get_world_size(self):
                return a.emulate_shard

            def get_rank(self):
                return 0

            def all_reduce(self, t, op=None):
                # every other rank's slice all-valid: feldman 1, pdl 7 (u1|u2|u3), range 1, ped 1, ck 1, dlog 3
                P, M = R * n, R + J
                for lo, hi, ok in ((0, P, 1), (P, 2 * P, 7), (2 * P, 3 * P, 1), (3 * P, 3 * P + 2 * M, 1),
                                   (3 * P + 2 * M, 3 * P + 2 * M + J, 3)):
                    t[lo:hi] = ok

        keys = [copy.deepcopy(lk) for _ in range(a.warmup + a.steps)]
        for k in range(a.warmup):
            shard.collect(_Rank0(), msgs, keys[k], new_dk, joins, ctx, key_bits=a.key_bits)
        torch.cuda.synchronize()
        tot, rank_ph = 0.0, {}
        for k in range(a.steps):
            if a.gap_ms:   # idle gap between steps so a kernel trace can be cut per step
                time.sleep(a.gap_ms * 1e-3)
            t0 = time.perf_counter()
            shard.collect(_Rank0(), msgs, keys[a.warmup + k], new_dk, joins, ctx, key_bits=a.key_bits,
                          timings=rank_ph)
            torch.cuda.synchronize()
            tot += time.perf_counter() - t0
        full_ms = tot / a.steps * 1e3
        rank_ph = {k: v / a.steps for k, v in rank_ph.items()}
        span = ctx.collect_last_span_ms() if hasattr(ctx, "collect_last_span_ms") else None
        host = sum(v for k, v in rank_ph.items() if k != "finish_wait_ms")
        print(json.dumps({"emulated_shard": a.emulate_shard, "note": "emulated rank 0 of a W-way shard on one GPU, "
                          "not a scaling curve", "refresh_slice": [r0, r1], "join_slice": [j0, j1],
                          "device_ms_per_step": dev_ms, "rank0_collect_ms_per_step": full_ms,
                          "rank0_phases_ms": rank_ph, "rank0_host_ms": host, "rank0_device_span_ms": span}),
              flush=True)
        return
    keys = [copy.deepcopy(lk) for _ in range(a.warmup + a.steps)]   # a fresh LocalKey per collect()

    def step(k):
        if dist is not None:
            shard.collect(dist, msgs, keys[k], new_dk, joins, ctx, device=dev, key_bits=a.key_bits)
        else:
            refresh.collect(msgs, keys[k], new_dk, joins, ctx=ctx, key_bits=a.key_bits)

    # correctness gate: every synthetic proof verifies (collect() raises otherwise)
    for k in range(a.warmup):
        step(k)
    assert keys[0].x_i != lk.x_i and len(keys[0].pk_vec) == n, "collect() did not update the LocalKey"
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(a.warmup + k)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed / a.steps * 1e3
    proofs = proofs_of(R, J, n)
    value = proofs * a.steps / elapsed
    # configs[3] (n = 256): on one GPU, or sharded over every rank of the group
    c3 = config3_bench(ctx, a.config3_steps, a.seed + 3, dist=dist, dev=dev) if a.config3_steps and n != 256 else None
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    ctx.set_cu_split(0)   # a shard slice may have split the CUs; the single-GPU figures below use the whole chip
    batch, verd, ph = phases(ctx, msgs, lk, joins, a.key_bits)
    roof = modexp_roofline(ctx, a.modexp_count, 3)
    roof_rows = modexp_roofline(ctx, a.modexp_count, 3, keyed=False)
    cpu = None
    if not a.no_cpu_baseline and world == 1:
        try:
            cpu = cpu_baseline(batch, verd, proofs, a.cpu_threads)
        except (ImportError, OSError) as e:
            cpu = cpu_baseline_python(msgs, joins, lk, 200)
            cpu["cpp_unavailable"] = str(e)
    s4 = sessions_bench(ctx, a.sessions, a.session_steps, a.seed + 4) if a.sessions and world == 1 else None
    kg = keygen_bench(ctx) if world == 1 else None
    W_collect = collect_work(R, J, n)
    traffic, traffic_src, l2_hit = pmc_traffic(roof["count"])
    out = {
        "metric": METRIC, "value": value, "unit": "proofs/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32 (radix-2^29 digits, u64 accumulators)",
        "data": "synthetic (seeded GPU prover fs-dkr_amd/fsdkr/synth.py; 2048-bit Paillier/DLog keys)" +
                (f"; {a.unique_msgs} distinct refresh messages tiled to {R}" if a.unique_msgs and a.unique_msgs < R
                 else ""),
        "config": {"workload": f"RefreshMessage::collect n={n} t={t}: {R} refresh + {J} JoinMessage, M=256, "
                               f"{a.key_bits}-bit N (BASELINE configs[{3 if n >= 256 else 2}]); one step = the whole "
                               f"collect() call (pack, pre-pass + upload, pipeline, first error, key updates, "
                               f"share recovery)",
                   "n": n, "t": t, "refresh": R, "joins": J,
                   "proofs_per_step": proofs, "parallelism": f"refresh messages sharded over {world} GPU(s)"},
        "phases_ms": ph,
        "device_pipeline_proofs_per_s": proofs / (ph["device_pipeline_ms"] * 1e-3),
        "modexp_4096_per_s": roof["modexp_per_s"],
        "modexp_4096_per_s_exponent_rows": {
            "value": roof_rows["modexp_per_s"], "kernel_ms": roof_rows["kernel_ms"], "lanes": roof_rows["group"],
            "what": "fsdkr_modexp_batch_device: a per-instance exponent row, fixed 5-bit windows (modexp_kernel)"},
        "roofline": {"bound": "valu-int", "achieved": roof["achieved_mac_per_s"] / 1e12, "peak": PEAK_MAC / 1e12,
                     "unit": "T u32-MAC/s", "frac": roof["achieved_mac_per_s"] / PEAK_MAC, "traffic": traffic,
                     "traffic_unit": "bytes past L2 per launch (PMC FETCH_SIZE x2 + WRITE_SIZE; Infinity-Cache "
                                     "hits included, so an upper bound on HBM bytes)",
                     "traffic_source": traffic_src, "l2_hit_rate": l2_hit,
                     "algorithmic_bytes": roof["count"] * (512 + 256 + 512),
                     "kernel": "modexp_slide_kernel (4096-bit modulus N^2, 2048-bit exponent N shared per key: "
                               "fsdkr_modexp_keyed_device, 16 keys x 4096 instances, sliding windows w = 7)",
                     "per_launch": f"{roof['count']} instances x {w_modexp(128, 2048) / 1e6:.2f} M MACs in "
                                   f"{roof['kernel_ms']:.2f} ms (HIP events)",
                     "accounting": "achieved / frac = SURVEY §8d MACs (32-bit limbs, 2k^2+k per modmul, fixed "
                                   "5-bit windows): an algorithmic-equivalent rate; the kernel runs w = 7 sliding "
                                   "windows and issues fewer products.  issued / issued_frac = the kernel's own "
                                   "v_mad_u64_u32 lane-ops (29-bit digits, squaring rows): the fraction of the "
                                   "int-MAC peak it actually uses",
                     "issued": roof["issued_mac_per_s"] / 1e12, "issued_frac": roof["issued_mac_per_s"] / PEAK_MAC,
                     "lanes_per_instance": roof["group"]},
        "collect_efficiency": efficiency(W_collect, collect_issued(R, J, n), ms_per_step * 1e-3, world,
                                         pmc=pmc_per_call("n64") if (n, J) == (64, 4) else None),
        "config3": c3,
        "config4_sessions": s4,
        "keygen": kg,
        "workload_gen_s": gen_s,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
