#!/usr/bin/env python3
"""Headline benchmark: RefreshMessage::collect() proofs verified per second at
n = 64 (60 refresh + 4 JoinMessage replacements, t = 32, 2048-bit Paillier N,
M = 256) — BASELINE.json configs[2], the configuration the metric is quoted
on; plus the metric's second half, 4096-bit modexp/s/GPU (exponent N,
modulus N^2).

One step = one pass of the batched collect() verification over the
device-resident batch (fsdkr_collect_run: every PDL, Alice range,
ring-Pedersen, correct-key and composite-DLog proof and every Feldman check)
plus verdict readback.  With --gpus N (torchrun) the refresh messages (and
the joins' proofs) are sharded across ranks and the verdict bitmask is
all-reduced over RCCL.  Inputs are synthetic, generated on the GPU with a
seeded prover (fsdkr.synth)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "fs-dkr_amd")]
# collect() runs up to eleven concurrent streams (csrc/collect.cpp stream plan); with
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


def proofs_of(R, J, n):
    return 2 * R * n + (R + J) + (R + J) + 2 * J


def collect_work(R, J, n, M=256):
    """Algorithmic MACs of one collect (SURVEY §8d accounting)."""
    k, kk = 64, 128
    pair = (w_modexp(kk, 2048) * 2 + w_modexp(kk, 256) * 2 + w_modexp(k, 769) * 2 + w_modexp(k, 2816) * 2 +
            w_modexp(k, 256) * 2 + 2 * (2 * kk * kk + kk))
    return R * n * pair + (R + J) * (M * w_modexp(k, 2048) + 11 * w_modexp(k, 2048)) + \
        J * 2 * (w_modexp(k, 2560) + w_modexp(k, 256))


def collect_issued(R, J, n, M=256, w=6):
    """MACs the GPU actually issues per collect: collect_work with the bases
    shared across exponents (h1_i, h2_i per receiver, ring-Pedersen T per
    message) evaluated by fixed-base BGMW windowing (fixedbase.hip): ceil(L/w) +
    2^w - 1 products per exponent plus one L-squaring table chain per base.
    Reported beside the algorithmic figure so the saving is not read as kernel
    efficiency."""
    k = 64
    mm = 2 * k * k + k

    def fb(bits):
        return ((bits + w - 1) // w + (1 << w) - 1) * mm

    var = collect_work(R, J, n, M)
    var -= R * n * 2 * (w_modexp(k, 769) + w_modexp(k, 2816)) + (R + J) * M * w_modexp(k, 2048)
    fixed = R * n * 2 * (fb(769) + fb(2816)) + (R + J) * M * fb(2048)
    tables = (n * (769 + 2816) + (R + J) * 2048) * mm
    return var + fixed + tables


def cpu_baseline(msgs, joins, lk, key_bits, n_pairs, seconds_budget=20.0):
    """Oracle restatement (bigint via GMP, the reference's own engine), ONE thread,
    on a bounded sample of the same workload; extrapolated to the n=64 proof mix."""
    from oracle import range_proofs, ring_pedersen
    from oracle import secp256k1 as ec
    from oracle import zk_pdl_with_slack as pdl
    from oracle.vss import VerifiableSS
    from oracle.zk_paillier import CompositeDLogProof, DLogStatement, NiCorrectKeyProof
    R, J = len(msgs), len(joins)
    n = R + J
    t_pair = t_rp = t_ck = t_dl = t_fel = 0.0
    done_pairs = 0
    t0 = time.perf_counter()
    for k in range(R):
        for i in range(n):
            m = msgs[k]
            st = pdl.PDLwSlackStatement(m.points_encrypted_vec[i], lk.paillier_key_vec[i], m.points_committed_vec[i],
                                        ec.G, lk.h1_h2_n_tilde_vec[i].g, lk.h1_h2_n_tilde_vec[i].ni,
                                        lk.h1_h2_n_tilde_vec[i].N)
            a = time.perf_counter()
            pdl.verify(m.pdl_proof_vec[i], st)
            ok = range_proofs.verify(m.range_proofs[i], st.ciphertext, st.ek, lk.h1_h2_n_tilde_vec[i])
            t_pair += time.perf_counter() - a
            assert ok
            done_pairs += 1
            if done_pairs >= n_pairs:
                break
        if done_pairs >= n_pairs:
            break
    m = msgs[0]
    a = time.perf_counter()
    assert ring_pedersen.verify(m.ring_pedersen_proof, m.ring_pedersen_statement, 256)
    t_rp = time.perf_counter() - a
    a = time.perf_counter()
    assert NiCorrectKeyProof(m.dk_correctness_proof.sigma_vec).verify(m.ek.n)
    t_ck = time.perf_counter() - a
    vss = VerifiableSS(lk.t, n, list(m.coefficients_committed_vec.commitments))
    a = time.perf_counter()
    for i in range(min(n, 8)):
        assert vss.validate_share_public(m.points_committed_vec[i], i + 1)
    t_fel = (time.perf_counter() - a) / min(n, 8)
    if J:
        j = joins[0]
        st = DLogStatement(j.dlog_statement.N, j.dlog_statement.g, j.dlog_statement.ni)
        a = time.perf_counter()
        assert CompositeDLogProof(j.composite_dlog_proof_base_h1.x, j.composite_dlog_proof_base_h1.y).verify(st)
        t_dl = time.perf_counter() - a
    total = time.perf_counter() - t0
    per_pair = t_pair / done_pairs
    t_collect = R * n * (per_pair + t_fel) + (R + J) * (t_rp + t_ck) + 2 * J * t_dl
    return {"value": proofs_of(R, J, n) / t_collect, "unit": "proofs/s", "cores": 1, "kind": "port",
            "sample": f"oracle (GMP mpz_powm via ctypes), 1 thread: {done_pairs} PDL+Alice pairs, 1 ring-Pedersen,"
                      f" 1 correct-key, {1 if J else 0} composite-DLog, {min(n, 8)} Feldman checks of the bench"
                      f" workload ({total:.1f} s); extrapolated to the n={n} proof mix",
            "per_pair_ms": per_pair * 1e3, "per_ring_pedersen_ms": t_rp * 1e3, "per_correct_key_ms": t_ck * 1e3,
            "collect_s": t_collect}


def modexp_roofline(ctx, count, reps, seed=1234):
    """The dominant kernel on the metric-2 shape: base^N mod N^2, N 2048-bit."""
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
    E = ints_to_limbs([Ns[i] for i in idx], 64)
    Mo = ints_to_limbs(mods, 128)
    dev = torch.device("cuda", torch.cuda.current_device())
    d_b = torch.from_numpy(base.view(np.int32)).to(dev)
    d_e = torch.from_numpy(E.view(np.int32)).to(dev)
    d_i = torch.from_numpy(idx.view(np.int32)).to(dev)
    d_m = torch.from_numpy(Mo.view(np.int32)).to(dev)
    d_o = torch.empty((count, 128), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    L = ctx._lib

    def once():
        ctx.check(L.fsdkr_modexp_batch_device(ctx.handle, 128, count, d_b.data_ptr(), d_e.data_ptr(), 64, 2048,
                                              d_i.data_ptr(), d_m.data_ptr(), nmod, d_o.data_ptr()))
    once()
    ctx.kernel_time_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    wall = (time.perf_counter() - t0) / reps
    ms, nl = ctx.kernel_time("modexp")
    ms /= max(nl, 1)
    out = d_o.cpu().numpy().view(np.uint32)
    for i in range(0, count, count // 4):
        b = int.from_bytes(base[i].tobytes(), "little")
        assert int.from_bytes(out[i].tobytes(), "little") == pow(b, Ns[idx[i]], mods[idx[i]]), "modexp parity"
    W = count * w_modexp(128, 2048)
    return {"count": count, "kernel_ms": ms, "wall_ms": wall * 1e3, "modexp_per_s": count / (ms * 1e-3),
            "achieved_mac_per_s": W / (ms * 1e-3)}


def pmc_traffic(count):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3
    --pmc passes (tools/pmc.sh + tools/pmc_summary.py: FETCH_SIZE x2 per the
    gfx950 correction + WRITE_SIZE, one pass each), scaled to `count`
    instances.  PMC cannot be collected inside the timed run."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_modexp4096.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    inst = d.get("instances", 65536)
    return d["hbm_traffic_bytes"] * count / inst, os.path.relpath(files[-1], REPO)


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
    ap.add_argument("--cpu-pairs", type=int, default=400)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--unique-msgs", type=int, default=0,
                    help="generate U distinct refresh messages and tile them to n (n = 256 run; the verifier "
                         "still checks every pair)")
    ap.add_argument("--emulate-shard", type=int, default=0,
                    help="analysis only: run rank 0's slice of a W-way shard on one GPU and report its step time")
    a = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from fsdkr import Context, synth
    from fsdkr.batch import CollectBatch
    ctx = Context(device=local, timing=True)
    R, J, t, n = a.n - a.joins, a.joins, a.t, a.n
    tg = time.perf_counter()
    if a.unique_msgs and a.unique_msgs < R:
        assert J == 0, "--unique-msgs tiles refresh-only batches"
        msgs, joins, lk = synth.synth_collect_tiled(ctx, R, t, a.seed, a.unique_msgs, key_bits=a.key_bits)
    else:
        msgs, joins, lk = synth.synth_collect(ctx, R, J, t, a.seed, key_bits=a.key_bits)
    gen_s = time.perf_counter() - tg
    # shard: contiguous slices of the refresh messages and of the joins (fsdkr.shard)
    from fsdkr import shard
    sw = a.emulate_shard if (a.emulate_shard and world == 1) else world
    r0, r1 = shard.shard_range(R, sw, rank)
    j0, j1 = shard.shard_range(J, sw, rank)
    batch = CollectBatch(msgs[r0:r1], lk, joins[j0:j1], 256, a.key_bits, n_recv=n)
    ctx.collect_prepare(batch)
    P = R * n
    dev = torch.device("cuda", local)

    def step():
        v = ctx.collect_run(batch)
        if dist is not None:
            return shard.MergedVerdicts(shard.merge(dist, shard.scatter(v, R, J, n, world, rank), dev), R, J, n)
        return v

    # per-kernel HIP events cost ~9 ms per collect (tools/ab_collect.py --timing):
    # the timed region runs without them; one extra step afterwards is timed per kernel
    ctx.set_timing(False)
    for _ in range(a.warmup):
        res = step()
    if sw != world:       # emulated shard: verdicts cover only this slice; report its step time
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        print(json.dumps({"emulated_shard": sw, "refresh_slice": [r0, r1], "join_slice": [j0, j1],
                          "ms_per_step": (time.perf_counter() - t0) / a.steps * 1e3}), flush=True)
        return
    # correctness gate: every synthetic proof verifies
    assert res.feldman[:P].all() and (res.pdl[:P] == 7).all() and res.range[:P].all() and \
        (res.ped[:R + J] == 1).all() and res.ck[:R + J].all() and (res.dlog[:J] == 3).all(), \
        "synthetic workload failed verification"
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ctx.set_timing(True)
    ctx.kernel_time_reset()
    step()
    torch.cuda.synchronize()
    mx_ms, mx_n = ctx.kernel_time("modexp")
    ms_per_step = elapsed / a.steps * 1e3
    proofs = proofs_of(R, J, n)
    value = proofs * a.steps / elapsed
    # full-call (PCIe-inclusive) rate: prepare + run, single measurement
    tp = time.perf_counter()
    ctx.collect_prepare(batch)
    ctx.collect_run(batch)
    full_ms = (time.perf_counter() - tp) * 1e3
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    roof = modexp_roofline(ctx, a.modexp_count, 3)
    cpu = None if a.no_cpu_baseline or world > 1 else cpu_baseline(msgs, joins, lk, a.key_bits, a.cpu_pairs)
    W_collect = collect_work(R, J, n)
    traffic, traffic_src = pmc_traffic(roof["count"])
    out = {
        "metric": METRIC, "value": value, "unit": "proofs/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32 (radix-2^29 digits, u64 accumulators)",
        "data": "synthetic (seeded GPU prover fs-dkr_amd/fsdkr/synth.py; 2048-bit Paillier/DLog keys)" +
                (f"; {a.unique_msgs} distinct refresh messages tiled to {R}" if a.unique_msgs and a.unique_msgs < R
                 else ""),
        "config": {"workload": f"RefreshMessage::collect n={n} t={t}: {R} refresh + {J} JoinMessage, M=256, "
                               f"{a.key_bits}-bit N (BASELINE configs[{3 if n >= 256 else 2}])",
                   "n": n, "t": t, "refresh": R, "joins": J,
                   "proofs_per_step": proofs, "parallelism": f"refresh messages sharded over {world} GPU(s)"},
        "modexp_4096_per_s": roof["modexp_per_s"],
        "roofline": {"bound": "valu-int", "achieved": roof["achieved_mac_per_s"] / 1e12, "peak": PEAK_MAC / 1e12,
                     "unit": "T u32-MAC/s", "frac": roof["achieved_mac_per_s"] / PEAK_MAC, "traffic": traffic,
                     "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": traffic_src,
                     "algorithmic_bytes": roof["count"] * (512 + 256 + 512),
                     "kernel": "modexp_kernel<144,8,128> (4096-bit modulus N^2, 2048-bit exponent N)",
                     "per_launch": f"{roof['count']} instances x {w_modexp(128, 2048) / 1e6:.2f} M MACs in "
                                   f"{roof['kernel_ms']:.2f} ms (HIP events)"},
        "collect_efficiency": {"algorithmic_mac_per_step": W_collect,
                               "frac_of_peak": W_collect / (ms_per_step * 1e-3) / PEAK_MAC / world,
                               "issued_mac_per_step": collect_issued(R, J, n),
                               "issued_frac_of_peak": collect_issued(R, J, n) / (ms_per_step * 1e-3) / PEAK_MAC
                               / world},
        "modexp_kernel_ms_per_step": mx_ms,   # summed over streams, one extra step with HIP events on
        "full_call_pcie_inclusive_ms": full_ms, "workload_gen_s": gen_s,
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
