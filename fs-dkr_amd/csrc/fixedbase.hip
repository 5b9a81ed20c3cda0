// Fixed-base exponentiation on gfx950 for the bases collect() shares across
// many exponents (Brickell-Gordon-McCurley-Wilson windowing):
//   h1_i, h2_i   receiver i's DLogStatement bases, shared by the 2n PDL/Alice
//                proofs addressed to i   (zk_pdl_with_slack.rs:144-157 via
//                commitment_unknown_order :170-188; range_proofs.rs:129-137)
//   T            one ring-Pedersen statement, shared by its M = 256 checks
//                T^Z_i mod N             (ring_pedersen_proof.rs:144)
// Results are bit-identical to base^exp mod N; only the order of the
// Montgomery products changes.
//
// Per base b, fb_table_kernel stores P_j = b^(2^(w j)) (Montgomery form) for
// j < h: a chain of w*h squarings, run once per base.  For an exponent with
// w-bit digits e_j, b^e = prod_{d=2^w-1..1} B_d with B_d = prod_{e_j >= d} P_j;
// fb_exp_kernel keeps B in registers and A in LDS and executes the
// instance's schedule (fb_sched_kernel): "B <- B*P_j" for every j with e_j = d,
// then "A <- A*B", for d from the largest digit down to 1.  That is
// nnz(e) + max(e_j) <= h + 2^w - 1 products per exponent instead of the
// ~bits*(1 + 1/w) of a variable-base window ladder (2048-bit exponent, w = 6:
// 405 vs 2458).
#include "fixedbase.h"
#include "mont29.hpp"

namespace fsdkr {

constexpr uint16_t FB_A_STEP = 0xFFFF;   // A <- A * B
constexpr uint16_t FB_NOP = 0xFFFE;      // idle lanes of a wave still multiply (lockstep); result dropped

// P_j = base^(2^(w j)) in Montgomery form, table[toff[b] + j][KD] in digit order.
template <int KD, int G, int K32>
__global__ __launch_bounds__(BLOCK) void fb_table_kernel(const FbTableArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t b = blockIdx.x * (blockDim.x / G) + li;   // few bases: one wave per block
  if (b >= a.count) return;
  // the table chain heads the fixed-base pipeline (the h2 chain is 2816
  // squarings long, as long as the 4096-bit s^N chains): few waves, top priority
  if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  uint32_t* stream = lds + li * KD;
  const uint32_t* C = a.consts + (size_t)a.mod_idx[b] * STRIDE;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = C[g * L + j];
  M.ninv = C[3 * KD];
  uint32_t acc[L];
  const uint32_t* B = reinterpret_cast<const uint32_t*>(a.base_ptr[b]);
  const int blen = (int)min(a.base_len[b], (uint32_t)K32);
#pragma unroll
  for (int j = 0; j < L; ++j) acc[j] = digit_of(B, blen, g * L + j);
  uint32_t* T = a.table + (size_t)a.toff[b] * KD;
  const uint32_t h = a.h[b];
  // step 0: acc * R^2 -> Montgomery form of the base; then w squarings per entry
  const uint32_t n_steps = 1 + (h > 0 ? (h - 1) * a.w : 0);
  uint32_t entry = 0;
  for (uint32_t st = 0; st < n_steps; ++st) {
    __builtin_amdgcn_wave_barrier();
    if (st == 0) {
#pragma unroll
      for (int j = 0; j < L; ++j) stream[g * L + j] = C[2 * KD + g * L + j];
    } else {
#pragma unroll
      for (int j = 0; j < L; ++j) stream[g * L + j] = acc[j];
    }
    __builtin_amdgcn_wave_barrier();
    if (st == 0) M.mul(acc, acc, stream);
    else M.sqr(acc, acc, stream);
    if (st == 0 || (st % a.w) == 0) {
#pragma unroll
      for (int j = 0; j < L; ++j) T[(size_t)entry * KD + g * L + j] = acc[j];
      ++entry;
    }
  }
}

// The same chain with one base per wave64 (Mont29 wave shape, product_w): lane g
// holds digits gL..gL+L-1, KR digits in the first KR/L lanes; the row digit and
// the quotient are wave-uniform (v_readlane, scalar-unit quotient).  For launches
// of at most one wave per SIMD, where the chain's latency is the critical path.
template <int KR, int L, int K32>
__global__ __launch_bounds__(64) void fb_table_wave_kernel(const FbTableArgs a) {
  constexpr int KD = 64 * L;
  using MT = Mont29<KD, 64, KR>;
  constexpr int STRIDE = cons_stride(KR);
  const int g = threadIdx.x;
  const uint32_t b = blockIdx.x;
  if (b >= a.count) return;
  if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  const uint32_t* C = a.consts + (size_t)a.mod_idx[b] * STRIDE;
  const bool live = g * L < KR;
  MT M;
  M.init_lane(g);
  uint32_t acc[L], r2[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    M.n[j] = live ? C[g * L + j] : 0u;
    r2[j] = live ? C[2 * KR + g * L + j] : 0u;
  }
  M.ninv = (uint32_t)__builtin_amdgcn_readfirstlane((int)C[3 * KR]);
  const uint32_t* B = reinterpret_cast<const uint32_t*>(a.base_ptr[b]);
  const int blen = (int)min(a.base_len[b], (uint32_t)K32);
#pragma unroll
  for (int j = 0; j < L; ++j) acc[j] = digit_of(B, blen, g * L + j);   // 0 past the class's digits
  uint32_t* T = a.table + (size_t)a.toff[b] * KR;
  const uint32_t h = a.h[b];
  const uint32_t n_steps = 1 + (h > 0 ? (h - 1) * a.w : 0);
  uint32_t entry = 0;
  for (uint32_t st = 0; st < n_steps; ++st) {
    if (st == 0) M.mul_w(acc, acc, r2);   // Montgomery form of the base
    else M.sqr_w(acc, acc);
    if (st == 0 || (st % a.w) == 0) {
      if (live) {
#pragma unroll
        for (int j = 0; j < L; ++j) T[(size_t)entry * KR + g * L + j] = acc[j];
      }
      ++entry;
    }
  }
}

// One wave64 per instance: the BGMW product schedule of its exponent, by a
// counting sort of its w-bit digits (O(h + 2^w)): for d = max digit .. 1 the
// windows j with e_j = d in ascending j, then one A-step.  The lanes read the
// exponent's digits coalesced (lane l: windows l, l + 64, ...) and count them
// with LDS atomics; the 2^w bins are scanned across the wave; then one uniform
// pass over the windows (scalar digit reads) appends window j to its digit's
// group, the lane owning bin d holding that group's cursor in a register, so
// every group lists its windows in ascending order (a deterministic schedule;
// an LDS-atomic scatter gives the same residues in any order).  Round 2
// ran one thread per instance (uncoalesced digit reads, 2-byte scatters over
// 64 rows per wave, 32 KB of LDS per 64 instances): ~110 ms ahead of the
// configs[4] fixed-base exponents.
constexpr int FB_SCHED_IPB = 4;   // instances (waves) per block
constexpr int FB_MAX_W = 8;
__global__ __launch_bounds__(64 * FB_SCHED_IPB) void fb_sched_kernel(const FbSchedArgs a) {
  __shared__ uint32_t cnt_lds[FB_SCHED_IPB][1 << FB_MAX_W];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t i = blockIdx.x * FB_SCHED_IPB + wv;   // wave-uniform
  if (i >= a.count) return;
  // no issue-priority raise: at s_setprio 3 this kernel ended in 0.9 ms, the
  // n = 64 fixed-base exponents then started ~8 ms earlier beside the prestarted
  // GA chains, and GA's last chain ended 14 ms later (whole call 53 -> 61 ms,
  // profiles/r03zc_*); at the default priority it runs beside GA in ~7 ms
  const uint32_t* E = reinterpret_cast<const uint32_t*>(a.exp_ptr[i]);
  const uint32_t elen = a.exp_len[i];
  const uint32_t h = a.h[i], w = a.w, nd = 1u << w, mask = nd - 1;
  uint32_t* cnt = cnt_lds[wv];
  auto digit = [&](uint32_t j) -> uint32_t {
    const uint32_t p = j * w, lo = p >> 5, sh = p & 31;
    const uint32_t v0 = (lo < elen) ? E[lo] : 0u;
    const uint32_t v1 = (lo + 1 < elen) ? E[lo + 1] : 0u;
    return (uint32_t)((((uint64_t)v1 << 32) | v0) >> sh) & mask;
  };
  for (uint32_t d = lane; d < nd; d += 64) cnt[d] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  uint32_t dmax = 0;
  for (uint32_t j = lane; j < h; j += 64) {
    const uint32_t d = digit(j);
    if (d) atomicAdd(&cnt[d], 1u);
    dmax = max(dmax, d);
  }
  for (int off = 32; off > 0; off >>= 1) dmax = max(dmax, (uint32_t)__shfl_xor((int)dmax, off));
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // start of digit d's group: sum over d' in (d, dmax] of (cnt[d'] + 1), one A-step
  // slot closing every group (empty ones too: A <- A * B once per digit value)
  uint16_t* S = a.sched + (size_t)i * a.stride;
  uint32_t base = 0;
  for (uint32_t top = dmax; top >= 1;) {   // 64 digit values per pass, descending
    const uint32_t d = top >= lane ? top - lane : 0u;
    const uint32_t c = d ? cnt[d] : 0u;
    const uint32_t v = d ? c + 1 : 0u;
    uint32_t incl = v;
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t u = (uint32_t)__shfl_up((int)incl, off);
      if (lane >= (uint32_t)off) incl += u;
    }
    if (d) {
      const uint32_t start = base + incl - v;
      S[start + c] = FB_A_STEP;
      cnt[d] = start;   // becomes the group's write cursor
    }
    base += (uint32_t)__shfl((int)incl, 63);
    top = top > 64 ? top - 64 : 0u;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // ordered scatter: lane l owns bins l, l + 64, l + 128, l + 192
  uint32_t cur[(1 << FB_MAX_W) / 64];
#pragma unroll
  for (int k = 0; k < (1 << FB_MAX_W) / 64; ++k) {
    const uint32_t d = lane + 64u * k;
    cur[k] = d < nd ? cnt[d] : 0u;
  }
  const uint32_t* Es = reinterpret_cast<const uint32_t*>(
      ((uint64_t)__builtin_amdgcn_readfirstlane((int)(a.exp_ptr[i] >> 32)) << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a.exp_ptr[i]));
  const uint32_t hs = (uint32_t)__builtin_amdgcn_readfirstlane((int)h);
  const uint32_t els = (uint32_t)__builtin_amdgcn_readfirstlane((int)elen);
  for (uint32_t j = 0; j < hs; ++j) {   // wave-uniform loop and digit
    const uint32_t p = j * w, lo = p >> 5, sh = p & 31;
    const uint32_t v0 = (lo < els) ? Es[lo] : 0u;
    const uint32_t v1 = (lo + 1 < els) ? Es[lo + 1] : 0u;
    const uint32_t d = (uint32_t)((((uint64_t)v1 << 32) | v0) >> sh) & mask;
    if (d && (d & 63u) == lane) {
#pragma unroll
      for (int k = 0; k < (1 << FB_MAX_W) / 64; ++k)
        if ((d >> 6) == (uint32_t)k) S[cur[k]++] = (uint16_t)j;
    }
  }
  if (lane == 0) a.nsteps[i] = base;
}

template <int KD, int G, int K32>
__global__ __launch_bounds__(BLOCK) void fb_exp_kernel(const FbExpArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  __shared__ uint32_t lds[2 * IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * (blockDim.x / G) + li;
  if (inst >= a.count) return;
  uint32_t* stream = lds + li * KD;             // streamed operand of each product
  uint32_t* abuf = lds + (IPB + li) * KD;       // accumulator A
  const uint32_t* C = a.consts + (size_t)a.mod_idx[inst] * STRIDE;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = C[g * L + j];
  M.ninv = C[3 * KD];
  const uint32_t toff = a.toff[inst];
  const uint32_t* T = (toff < a.split) ? a.table_pre + (size_t)toff * KD : a.table + (size_t)(toff - a.split) * KD;
  const uint16_t* S = a.sched + (size_t)inst * a.stride;
  const uint32_t nst = a.nsteps[inst];
  uint32_t Bd[L], r[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    Bd[j] = C[KD + g * L + j];                   // B = A = 1 (R mod N)
    abuf[g * L + j] = Bd[j];
  }
  for (uint32_t st = 0;; ++st) {
    // the wave runs until its longest schedule ends (all lanes stay in lockstep: DPP)
    if (__builtin_amdgcn_ballot_w64(st < nst) == 0) break;
    const uint32_t code = (st < nst) ? S[st] : FB_NOP;
    const bool bstep = code < 0xFFFEu;
    __builtin_amdgcn_wave_barrier();
    if (bstep) {
      const uint32_t* P = T + (size_t)code * KD;
#pragma unroll
      for (int j = 0; j < L; ++j) stream[j * G + g] = P[j * G + g];      // coalesced over the group
    }
    __builtin_amdgcn_wave_barrier();
    // B-step: B * P_j (P_j staged in LDS); A-step / idle: A * B with A read in place
    M.mul(r, Bd, bstep ? stream : abuf);
    if (bstep) {
#pragma unroll
      for (int j = 0; j < L; ++j) Bd[j] = r[j];
    } else if (code == FB_A_STEP) {
#pragma unroll
      for (int j = 0; j < L; ++j) abuf[g * L + j] = r[j];
    }
  }
  // leave Montgomery form: A * 1 / R, then exact reduction
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < L; ++j) {
    r[j] = abuf[g * L + j];
    stream[g * L + j] = (g == 0 && j == 0) ? 1u : 0u;
  }
  __builtin_amdgcn_wave_barrier();
  M.mul(r, r, stream);
  M.carry_exact(r);
  M.sub_if_ge(r);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = r[j];
  __builtin_amdgcn_wave_barrier();
  uint32_t* O = reinterpret_cast<uint32_t*>(a.out_ptr[inst]);
  constexpr int LO = K32 / G;
#pragma unroll
  for (int k = 0; k < LO; ++k) O[g * LO + k] = limb_of(stream, KD, g * LO + k);
}

// ---- launchers ------------------------------------------------------------------
// launches with fewer waves than SIMDs: one wave per block (see modexp.hip)
static inline uint32_t fb_block_threads(uint32_t lanes) { return lanes <= 256u * 4u * 64u ? 64u : (uint32_t)BLOCK; }

template <int KD, int G, int K32>
static hipError_t table_launch(const FbTableArgs& a, hipStream_t st) {
  const uint32_t bs = fb_block_threads(a.count * G), ipb = bs / G;
  hipLaunchKernelGGL((fb_table_kernel<KD, G, K32>), dim3((a.count + ipb - 1) / ipb), dim3(bs), 0, st, a);
  return hipGetLastError();
}
template <int KD, int G, int K32>
static hipError_t exp_launch(const FbExpArgs& a, hipStream_t st) {
  const uint32_t bs = fb_block_threads(a.count * G), ipb = bs / G;
  hipLaunchKernelGGL((fb_exp_kernel<KD, G, K32>), dim3((a.count + ipb - 1) / ipb), dim3(bs), 0, st, a);
  return hipGetLastError();
}

template <int KR, int L, int K32>
static hipError_t table_launch_wave(const FbTableArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((fb_table_wave_kernel<KR, L, K32>), dim3(a.count), dim3(64), 0, st, a);
  return hipGetLastError();
}

// Few bases (n = 64: 192 chains; a multi-GPU rank's receivers) run one per wave,
// latency first; more (n = 256: 768 chains, many sessions) the 8- / 4-lane group
// shapes, whose MACs per issued instruction are higher (the wave shape at n = 256
// measured 606 -> 728 ms per collect, profiles/r03o_bench.json config3).
constexpr uint32_t kFbWaveMax = 256;

hipError_t launch_fb_table(uint32_t k32, const FbTableArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  const bool wave = a.count <= kFbWaveMax;
  switch (k32) {
    case 64: return wave ? table_launch_wave<72, 2, 64>(a, st) : table_launch<72, 8, 64>(a, st);
    case 96: return wave ? table_launch_wave<108, 2, 96>(a, st) : table_launch<108, 4, 96>(a, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_fb_sched(const FbSchedArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  if (a.w > FB_MAX_W) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fb_sched_kernel, dim3((a.count + FB_SCHED_IPB - 1) / FB_SCHED_IPB), dim3(64 * FB_SCHED_IPB), 0,
                     st, a);
  return hipGetLastError();
}

hipError_t launch_fb_exp(uint32_t k32, const FbExpArgs& a, int group, hipStream_t st) {
  if (!a.count) return hipSuccess;
  switch (k32) {
    case 64:
      switch (group) {
        case 8: return exp_launch<72, 8, 64>(a, st);
        case 2: return exp_launch<72, 2, 64>(a, st);
        default: return exp_launch<72, 4, 64>(a, st);
      }
    case 96: return exp_launch<108, 4, 96>(a, st);
    default: return hipErrorInvalidValue;
  }
}

uint32_t fb_window(uint32_t ebits) {
  // products per exponent ~ ceil(bits/w) + 2^w - 1 (the table chain is per base)
  uint32_t best = 1, cost = 0xFFFFFFFFu;
  for (uint32_t w = 1; w <= 8; ++w) {
    const uint32_t c = (ebits + w - 1) / w + (1u << w) - 1;
    if (c < cost) {
      cost = c;
      best = w;
    }
  }
  return best;
}

}  // namespace fsdkr
