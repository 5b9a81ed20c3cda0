// Lim-Lee comb fixed-base exponentiation on gfx950 for bases shared by many
// exponents: the ring-Pedersen T^Z_k checks (ring_pedersen_proof.rs:144, M =
// 256 exponents per T) of collect() and of many sessions at once (BASELINE
// configs[4]), and the stand-alone fsdkr_fixed_base_modexp.  Results are
// bit-identical to base^exp mod N; only the order of the Montgomery products
// changes (fixedbase.h: the exponent as an h x v x b bit array).
//
// Per base: the squaring chain P_m = base^(2^(m b)) (fb_table_kernel, or the
// BGMW table chain every pstep-th entry), then comb_build_kernel fills the v
// tables of 2^h products one popcount level at a time (G[u] = G[u - top] *
// P_top), comb_sched_kernel transposes every exponent into its v b table
// indices, and comb_exp_kernel runs b - 1 squarings and v b products per
// exponent in lockstep (every instance has the same schedule shape).
#include "fixedbase.h"
#include "mont29.hpp"

namespace fsdkr {

// Level 1 of every base's v tables: u = 0 (the Montgomery one) and the single
// bits (copies of chain entries).  No LDS: it fits beside running launches.
template <int KD>
__global__ __launch_bounds__(BLOCK) void comb_copy_kernel(const CombBuildArgs a) {
  const uint32_t per_base = a.v * a.nu;
  const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint64_t inst = t / KD;
  if (inst >= (uint64_t)a.nbase * per_base) return;
  const uint32_t k = (uint32_t)(t - inst * KD);
  const uint32_t base = (uint32_t)(inst / per_base), rem = (uint32_t)(inst - (uint64_t)base * per_base);
  const uint32_t j = rem / a.nu, u = a.ulist[rem - j * a.nu];
  if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  const uint32_t* src = u == 0 ? a.consts + (size_t)a.mod_idx[base] * cons_stride(KD) + KD
                               : a.chain + ((size_t)a.ptoff[base] + (size_t)(__builtin_ctz(u) * a.v + j) * a.pstep) * KD;
  a.comb[(((size_t)base * a.v + j) * ((size_t)1 << a.h) + u) * KD + k] = src[k];
}

// One popcount level p >= 2 of every base's v tables: the u of popcount p,
// G[u] = G[u without its top bit] * P_top.
template <int KD, int G, int K32>
__global__ __launch_bounds__(BLOCK) void comb_build_kernel(const CombBuildArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * IPB + li;
  const uint32_t per_base = a.v * a.nu;
  if (inst >= a.nbase * per_base) return;
  const uint32_t base = inst / per_base, rem = inst - base * per_base;
  const uint32_t j = rem / a.nu, u = a.ulist[rem - j * a.nu];
  const uint32_t TS = 1u << a.h;
  const uint32_t* C = a.consts + (size_t)a.mod_idx[base] * STRIDE;
  uint32_t* tab = a.comb + ((size_t)base * a.v + j) * TS * KD;
  if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  uint32_t* stream = lds + li * KD;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int k = 0; k < L; ++k) M.n[k] = C[g * L + k];
  M.ninv = C[3 * KD];
  const uint32_t top = 31u - __builtin_clz(u);
  const uint32_t* prev = tab + (size_t)(u ^ (1u << top)) * KD;
  const uint32_t* P = a.chain + ((size_t)a.ptoff[base] + (size_t)(top * a.v + j) * a.pstep) * KD;
  uint32_t acc[L];
#pragma unroll
  for (int k = 0; k < L; ++k) acc[k] = prev[g * L + k];
#pragma unroll
  for (int k = 0; k < L; ++k) stream[k * G + g] = P[k * G + g];
  __builtin_amdgcn_wave_barrier();
  M.mul(acc, acc, stream);
#pragma unroll
  for (int k = 0; k < L; ++k) tab[(size_t)u * KD + g * L + k] = acc[k];
}

// One wave64 per exponent: its words into LDS (coalesced), then the lanes write
// the v b table indices in step order s = (b - 1 - k) v + j (coalesced u16 rows).
constexpr int COMB_SCHED_IPB = 4;
constexpr uint32_t COMB_MAX_WORDS = 256;   // exponents of up to 8192 bits (host-checked)
__global__ __launch_bounds__(64 * COMB_SCHED_IPB) void comb_sched_kernel(const CombSchedArgs a) {
  __shared__ uint32_t e_lds[COMB_SCHED_IPB][COMB_MAX_WORDS];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t i = blockIdx.x * COMB_SCHED_IPB + wv;   // wave-uniform
  if (i >= a.count) return;
  const uint32_t* E = reinterpret_cast<const uint32_t*>(a.exp_ptr[i]);
  const uint32_t elen = a.exp_len[i];
  const uint32_t words = (a.h * a.v * a.b + 31) / 32;   // bits past h v b are zero (host-checked)
  uint32_t* e = e_lds[wv];
  for (uint32_t q = lane; q < words; q += 64) e[q] = q < elen ? E[q] : 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const uint32_t steps = a.v * a.b;
  uint16_t* S = a.sched + (size_t)i * steps;
  for (uint32_t s = lane; s < steps; s += 64) {
    const uint32_t k = a.b - 1 - s / a.v, j = s % a.v;
    uint32_t u = 0;
    for (uint32_t r = 0; r < a.h; ++r) {
      const uint32_t t = (r * a.v + j) * a.b + k;
      u |= ((e[t >> 5] >> (t & 31)) & 1u) << r;
    }
    S[s] = (uint16_t)u;
  }
}

// base^e from the instance's tables: acc = G[0][u_0], then per step a product by
// G[j][u] (a squaring first at every j = 0 after the first column), lockstep.
// QS: quotient-scaled rows (the chain modulo N' = N (-N^-1 mod 2^29), exit modulo N;
// the tables' residues mod N are valid inputs, as in modexp_kernel QS)
template <int KD, int G, int K32, bool QS>
__global__ __launch_bounds__(BLOCK) void comb_exp_kernel(const CombExpArgs args) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  static_assert(!QS || scaled_ok(KD, K32), "quotient-scaled chains: N' within R/4");
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  uint32_t gk = 0;   // the block's group (block-uniform)
  for (uint32_t k = 1; k < args.ngroups; ++k)
    if (blockIdx.x >= args.g[k].block0) gk = k;
  const CombGroupDev& a = args.g[gk];
  const uint32_t inst = (blockIdx.x - a.block0) * (blockDim.x / G) + li;
  if (inst >= a.count) return;
  if (args.prio >= 3) __builtin_amdgcn_s_setprio(3);
  else if (args.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (args.prio == 1) __builtin_amdgcn_s_setprio(1);
  uint32_t* stream = lds + li * KD;
  const uint32_t* C0 = args.consts + (size_t)a.mod_idx[inst] * STRIDE;
  const uint32_t* C = QS ? C0 + cons_scaled(KD) : C0;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int k = 0; k < L; ++k) M.n[k] = C[g * L + k];
  M.ninv = C[3 * KD];
  const uint32_t TS = 1u << a.h;
  const uint32_t* tab = a.comb + (size_t)a.ibase[inst] * a.v * TS * KD;
  const uint16_t* S = a.sched + (size_t)inst * a.steps;
  uint32_t acc[L];
  {
    const uint32_t* E0 = tab + (size_t)S[0] * KD;
#pragma unroll
    for (int k = 0; k < L; ++k) acc[k] = E0[g * L + k];
  }
  uint32_t j = 0;
  for (uint32_t st = 1; st < a.steps; ++st) {
    if (++j == a.v) {   // next column: square first
      j = 0;
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < L; ++k) stream[g * L + k] = acc[k];
      __builtin_amdgcn_wave_barrier();
      if constexpr (QS) M.sqr_s(acc, acc, stream);
      else M.sqr(acc, acc, stream);
    }
    const uint32_t* P = tab + ((size_t)j * TS + S[st]) * KD;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < L; ++k) stream[k * G + g] = P[k * G + g];   // coalesced over the group
    __builtin_amdgcn_wave_barrier();
    if constexpr (QS) M.mul_s(acc, acc, stream);
    else M.mul(acc, acc, stream);
  }
  // leave Montgomery form: acc * 1 / R, then exact reduction (modulo N itself)
  if constexpr (QS) {
#pragma unroll
    for (int k = 0; k < L; ++k) M.n[k] = C0[g * L + k];
    M.ninv = C0[3 * KD];
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < L; ++k) stream[g * L + k] = (g == 0 && k == 0) ? 1u : 0u;
  __builtin_amdgcn_wave_barrier();
  M.mul(acc, acc, stream);
  M.carry_exact(acc);
  M.sub_if_ge(acc);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < L; ++k) stream[g * L + k] = acc[k];
  __builtin_amdgcn_wave_barrier();
  uint32_t* O = reinterpret_cast<uint32_t*>(a.out_ptr[inst]);
  constexpr int LO = K32 / G;
#pragma unroll
  for (int k = 0; k < LO; ++k) O[g * LO + k] = limb_of(stream, KD, g * LO + k);
}

// ---- launchers ------------------------------------------------------------------
template <int KD, int G, int K32>
static hipError_t build_launch(const CombBuildArgs& a, hipStream_t st) {
  constexpr uint32_t IPB = BLOCK / G;
  const size_t n = (size_t)a.nbase * a.v * a.nu;
  if (!n) return hipSuccess;
  if (a.nu && a.ulist_level1) {   // copies: one thread per word
    const size_t words = n * KD;
    hipLaunchKernelGGL((comb_copy_kernel<KD>), dim3((uint32_t)((words + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, a);
  } else {
    hipLaunchKernelGGL((comb_build_kernel<KD, G, K32>), dim3((uint32_t)((n + IPB - 1) / IPB)), dim3(BLOCK), 0, st, a);
  }
  return hipGetLastError();
}
template <int KD, int G, int K32, bool QS>
static hipError_t exp_launch(CombExpArgs& a, hipStream_t st) {
  uint64_t lanes = 0;
  for (uint32_t k = 0; k < a.ngroups; ++k) lanes += (uint64_t)a.g[k].count * G;
  const uint32_t bs = lanes <= 256u * 4u * 64u ? 64u : (uint32_t)BLOCK, ipb = bs / G;
  uint32_t blocks = 0;
  for (uint32_t k = 0; k < a.ngroups; ++k) {
    a.g[k].block0 = blocks;
    blocks += (a.g[k].count + ipb - 1) / ipb;
  }
  if (!blocks) return hipSuccess;
  hipLaunchKernelGGL((comb_exp_kernel<KD, G, K32, QS>), dim3(blocks), dim3(bs), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_comb_build(uint32_t k32, const CombBuildArgs& a, hipStream_t st) {
  switch (k32) {
    case 64: return build_launch<72, 4, 64>(a, st);
    case 96: return build_launch<108, 4, 96>(a, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_comb_sched(const CombSchedArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  if ((a.h * a.v * a.b + 31) / 32 > COMB_MAX_WORDS || a.h > 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL(comb_sched_kernel, dim3((a.count + COMB_SCHED_IPB - 1) / COMB_SCHED_IPB),
                     dim3(64 * COMB_SCHED_IPB), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_comb_exp(uint32_t k32, CombExpArgs& a, int group, hipStream_t st) {
  if (a.ngroups == 0 || a.ngroups > (uint32_t)kCombGroups) return hipErrorInvalidValue;
  for (uint32_t k = 0; k < a.ngroups; ++k)
    if (!a.g[k].steps) return hipErrorInvalidValue;
  // quotient-scaled rows (no v_mul_lo_u32 per row: -0.9 % kernel time against the
  // plain rows, profiles/r05/r05cqs_ab/)
  switch (k32) {
    case 64: return group == 8 ? exp_launch<72, 8, 64, true>(a, st) : exp_launch<72, 4, 64, true>(a, st);
    case 96: return exp_launch<108, 4, 96, true>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace fsdkr
