// Montgomery-form checks of the batched collect() job (gfx950), on the
// lane-distributed radix-2^29 arithmetic of mont29.hpp:
//   eq_check        a*b == c*d (mod N), optionally c < N      PDL u2/u3, RP, correct-key, DLog
//   prod3           a*b*c mod N (exact)                        range_proofs.rs:136-148 (w, u)
//   inverse         launcher of the lane-cooperative Pornin inverse (inverse.hip)
//                   mod_inv / unit tests                       zk_pdl_with_slack.rs:180, range_proofs.rs:129,142
#include "mont29.hpp"
#include "verify.h"
#include <cstdlib>

namespace fsdkr {

__device__ __forceinline__ const uint32_t* P32(uint64_t a) { return reinterpret_cast<const uint32_t*>(a); }
static inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

// -------------------------------------------------- Montgomery-form checks ----
template <int KD, int G>
__device__ __forceinline__ void load_digits(uint32_t* d, const uint32_t* x, int len, int g) {
  constexpr int L = KD / G;
#pragma unroll
  for (int j = 0; j < L; ++j) d[j] = digit_of(x, len, g * L + j);
}

// group-uniform: exact digits d >= n ?
template <int KD, int G>
__device__ __forceinline__ bool ge_mod(const Mont29<KD, G>& M, const uint32_t* d) {
  constexpr int L = KD / G;
  uint32_t bin = 0;
  for (int round = 0; round < G; ++round) {
    uint32_t bw = (round == 0) ? 0u : (dpp_prev<G>(bin) & M.m_first);
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint32_t v = d[j] - M.n[j] - bw;
      bw = v >> 31;
    }
    bin = bw;
  }
  return bcast_top<G>(bin == 0u ? 1u : 0u) != 0u;
}

// a*b == c*d (mod N)  [and c < N if flagged]
template <int KD, int G, int K32>
__global__ __launch_bounds__(BLOCK) void eq_check_kernel(const EqCheckArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * IPB + li;
  if (inst >= a.count) return;
  uint32_t* stream = lds + li * KD;
  const uint32_t* C = a.consts + (size_t)a.mod_idx[inst] * STRIDE;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = C[g * L + j];
  M.ninv = C[3 * KD];
  const EqOperand op = a.ops[inst];
  uint64_t dptr = op.d;
  if (op.sel != 0xFFFFFFFFu) {  // ring-Pedersen: d = S if challenge bit set, else 1
    const uint32_t bit = (a.sel_bits[op.sel >> 5] >> (op.sel & 31)) & 1u;
    if (!bit) dptr = a.one;
  }
  uint32_t x[L], y[L], cd[L];
  // x = a*b/R
  load_digits<KD, G>(x, P32(op.b), op.b_len, g);
  {
    const uint32_t* src = P32(op.a);
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = digit_of(src, op.a_len, g * L + j);
  }
  __builtin_amdgcn_wave_barrier();
  M.mul(x, x, stream);
  __builtin_amdgcn_wave_barrier();
  // y = c*d/R
  load_digits<KD, G>(cd, P32(op.c), op.c_len, g);
  load_digits<KD, G>(y, P32(dptr), op.d_len, g);
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = cd[j];
  __builtin_amdgcn_wave_barrier();
  M.mul(y, y, stream);
  M.carry_exact(x);
  M.sub_if_ge(x);
  M.carry_exact(y);
  M.sub_if_ge(y);
  uint32_t diff = 0;
#pragma unroll
  for (int j = 0; j < L; ++j) diff |= x[j] ^ y[j];
  // group-wide OR
  if constexpr (G >= 2) diff |= __builtin_amdgcn_mov_dpp(diff, 0xB1, 0xF, 0xF, false);
  if constexpr (G == 4) diff |= __builtin_amdgcn_mov_dpp(diff, 0x4E, 0xF, 0xF, false);
  bool ok = (diff == 0);
  if (op.flags & 1u) {
    // c < N  (c is a proof value compared for exact equality in the reference);
    // digits of c beyond KD do not exist: c < 2^(32*K32) <= R, so exactness holds
    bool c_big = false;
    {
      const uint32_t* cs = P32(op.c);
      for (uint32_t k = K32; k < op.c_len; ++k) c_big = c_big || (cs[k] != 0);
    }
    ok = ok && !c_big && !ge_mod<KD, G>(M, cd);
  }
  if (g == 0) a.out[inst] = ok ? 1u : 0u;
}

// out = a*b*c mod N  (exact, K32 limbs)
template <int KD, int G, int K32>
__global__ __launch_bounds__(BLOCK) void prod3_kernel(const Prod3Args a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * IPB + li;
  if (inst >= a.count) return;
  uint32_t* stream = lds + li * KD;
  const uint32_t* C = a.consts + (size_t)a.mod_idx[inst] * STRIDE;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = C[g * L + j];
  M.ninv = C[3 * KD];
  const Prod3Operand op = a.ops[inst];
  uint32_t x[L];
  load_digits<KD, G>(x, P32(op.b), op.b_len, g);
  {
    const uint32_t* src = P32(op.a);
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = digit_of(src, op.a_len, g * L + j);
  }
  __builtin_amdgcn_wave_barrier();
  M.mul(x, x, stream);                       // ab/R
  __builtin_amdgcn_wave_barrier();
  {
    const uint32_t* src = P32(op.c);
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = digit_of(src, op.c_len, g * L + j);
  }
  __builtin_amdgcn_wave_barrier();
  M.mul(x, x, stream);                       // abc/R^2
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = C[2 * KD + g * L + j];   // R^2 mod N
  __builtin_amdgcn_wave_barrier();
  M.mul(x, x, stream);                       // abc/R
  M.mul(x, x, stream);                       // abc
  M.carry_exact(x);
  M.sub_if_ge(x);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = x[j];
  __builtin_amdgcn_wave_barrier();
  uint32_t* O = a.out + (size_t)inst * K32;
  constexpr int LO = K32 / G;
#pragma unroll
  for (int k = 0; k < LO; ++k) O[g * LO + k] = limb_of(stream, KD, g * LO + k);
}

// ------------------------------------------------------------- launchers -------
hipError_t launch_inverse(uint32_t k32, const InverseArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  return launch_inverse_coop(k32, a, st);
}
template <int KD, int G, int K32>
static hipError_t eq_launch(const EqCheckArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((eq_check_kernel<KD, G, K32>), dim3(blocks_for(a.count, BLOCK / G)), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_eq_check(uint32_t k32, const EqCheckArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  switch (k32) {
    // 8-lane shapes: a few products per instance; the 2/4-lane shapes spilled
    // (256 VGPRs + 256 AGPRs + scratch) at the tail of every pipeline
    case 64: return eq_launch<72, 8, 64>(a, st);
    case 96: return eq_launch<108, 4, 96>(a, st);
    case 128: return eq_launch<144, 8, 128>(a, st);
    case 192: return eq_launch<216, 8, 192>(a, st);
    default: return hipErrorInvalidValue;
  }
}
template <int KD, int G, int K32>
static hipError_t p3_launch(const Prod3Args& a, hipStream_t st) {
  hipLaunchKernelGGL((prod3_kernel<KD, G, K32>), dim3(blocks_for(a.count, BLOCK / G)), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_prod3(uint32_t k32, const Prod3Args& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  switch (k32) {
    case 64: return p3_launch<72, 8, 64>(a, st);
    case 96: return p3_launch<108, 4, 96>(a, st);
    case 128: return p3_launch<144, 8, 128>(a, st);
    case 192: return p3_launch<216, 8, 192>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace fsdkr
