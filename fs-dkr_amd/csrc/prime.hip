// Batched Miller–Rabin for key generation, gfx950.
//
// Replaces the primality test behind kzen-paillier 0.4.3
// Paillier::keypair_with_modulus_size (called at refresh_message.rs:118,
// ring_pedersen_proof.rs:50, add_party_message.rs:51; the crate is a
// dependency, not vendored): one strong-probable-prime round per instance,
//   c - 1 = d 2^s,  pass  <=>  b^d == 1  or  b^(d 2^j) == c - 1 for some j < s.
//
// b^d mod c runs through the batched modexp engine (modexp.hip, every candidate
// its own modulus); this file is the witness tail: up to s - 1 Montgomery
// squarings of the lane-distributed radix-2^29 arithmetic (mont29.hpp), each
// compared exactly against 1 and c - 1.  The loop runs s_max (a launch
// argument) times for every group, so DPP moves never sit in divergent code;
// an instance past its own s or already settled keeps its verdict.
#include "mont29.hpp"
#include "kernels.h"

namespace fsdkr {

template <int KD, int G, int K32>
__global__ __launch_bounds__(BLOCK) void mr_tail_kernel(const MrTailArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * IPB + li;
  if (inst >= a.count) return;   // whole groups only: DPP stays inside a group
  uint32_t* stream = lds + li * KD;
  const uint32_t* C = a.consts + (size_t)inst * STRIDE;   // candidate inst is modulus inst
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = C[g * L + j];
  M.ninv = C[3 * KD];
  // exact comparisons of d (digits < 2^29, value < c) with 1 and c - 1
  // (c is odd, so c - 1 differs from c only in digit 0, without a borrow)
  auto is_one = [&](const uint32_t* d) -> bool {
    int bad = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) bad |= (d[j] != ((g == 0 && j == 0) ? 1u : 0u)) ? 1 : 0;
    return group_max<G>(bad) == 0;
  };
  auto is_minus1 = [&](const uint32_t* d) -> bool {
    int bad = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) bad |= (d[j] != ((g == 0 && j == 0) ? M.n[0] - 1u : M.n[j])) ? 1 : 0;
    return group_max<G>(bad) == 0;
  };
  uint32_t e[L], xm[L];
  const uint32_t* X = a.x + (size_t)inst * K32;   // b^d mod c, exact
#pragma unroll
  for (int j = 0; j < L; ++j) e[j] = digit_of(X, K32, g * L + j);
  const uint32_t s = a.s[inst];
  bool pass = is_one(e) || is_minus1(e);
  bool done = pass;
  // xm = x R mod c: Montgomery product with R^2
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = C[2 * KD + g * L + j];
  __builtin_amdgcn_wave_barrier();
  M.mul(xm, e, stream);
  for (uint32_t k = 1; k < a.s_max; ++k) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = xm[j];
    __builtin_amdgcn_wave_barrier();
    M.sqr(xm, xm, stream);                         // x^(2^k) in Montgomery form (< 2c)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = (g == 0 && j == 0) ? 1u : 0u;
    __builtin_amdgcn_wave_barrier();
    M.mul(e, xm, stream);                          // leave Montgomery form
    M.carry_exact(e);
    M.sub_if_ge(e);
    const bool m1 = is_minus1(e), one = is_one(e);
    if (k < s && !done) {
      if (m1) pass = true;
      done = m1 || one;                            // 1 before -1: composite
    }
  }
  if (g == 0) a.verdict[inst] = pass ? 1u : 0u;
}

template <int KD, int G, int K32>
static hipError_t mr_tail_launch(const MrTailArgs& a, hipStream_t st) {
  constexpr uint32_t IPB = BLOCK / G;
  const uint32_t blocks = (a.count + IPB - 1) / IPB;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((mr_tail_kernel<KD, G, K32>), dim3(blocks), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}

hipError_t mr_tail(uint32_t k32, const MrTailArgs& a, hipStream_t st) {
  switch (k32) {
    case 32: return mr_tail_launch<36, 4, 32>(a, st);
    case 64: return mr_tail_launch<72, 4, 64>(a, st);
    case 96: return mr_tail_launch<108, 4, 96>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace fsdkr
