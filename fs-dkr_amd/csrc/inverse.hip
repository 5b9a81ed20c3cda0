// Modular inverse / unit test for the collect() path on gfx950:
//   out = y^-1 mod m  and  unit = (gcd(y, m) == 1)        (m odd)
//
// Replaces curv BigInt::mod_inv (GMP mpz_invert) at zk_pdl_with_slack.rs:180
// (the PDL verifier unwraps it: a non-unit panics) and range_proofs.rs:129,142
// (AliceProof::verify returns false on None).
//
// Algorithm: Pornin's optimised binary GCD (eprint 2020/972, Alg. 2) with
// k-1 = 30 inner steps per outer step, so |f|,|g| <= 2^30 fit one signed 32-bit
// operand (one v_mad_i64_i32 per limb product) and the exact division by 2^30
// that closes every outer step is a one-limb shift in radix 2^30.
//
// Layout: one instance = G consecutive lanes; the four working integers
// a, b (the GCD pair) and u, v (their cofactors mod m) live in registers as
// LL radix-2^30 limbs per lane (NLT = G*LL limbs >= bits(m)/30 + 1).  Carries
// between lanes move by DPP; the 62-bit approximations of a, b that drive the
// inner loop are read back through a per-instance LDS mirror.  All G lanes run
// the (tiny) inner loop redundantly, so every decision is group-uniform.
#include "mont29.hpp"
#include "verify.h"

namespace fsdkr {

constexpr uint32_t M30 = (1u << 30) - 1;

__device__ __forceinline__ uint32_t digit30_of(const uint32_t* __restrict__ x, int K32, int j) {
  const int bit = 30 * j;
  const int w = bit >> 5, sh = bit & 31;
  const uint32_t lo = (w < K32) ? x[w] : 0u;
  const uint32_t hi = (w + 1 < K32) ? x[w + 1] : 0u;
  return (uint32_t)(mk64(lo, hi) >> sh) & M30;
}

template <int G, int LL>
struct Coop {
  int g;
  uint32_t m_first, m_top;

  __device__ __forceinline__ int64_t prev_s64(int64_t v) const {
    const uint32_t lo = dpp_prev<G>((uint32_t)v) & m_first;
    const uint32_t hi = dpp_prev<G>((uint32_t)((uint64_t)v >> 32)) & m_first;
    return (int64_t)mk64(lo, hi);
  }
  __device__ __forceinline__ int64_t top_s64(int64_t v) const {
    return (int64_t)mk64(bcast_top<G>((uint32_t)v), bcast_top<G>((uint32_t)((uint64_t)v >> 32)));
  }
  __device__ __forceinline__ uint32_t group_or(uint32_t v) const {
    if constexpr (G >= 2) v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
    if constexpr (G >= 4) v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
    if constexpr (G >= 8) v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
    if constexpr (G >= 16) v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);
    return v;
  }

  // Normalise signed column values t (|t_j| < 2^62) into limbs x in [0, 2^30).
  // Returns T (every lane): value = sum x_j 2^(30 j) + T 2^(30 NLT).
  __device__ __forceinline__ int64_t norm(const int64_t* t, uint32_t* x) const {
    int64_t c = 0;
#pragma unroll
    for (int j = 0; j < LL; ++j) {
      const int64_t v = t[j] + c;
      x[j] = (uint32_t)v & M30;
      c = v >> 30;
    }
    int64_t top = c;
    int64_t in = prev_s64(c);
    // |in| < 2^33: after two limbs the remaining carry is -1, 0 or 1 and a
    // longer ripple (a run of all-zero / all-one limbs) is rare
    for (int round = 0; round < G; ++round) {
      int64_t v = (int64_t)x[0] + in;
      x[0] = (uint32_t)v & M30;
      int64_t r = v >> 30;
      v = (int64_t)x[1] + r;
      x[1] = (uint32_t)v & M30;
      r = v >> 30;
      if (r != 0) {
#pragma unroll
        for (int j = 2; j < LL; ++j) {
          v = (int64_t)x[j] + r;
          x[j] = (uint32_t)v & M30;
          r = v >> 30;
        }
      }
      top += r;
      in = prev_s64(r);
      if (!__any(in != 0)) break;
    }
    return top_s64(top);
  }

  // x <- x / 2^30 (limb 0 is zero by construction); the top limb becomes 0
  __device__ __forceinline__ void shift_down(uint32_t* x) const {
    const uint32_t nx = dpp_next<G>(x[0]) & m_top;
#pragma unroll
    for (int j = 0; j < LL - 1; ++j) x[j] = x[j + 1];
    x[LL - 1] = nx;
  }

  // x <- -x for a value held as two's complement limbs below the top limb
  __device__ __forceinline__ void negate(uint32_t* x) const {
    int64_t t[LL];
#pragma unroll
    for (int j = 0; j < LL; ++j) t[j] = (int64_t)(M30 - x[j]);
    if (g == G - 1) t[LL - 1] = 0;          // limb NLT-1 stays 0
    if (g == 0) t[0] += 1;
    (void)norm(t, x);
  }
};

// The inverse of one instance by its G lanes: Y (value, K32 u32 limbs, any
// pointer: global or LDS), Mo (odd modulus); O (K32 limbs) receives y^-1 mod m
// when not null; `mir` is the instance's 2 NLT-word LDS mirror.  Returns the
// unit flag (gcd(y, m) == 1), group-uniform.
template <int K32, int G>
struct CoopShape {
  static constexpr int NLT0 = (32 * K32 + 29) / 30 + 1;
  static constexpr int LL = (NLT0 + G - 1) / G;
  static constexpr int NLT = LL * G;
};

template <int K32, int G>
__device__ bool coop_inverse(const uint32_t* Y, const uint32_t* Mo, uint32_t* O, uint32_t* mir, int g) {
  constexpr int LL = CoopShape<K32, G>::LL;
  constexpr int NLT = CoopShape<K32, G>::NLT;
  Coop<G, LL> C;
  C.g = g;
  C.m_first = (g == 0) ? 0u : 0xFFFFFFFFu;
  C.m_top = (g == G - 1) ? 0u : 0xFFFFFFFFu;
  asm volatile("" : "+v"(C.m_first), "+v"(C.m_top));

  uint32_t A[LL], B[LL], U[LL], V[LL], Mx[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) {
    A[j] = digit30_of(Y, K32, g * LL + j);
    B[j] = Mx[j] = digit30_of(Mo, K32, g * LL + j);
    U[j] = (g == 0 && j == 0) ? 1u : 0u;
    V[j] = 0u;
  }
  // -m^-1 mod 2^30 (every lane: m's limb 0 word is read directly)
  const uint32_t m0 = Mo[0];
  uint32_t inv = m0;
#pragma unroll
  for (int it = 0; it < 5; ++it) inv *= 2u - m0 * inv;
  const uint32_t mneg_inv = (0u - inv) & M30;
  // bit length of m
  int mlen = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j)
    if (Mx[j]) mlen = (g * LL + j) * 30 + 32 - __builtin_clz(Mx[j]);
  mlen = group_max<G>(mlen);
  const int iters = (2 * mlen - 1 + 29) / 30;

  for (int it = 0; it < iters; ++it) {
    // ---- n = max(len(a), len(b), 62) and the 62-bit approximations
    int ln = 0;
#pragma unroll
    for (int j = 0; j < LL; ++j) {
      const uint32_t t = A[j] | B[j];
      if (t) ln = (g * LL + j) * 30 + 32 - __builtin_clz(t);
    }
    ln = group_max<G>(ln);
    const int nbits = ln < 62 ? 62 : ln;
#pragma unroll
    for (int j = 0; j < LL; ++j) {
      mir[g * LL + j] = A[j];
      mir[NLT + g * LL + j] = B[j];
    }
    __builtin_amdgcn_wave_barrier();
    const int sh = nbits - 32, p = sh / 30, o = sh % 30;
    auto top32 = [&](const uint32_t* x) -> uint64_t {
      const uint64_t x0 = x[p];
      const uint64_t x1 = (p + 1 < NLT) ? x[p + 1] : 0u;
      const uint64_t x2 = (p + 2 < NLT) ? x[p + 2] : 0u;
      return ((x0 | (x1 << 30) | (x2 << 60)) >> o) & 0xFFFFFFFFull;   // x2 << 60 keeps its low 4 bits
    };
    uint64_t ah = (top32(mir) << 30) | mir[0];
    uint64_t bh = (top32(mir + NLT) << 30) | mir[NLT];
    __builtin_amdgcn_wave_barrier();
    // ---- 30 inner steps on the approximations
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll 6
    for (int j = 0; j < 30; ++j) {
      const bool odd = (ah & 1u) != 0;
      const bool sw = odd && (ah < bh);
      const uint64_t na = sw ? bh : ah, nb = sw ? ah : bh;
      const int32_t nf0 = sw ? f1 : f0, nf1 = sw ? f0 : f1, ng0 = sw ? g1 : g0, ng1 = sw ? g0 : g1;
      ah = odd ? na - nb : na;
      bh = nb;
      f0 = odd ? nf0 - nf1 : nf0;
      g0 = odd ? ng0 - ng1 : ng0;
      f1 = nf1 * 2;
      g1 = ng1 * 2;
      ah >>= 1;
    }
    // ---- (a, b) <- ((a f0 + b g0) / 2^30, (a f1 + b g1) / 2^30), made non-negative
    int64_t t[LL];
    uint32_t NA[LL];
#pragma unroll
    for (int j = 0; j < LL; ++j) t[j] = (int64_t)(int32_t)A[j] * f0 + (int64_t)(int32_t)B[j] * g0;
    int64_t T = C.norm(t, NA);
    C.shift_down(NA);
    if (T < 0) {            // group-uniform
      C.negate(NA);
      f0 = -f0;
      g0 = -g0;
    }
#pragma unroll
    for (int j = 0; j < LL; ++j) t[j] = (int64_t)(int32_t)A[j] * f1 + (int64_t)(int32_t)B[j] * g1;
    T = C.norm(t, B);
    C.shift_down(B);
    if (T < 0) {
      C.negate(B);
      f1 = -f1;
      g1 = -g1;
    }
#pragma unroll
    for (int j = 0; j < LL; ++j) A[j] = NA[j];
    // ---- (u, v) <- ((u f0 + v g0) / 2^30 mod m, (u f1 + v g1) / 2^30 mod m), kept in [0, m)
    auto mdiv = [&](int32_t f, int32_t gg, uint32_t* out) {
      const uint32_t lo = (U[0] * (uint32_t)f + V[0] * (uint32_t)gg) & M30;   // lane 0's limb 0 (mod 2^30)
      const uint32_t q = bcast_lane0<G>((uint32_t)(lo * mneg_inv) & M30);
      int64_t w[LL];
#pragma unroll
      for (int j = 0; j < LL; ++j)
        w[j] = (int64_t)(int32_t)U[j] * f + (int64_t)(int32_t)V[j] * gg + (int64_t)((uint64_t)q * Mx[j]);
      const int64_t T0 = C.norm(w, out);
      C.shift_down(out);
      // result in (-m, 2m): add m if negative, else subtract m if >= m
      const bool neg = T0 < 0;
#pragma unroll
      for (int j = 0; j < LL; ++j) w[j] = neg ? (int64_t)out[j] + Mx[j] : (int64_t)out[j] - (int64_t)Mx[j];
      if (neg && g == G - 1) w[LL - 1] -= 1;   // the sign T0 = -1 sits at limb NLT-1 after the shift
      uint32_t R[LL];
      const int64_t T1 = C.norm(w, R);
      const bool take = neg || T1 >= 0;
#pragma unroll
      for (int j = 0; j < LL; ++j) out[j] = take ? R[j] : out[j];
    };
    uint32_t NU[LL];
    mdiv(f0, g0, NU);
    mdiv(f1, g1, V);
#pragma unroll
    for (int j = 0; j < LL; ++j) U[j] = NU[j];
  }
  // ---- unit <=> b == 1; inverse = v
  uint32_t nz = 0;
#pragma unroll
  for (int j = 0; j < LL; ++j) nz |= (g == 0 && j == 0) ? (B[j] ^ 1u) : B[j];
  nz = C.group_or(nz);
  if (O) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < LL; ++j) mir[g * LL + j] = V[j];
    __builtin_amdgcn_wave_barrier();
    for (int k = g; k < K32; k += G) {
      const int bit = 32 * k, j = bit / 30, s = bit % 30;
      const uint64_t d0 = mir[j], d1 = (j + 1 < NLT) ? mir[j + 1] : 0u, d2 = (j + 2 < NLT) ? mir[j + 2] : 0u;
      O[k] = (uint32_t)((d0 | (d1 << 30) | (d2 << 60)) >> s);
    }
    __builtin_amdgcn_wave_barrier();
  }
  return nz == 0;
}

template <int K32, int G>
__global__ __launch_bounds__(256) void inverse_coop_kernel(const InverseArgs a) {
  constexpr int NLT = CoopShape<K32, G>::NLT;
  constexpr int IPB = 256 / G;
  __shared__ uint32_t lds[IPB * 2 * NLT];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * IPB + li;
  if (inst >= a.count) return;
  uint32_t* mir = lds + li * 2 * NLT;       // [a | b] mirror for the approximations
  const uint32_t* Y = reinterpret_cast<const uint32_t*>(a.y_ptr[inst]);
  const uint32_t* Mo = reinterpret_cast<const uint32_t*>(a.m_ptr[inst]);
  const bool unit = coop_inverse<K32, G>(Y, Mo, a.out ? a.out + (size_t)inst * K32 : nullptr, mir, g);
  if (g == 0) a.unit[inst] = unit ? 1u : 0u;
}

// Montgomery's simultaneous inversion over the instances of one modulus (one
// group of G lanes per modulus).  With mont(a, b) = a b / R and raw values:
//   P'_1 = y_1,  P'_k = mont(P'_{k-1}, y_k) = (y_1 .. y_k) R^-(k-1)
//   I_m  = P'_m^-1 (one binary-GCD inverse, coop_inverse)
//   y_k^-1 = mont(P'_{k-1}, I_k),  I_{k-1} = mont(I_k, y_k),  y_1^-1 = I_1
// so m elements cost 3 (m - 1) products and one inverse instead of m inverses,
// with no conversion into or out of Montgomery form.  The values are exact
// (carry_exact + sub_if_ge on every output).  gcd(P'_m, N) = 1 iff every y_k is a
// unit; otherwise every element of the group is inverted on its own (the unit
// flags and values the reference's per-element mod_inv gives).  Even moduli
// (no Montgomery form) take the per-element path too.
template <int KD, int G, int K32>
__global__ __launch_bounds__(64) void inverse_batch_kernel(const BatchInverseArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int NLT = CoopShape<K32, G>::NLT;
  constexpr int IPB = 64 / G;
  constexpr int W = KD + 2 * NLT + K32;
  constexpr int LO = K32 / G;
  __shared__ uint32_t lds[IPB * W];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t grp = blockIdx.x * IPB + li;
  if (grp >= a.ngroups) return;
  uint32_t* stream = lds + li * W;      // the streamed product operand (KD digits)
  uint32_t* mir = stream + KD;          // coop_inverse's mirror
  uint32_t* limbs = mir + 2 * NLT;      // u32 limbs of the inverse's operand / result
  const uint32_t s0 = a.gstart[grp], s1 = a.gstart[grp + 1];
  if (s1 <= s0) return;
  auto Yp = [&](uint32_t t) { return reinterpret_cast<const uint32_t*>(a.y_ptr[a.order[t]]); };
  const uint32_t* Mo = reinterpret_cast<const uint32_t*>(a.m_ptr[a.order[s0]]);
  auto put_out = [&](uint32_t t, const uint32_t* x) {   // exact digits x -> u32 limbs of instance order[t]
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = x[j];
    __builtin_amdgcn_wave_barrier();
    uint32_t* O = a.out + (size_t)a.order[t] * K32;
#pragma unroll
    for (int k = 0; k < LO; ++k) O[g * LO + k] = limb_of(stream, KD, g * LO + k);
    __builtin_amdgcn_wave_barrier();
  };
  auto per_element = [&]() {
    for (uint32_t t = s0; t < s1; ++t) {
      const uint32_t i = a.order[t];
      const bool u = coop_inverse<K32, G>(Yp(t), Mo, a.out ? a.out + (size_t)i * K32 : nullptr, mir, g);
      if (g == 0) a.unit[i] = u ? 1u : 0u;
    }
  };
  if ((Mo[0] & 1u) == 0u || s1 - s0 == 1) {   // even modulus, or one element: nothing to share
    per_element();
    return;
  }
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = digit_of(Mo, K32, g * L + j);
  {
    const uint32_t n0 = Mo[0];
    uint32_t inv = n0;
#pragma unroll
    for (int it = 0; it < 5; ++it) inv *= 2u - n0 * inv;   // N^-1 mod 2^32
    M.ninv = (0u - inv) & M29;
  }
  uint32_t* S = a.scratch;
  // ---- prefix products P'_k (scratch row t holds P'_{t - s0 + 1})
  uint32_t acc[L];
  {
    const uint32_t* Y = Yp(s0);
#pragma unroll
    for (int j = 0; j < L; ++j) acc[j] = digit_of(Y, K32, g * L + j);
  }
#pragma unroll
  for (int j = 0; j < L; ++j) S[(size_t)s0 * KD + g * L + j] = acc[j];
  for (uint32_t t = s0 + 1; t < s1; ++t) {
    const uint32_t* Y = Yp(t);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = digit_of(Y, K32, g * L + j);
    __builtin_amdgcn_wave_barrier();
    M.mul(acc, acc, stream);
#pragma unroll
    for (int j = 0; j < L; ++j) S[(size_t)t * KD + g * L + j] = acc[j];
  }
  // ---- one inverse of the product (exact u32 limbs in and out, through LDS)
  M.carry_exact(acc);
  M.sub_if_ge(acc);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = acc[j];
  __builtin_amdgcn_wave_barrier();
  for (int k = g; k < K32; k += G) limbs[k] = limb_of(stream, KD, k);
  __builtin_amdgcn_wave_barrier();
  if (!coop_inverse<K32, G>(limbs, Mo, limbs, mir, g)) {   // group-uniform
    per_element();
    return;
  }
  // every element is a unit
  for (uint32_t t = s0 + g; t < s1; t += G) a.unit[a.order[t]] = 1u;
  if (!a.out) return;
  // ---- backward pass: y_k^-1 = mont(P'_{k-1}, I_k), I_{k-1} = mont(I_k, y_k)
  uint32_t I[L];
#pragma unroll
  for (int j = 0; j < L; ++j) I[j] = digit_of(limbs, K32, g * L + j);
  for (uint32_t t = s1 - 1; t > s0; --t) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = S[(size_t)(t - 1) * KD + g * L + j];
    __builtin_amdgcn_wave_barrier();
    uint32_t x[L];
#pragma unroll
    for (int j = 0; j < L; ++j) x[j] = I[j];
    M.mul(x, x, stream);
    M.carry_exact(x);
    M.sub_if_ge(x);
    put_out(t, x);
    const uint32_t* Y = Yp(t);
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = digit_of(Y, K32, g * L + j);
    __builtin_amdgcn_wave_barrier();
    M.mul(I, I, stream);
  }
  M.carry_exact(I);
  M.sub_if_ge(I);
  put_out(s0, I);
}

template <int KD, int G, int K32>
static hipError_t launch_batch(const BatchInverseArgs& a, hipStream_t st) {
  constexpr int IPB = 64 / G;
  const uint32_t blocks = (a.ngroups + IPB - 1) / IPB;
  hipLaunchKernelGGL((inverse_batch_kernel<KD, G, K32>), dim3(blocks), dim3(64), 0, st, a);
  return hipGetLastError();
}

// the 2048 / 4096-bit widths (2048-bit keys: Ñ and N^2); others: 0 (per-element
// inverse_coop; their 8-lane Montgomery and inverse shapes do not share a lane count)
size_t inverse_batch_scratch_words(uint32_t k32) {
  switch (k32) {
    case 64: return 72;
    case 128: return 144;
    default: return 0;
  }
}

hipError_t launch_inverse_batch(uint32_t k32, const BatchInverseArgs& a, hipStream_t st) {
  if (!a.ngroups) return hipSuccess;
  switch (k32) {
    case 64: return launch_batch<72, 8, 64>(a, st);
    case 128: return launch_batch<144, 8, 128>(a, st);
    default: return hipErrorInvalidValue;
  }
}

template <int K32, int G>
static hipError_t launch_coop(const InverseArgs& a, hipStream_t st) {
  constexpr int IPB = 256 / G;
  const uint32_t blocks = (a.count + IPB - 1) / IPB;
  hipLaunchKernelGGL((inverse_coop_kernel<K32, G>), dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_inverse_coop(uint32_t k32, const InverseArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  switch (k32) {
    case 64: return launch_coop<64, 8>(a, st);
    case 96: return launch_coop<96, 8>(a, st);
    case 128: return launch_coop<128, 8>(a, st);
    case 192: return launch_coop<192, 16>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace fsdkr
