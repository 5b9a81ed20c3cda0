// Batched modular exponentiation on gfx950:  out[i] = base[i]^exp[i] mod N[mod_idx[i]].
//
// Replaces the GMP mpz_powm behind curv BigInt::mod_pow on the collect() hot
// path (zk_pdl_with_slack.rs:129-157 via commitment_unknown_order :170-188;
// range_proofs.rs:129-148; ring_pedersen_proof.rs:144-148; zk-paillier
// NiCorrectKeyProof/CompositeDLogProof verify called at refresh_message.rs:376-378,
// 401-425) and r^N mod N^2 of Paillier encryption (refresh_message.rs:72-84).
//
// One instance = G lanes (mont29.hpp); 256-thread blocks of 256/G instances.
// Fixed-window left-to-right exponentiation (window w chosen by the host), the
// window table lives in a per-instance global scratch slab, the streamed row
// operand of every Montgomery product in LDS.
#include "mont29.hpp"
#include "kernels.h"
#include <cstdlib>
#include <initializer_list>

namespace fsdkr {

template <int KD, int G>
__device__ __forceinline__ void lds_put(uint32_t* stream, const uint32_t* d, int g) {
  constexpr int L = KD / G;
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = d[j];
}

// consts row m (cons_stride(KD) words, kernels.h) = {N digits | R mod N | R^2 mod N |
// ninv}, then when scaled_ok(KD, K32) the same block for N' = N (-N^-1 mod 2^29)
// (the quotient-scaled chains of modexp_kernel<..., QS>).  Instances m < n_mod
// write the N block of modulus m, instances n_mod + m its N' block.
template <int KD, int G, int K32>
__global__ __launch_bounds__(BLOCK) void mod_setup_kernel(const uint32_t* __restrict__ mods, uint32_t n_mod,
                                                          uint32_t* __restrict__ consts) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr bool SC = scaled_ok(KD, K32);
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t mi = blockIdx.x * IPB + li;
  if (mi >= (SC ? 2 * n_mod : n_mod)) return;
  const bool scaled = SC && mi >= n_mod;
  const uint32_t m = scaled ? mi - n_mod : mi;
  // a few waves at the head of every job's chain: they win issue arbitration
  // against the exponentiation waves already on the SIMD
  __builtin_amdgcn_s_setprio(3);
  uint32_t* stream = lds + li * KD;
  const uint32_t* N = mods + (size_t)m * K32;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = digit_of(N, K32, g * L + j);
  const uint32_t n0 = N[0];
  uint32_t inv = n0;
#pragma unroll
  for (int it = 0; it < 5; ++it) inv *= 2u - n0 * inv;
  M.ninv = (0u - inv) & M29;
  if (scaled) M.scale_modulus();   // n <- N', ninv <- 1
  int hb = -1;
#pragma unroll
  for (int j = 0; j < L; ++j)
    if (M.n[j]) hb = (g * L + j) * 29 + 31 - __builtin_clz(M.n[j]);
  hb = group_max<G>(hb);
  uint32_t y[L];
#pragma unroll
  for (int j = 0; j < L; ++j) y[j] = ((g * L + j) == hb / 29) ? (1u << (hb % 29)) : 0u;  // 2^(bitlen-1) < N
  const int nd1 = 29 * KD - hb;                 // -> 2^(29 KD) = R mod N
  for (int k = 0; k < nd1; ++k) M.dbl(y);
  uint32_t* out = consts + (size_t)m * cons_stride(KD) + (scaled ? cons_scaled(KD) : 0);
#pragma unroll
  for (int j = 0; j < L; ++j) out[KD + g * L + j] = y[j];
  // R^2 mod N: 2^c * R (Montgomery form of 2^c) squared s times, c * 2^s = 29 KD
  constexpr int TWO_S = ((29 * KD) % 16 == 0) ? 16 : ((29 * KD) % 8 == 0) ? 8 : ((29 * KD) % 4 == 0) ? 4 : ((29 * KD) % 2 == 0) ? 2 : 1;
  constexpr int S = (TWO_S == 16) ? 4 : (TWO_S == 8) ? 3 : (TWO_S == 4) ? 2 : (TWO_S == 2) ? 1 : 0;
  constexpr int C = 29 * KD / TWO_S;
  for (int k = 0; k < C; ++k) M.dbl(y);
  for (int s = 0; s < S; ++s) {
    lds_put<KD, G>(stream, y, g);
    __builtin_amdgcn_wave_barrier();
    M.sqr(y, y, stream);
    __builtin_amdgcn_wave_barrier();
  }
  M.carry_exact(y);
  M.sub_if_ge(y);
  M.sub_if_ge(y);
#pragma unroll
  for (int j = 0; j < L; ++j) {
    out[g * L + j] = M.n[j];
    out[2 * KD + g * L + j] = y[j];
  }
  if (g == 0) out[3 * KD] = M.ninv;
}

// mod_setup_kernel's constants from one wave per modulus (Mont29<64 L, 64, KR>:
// L digits per lane, KR = the class's digits), so the setup takes ~20 VGPRs and
// little time: it is dispatched beside long-running throughput waves instead of
// waiting for a whole free slot.  (The 4-lane 3072-bit group setup took 196
// VGPRs and waited ~90 ms beside configs[4]'s GA at 2 waves/SIMD of 228 VGPRs,
// profiles/r05/r05j_config4_trace_head.txt.)  R^2 mod N by an addition chain on
// the exponent: x_a = 2^a R mod N, x_2a = mont(x_a, x_a), x_(a+1) = 2 x_a, from
// a = 1 to a = 29 KR (12 squarings and a few doublings instead of 29 KR / 4
// doublings).  Every value is exact, so the constants equal mod_setup_kernel's.
template <int KR, int L, int K32>
__global__ __launch_bounds__(64) void mod_setup_wave_kernel(const uint32_t* __restrict__ mods, uint32_t n_mod,
                                                            uint32_t* __restrict__ consts) {
  constexpr int KD = 64 * L;
  using MT = Mont29<KD, 64, KR>;
  constexpr bool SC = scaled_ok(KR, K32);
  const uint32_t mi = blockIdx.x;
  if (mi >= (SC ? 2 * n_mod : n_mod)) return;
  const bool scaled = SC && mi >= n_mod;
  const uint32_t m = scaled ? mi - n_mod : mi;
  __builtin_amdgcn_s_setprio(3);
  const int g = threadIdx.x;
  const bool live = g * L < KR;
  const uint32_t* N = mods + (size_t)m * K32;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = live ? digit_of(N, K32, g * L + j) : 0u;
  const uint32_t n0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)N[0]);
  uint32_t inv = n0;
#pragma unroll
  for (int it = 0; it < 5; ++it) inv *= 2u - n0 * inv;
  M.ninv = (0u - inv) & M29;
  if (scaled) M.scale_modulus();   // n <- N', ninv <- 1
  int hb = -1;
#pragma unroll
  for (int j = 0; j < L; ++j)
    if (M.n[j]) hb = (g * L + j) * 29 + 31 - __builtin_clz(M.n[j]);
  hb = group_max<64>(hb);
  uint32_t y[L];
#pragma unroll
  for (int j = 0; j < L; ++j) y[j] = ((g * L + j) == hb / 29) ? (1u << (hb % 29)) : 0u;   // 2^(bitlen-1) < N
  for (int k = 0; k < 29 * KR - hb; ++k) M.dbl(y);                                     // R mod N (exact)
  uint32_t* out = consts + (size_t)m * cons_stride(KR) + (scaled ? cons_scaled(KR) : 0);
  if (live) {
#pragma unroll
    for (int j = 0; j < L; ++j) out[KR + g * L + j] = y[j];
  }
  constexpr int E = 29 * KR;
  constexpr int TOP = 31 - __builtin_clz(E);
  M.dbl(y);   // x_1
  for (int b = TOP - 1; b >= 0; --b) {
    M.sqr_w(y, y);   // x_2a (almost Montgomery, < 2N)
    M.carry_exact(y);
    M.sub_if_ge(y);
    if ((E >> b) & 1) M.dbl(y);   // x_(a+1)
  }
  if (live) {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      out[g * L + j] = M.n[j];
      out[2 * KR + g * L + j] = y[j];
    }
  }
  if (g == 0) out[3 * KR] = M.ninv;
}

// dst = this lane's digits of table row d, read by scanning every row and keeping
// row d through a mask: the addresses and the instruction stream do not depend
// on d (a secret exponent's window digit).
template <int L>
__device__ __forceinline__ void ct_row(uint32_t* dst, const uint32_t* T, uint32_t d, uint32_t rows, int KD, int g) {
#pragma unroll
  for (int j = 0; j < L; ++j) dst[j] = 0u;
  for (uint32_t e = 0; e < rows; ++e) {
    const uint32_t m = 0u - (uint32_t)(e == d);
#pragma unroll
    for (int j = 0; j < L; ++j) dst[j] |= T[(size_t)e * KD + g * L + j] & m;
  }
}

// CT: the regular-access variant for secret exponents (a separate instantiation:
// its table scans would cost the throughput shapes occupancy).
// QS: the chain runs modulo N' = N (-N^-1 mod 2^29) with quotient-scaled rows
// (Mont29::row: the quotient digit is the retiring column, no multiply), from
// the N' block of the constants row; a^e mod N' = a^e mod N (mod N), and the
// exit product, a plain row pass modulo N, both leaves Montgomery form and
// reduces: (acc + m N) / R < N + 2N'/R <= N + 1.
template <int KD, int G, int K32, bool CT = false, bool QS = false>
__global__ __launch_bounds__(BLOCK) void modexp_kernel(const ModexpArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * (blockDim.x / G) + li;   // blocks of BLOCK or 64 threads (small launches)
  if (inst >= a.count) return;
  // a latency-critical launch sharing the chip with throughput launches on other
  // streams: its waves win the SIMD issue arbitration
  if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  uint32_t* stream = lds + li * KD;
  static_assert(!QS || (scaled_ok(KD, K32) && !CT), "quotient-scaled chains: public exponents, N' within R/4");
  const uint32_t* C0 = a.consts + (size_t)a.mod_idx[inst] * STRIDE;   // N: the exit product
  const uint32_t* C = QS ? C0 + cons_scaled(KD) : C0;                  // the chain's modulus
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = C[g * L + j];
  M.ninv = C[3 * KD];
  const uint32_t w = a.window;
  const uint32_t tsize = 1u << w;
  uint32_t* T = a.table + (size_t)inst * tsize * KD;
  const uint32_t* E = reinterpret_cast<const uint32_t*>(a.exp_ptr[inst]);
  const uint32_t exp_limbs = a.exp_len[inst];

  uint32_t acc[L];
  const uint32_t* B = reinterpret_cast<const uint32_t*>(a.base_ptr[inst]);
  const int blen = (int)min(a.base_len[inst], (uint32_t)K32);
#pragma unroll
  for (int j = 0; j < L; ++j) acc[j] = digit_of(B, blen, g * L + j);
#pragma unroll
  for (int j = 0; j < L; ++j) T[g * L + j] = C[KD + g * L + j];             // T[0] = R mod N
  // regular access (secret exponents): every instance runs the launch's window
  // count and every window-table read scans the whole table (ct_row below)
  const uint32_t nwin = (a.nwin_i && !CT) ? max(1u, a.nwin_i[inst]) : a.nwin;
  auto digit = [&](uint32_t k) -> uint32_t {
    const uint32_t p = (nwin - 1 - k) * w;
    const uint32_t lo = p >> 5, sh = p & 31;
    const uint32_t v0 = (lo < exp_limbs) ? E[lo] : 0u;
    const uint32_t v1 = (lo + 1 < exp_limbs) ? E[lo + 1] : 0u;
    return (uint32_t)(mk64(v0, v1) >> sh) & (tsize - 1);
  };
  // Every Montgomery product of the exponentiation is acc <- acc * stream, issued
  // from two sites (squaring rows for the ladder's squarings, plain rows for the
  // rest) so each unrolled product body exists once in the I-cache.
  //   step 0                      : stream = R^2            -> acc = xm, T[1] = xm
  //   step 1 .. tsize-2           : stream = T[1]           -> T[step+1]
  //   then per window k=1..nwin-1 : w x (stream = acc), then stream = T[d_k]
  //   last                        : stream = 1 (leave Montgomery form)
  const uint32_t n_build = tsize - 1;
  const uint32_t n_steps = n_build + (nwin - 1) * (w + 1) + 1;
  uint32_t k = 1, sub = 0;
  // QS: the last step (the exit product) runs after the loop with N's rows
  for (uint32_t st = 0; st < n_steps - (QS ? 1 : 0); ++st) {
    const uint32_t* src = nullptr;
    bool from_acc = false, one = false;
    if (st == n_build) {                                                    // start of the ladder
      const uint32_t d0 = digit(0);
      if constexpr (CT) ct_row<L>(acc, T, d0, tsize, KD, g);
      else {
#pragma unroll
        for (int j = 0; j < L; ++j) acc[j] = T[(size_t)d0 * KD + g * L + j];
      }
    }
    if (st >= n_build && st < n_steps - 1 && sub < w) {
      // the window's squarings in a loop of their own (no step logic or
      // register shuffles of the general step between them), then this
      // iteration continues as the window multiply
      for (; sub < w; ++sub, ++st) {
        __builtin_amdgcn_wave_barrier();
        lds_put<KD, G>(stream, acc, g);
        __builtin_amdgcn_wave_barrier();
        if constexpr (QS) M.sqr_s(acc, acc, stream);
        else M.sqr(acc, acc, stream);
      }
    }
    if (st == 0) {
      src = C + 2 * KD;
    } else if (st < n_build) {
      src = T + KD;
    } else if (st == n_steps - 1) {
      one = true;
    } else {
      if (sub < w) from_acc = true;
      else src = T + (size_t)digit(k) * KD;
    }
    __builtin_amdgcn_wave_barrier();
    if (from_acc) {
      lds_put<KD, G>(stream, acc, g);
    } else if (CT && st > n_build && st < n_steps - 1) {   // window multiply: scan the table
      uint32_t row[L];
      ct_row<L>(row, T, digit(k), tsize, KD, g);
      lds_put<KD, G>(stream, row, g);
    } else if (one) {
#pragma unroll
      for (int j = 0; j < L; ++j) stream[g * L + j] = (g == 0 && j == 0) ? 1u : 0u;
    } else {
#pragma unroll
      for (int j = 0; j < L; ++j) stream[g * L + j] = src[g * L + j];
    }
    __builtin_amdgcn_wave_barrier();
    if constexpr (QS) {
      if (from_acc) M.sqr_s(acc, acc, stream);
      else M.mul_s(acc, acc, stream);
    } else {
      if (from_acc) M.sqr(acc, acc, stream);   // the ladder's squarings: tournament rows
      else M.mul(acc, acc, stream);
    }
    if (st < n_build) {
#pragma unroll
      for (int j = 0; j < L; ++j) T[(size_t)(st + 1) * KD + g * L + j] = acc[j];
    } else if (st < n_steps - 1) {
      if (++sub == w + 1) { sub = 0; ++k; }
    }
  }
  if constexpr (QS) {   // exit: acc * 1 / R modulo N itself (acc = x R mod N' is x R mod N)
    // one window (an exponent below 2^w, e.g. 0 or 1): the loop above ends with
    // the table (st < n_steps - 1 = n_build), so the ladder start T[d0] is loaded here
    if (n_steps - 1 == n_build) {
      const uint32_t d0 = digit(0);
#pragma unroll
      for (int j = 0; j < L; ++j) acc[j] = T[(size_t)d0 * KD + g * L + j];
    }
#pragma unroll
    for (int j = 0; j < L; ++j) M.n[j] = C0[g * L + j];
    M.ninv = C0[3 * KD];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = (g == 0 && j == 0) ? 1u : 0u;
    __builtin_amdgcn_wave_barrier();
    M.mul(acc, acc, stream);
  }
  M.carry_exact(acc);
  M.sub_if_ge(acc);
  __builtin_amdgcn_wave_barrier();
  lds_put<KD, G>(stream, acc, g);
  __builtin_amdgcn_wave_barrier();
  uint32_t* O = a.out + (size_t)(a.out_idx ? a.out_idx[inst] : inst) * K32;
  constexpr int LO = K32 / G;
#pragma unroll
  for (int k = 0; k < LO; ++k) O[g * LO + k] = limb_of(stream, KD, g * LO + k);
}

// Sliding-window exponentiation for launches whose instances share their
// exponent within every wave (ModexpArgs.slide): the 2R chains s^N_i of
// receiver i in GA (the host orders them receiver-major), or a shared-exponent
// batch.  The schedule -- the odd powers x, x^3, .., x^(2^w - 1) (one squaring
// and 2^(w-1) - 1 products), then per 1 bit of the exponent a window of up to w
// bits ending in a 1 bit (its squarings and ONE product), a squaring per 0 bit
// between windows -- depends only on the exponent bits, so every lane of the
// wave takes the same path.  For a 2048-bit exponent at w = 6: 2048 squarings
// and ~325 other products instead of 2045 + 441 (fixed 5-bit windows).  Results
// are bit-identical to base^exp mod N.
// (at most 256 registers per lane: two waves per SIMD, like modexp_kernel's
// 4-lane shape; unbounded, the 4-lane schedule state took 256 VGPRs + 27 AGPRs)
template <int KD, int G, int K32, bool QS>
__global__ __launch_bounds__(BLOCK, 2) void modexp_slide_kernel(const ModexpArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  static_assert(!QS || scaled_ok(KD, K32), "quotient-scaled chains: N' within R/4");
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * (blockDim.x / G) + li;
  if (inst >= a.count) return;
  if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  uint32_t* stream = lds + li * KD;
  const uint32_t* C0 = a.consts + (size_t)a.mod_idx[inst] * STRIDE;
  const uint32_t* C = QS ? C0 + cons_scaled(KD) : C0;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = C[g * L + j];
  M.ninv = C[3 * KD];
  const uint32_t w = a.window, tw = 1u << (w - 1);   // odd powers T[0..tw), x^2 at T[tw]
  uint32_t* T = a.table + (size_t)inst * (tw + 1) * KD;
  // the wave's instances share the exponent (the caller's layout): its address
  // and length are made wave-uniform, so the window schedule below runs on the
  // scalar unit in SGPRs (per-lane copies held the 4-lane shape at 256 VGPRs +
  // 29 AGPRs, one wave per SIMD)
  const uint64_t ea = a.exp_ptr[inst];
  const uint32_t* E = reinterpret_cast<const uint32_t*>(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(ea >> 32)) << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ea));
  const int exp_limbs = __builtin_amdgcn_readfirstlane((int)a.exp_len[inst]);
  auto bit = [&](int i) -> uint32_t { return (E[i >> 5] >> (i & 31)) & 1u; };
  int top = 32 * exp_limbs - 1;
  while (top >= 0 && E[top >> 5] == 0) top = (top & ~31) - 1;   // skip zero limbs
  while (top >= 0 && !bit(top)) --top;
  // a head launch (lo > 0) runs the bits >= lo only (the tail kernel the rest)
  const int lo = (int)a.lo_bit;
  // the window that ends the run of bits at i (bit i set): lowest set bit jl >= i - w + 1
  auto window = [&](int i, int* jl) -> uint32_t {
    int j = max(i - (int)w + 1, lo);
    while (!bit(j)) ++j;
    uint32_t d = 0;
    for (int k = i; k >= j; --k) d = (d << 1) | bit(k);
    *jl = j;
    return d;   // odd
  };
  uint32_t acc[L];
  const uint32_t* B = reinterpret_cast<const uint32_t*>(a.base_ptr[inst]);
  const int blen = (int)min(a.base_len[inst], (uint32_t)K32);
#pragma unroll
  for (int j = 0; j < L; ++j) acc[j] = digit_of(B, blen, g * L + j);
  auto load = [&](const uint32_t* row) {
#pragma unroll
    for (int j = 0; j < L; ++j) acc[j] = row[g * L + j];
  };
  auto store = [&](uint32_t* row) {
#pragma unroll
    for (int j = 0; j < L; ++j) row[g * L + j] = acc[j];
  };
  // phase 0: x = base * R^2;  1: x^2;  2: T[jt] = T[jt-1] * x^2;  3: the windows
  int phase = top < 0 ? 4 : 0, i = top, pend_mul = -1;
  uint32_t jt = 1, pend_sq = 0;
  if (top < 0) load(C + KD);   // exponent 0: the Montgomery one
  while (phase < 4) {
    if (phase == 3) {
      // the squarings between two products in a loop of their own (a
      // window's, or a run of 0 bits): no schedule logic or register shuffles
      // of the general step between them (16 lanes: ~210 -> 90 VALU
      // instructions per squaring outside its cycle loop)
      if (pend_sq == 0 && pend_mul < 0)
        while (i >= lo && !bit(i)) {
          ++pend_sq;
          --i;
        }
      for (; pend_sq; --pend_sq) {
        __builtin_amdgcn_wave_barrier();
        lds_put<KD, G>(stream, acc, g);
        __builtin_amdgcn_wave_barrier();
        if constexpr (QS) M.sqr_s(acc, acc, stream);
        else M.sqr(acc, acc, stream);
      }
    }
    const uint32_t* src = nullptr;
    bool sq = false;
    if (phase == 0) {
      src = C + 2 * KD;
    } else if (phase == 1) {
      sq = true;
    } else if (phase == 2) {
      src = T + (size_t)tw * KD;
    } else if (pend_sq) {
      sq = true;
      --pend_sq;
    } else if (pend_mul >= 0) {
      src = T + (size_t)pend_mul * KD;
      pend_mul = -1;
    } else if (i < lo) {
      break;
    } else if (!bit(i)) {
      sq = true;
      --i;
    } else {
      int jl;
      const uint32_t d = window(i, &jl);
      pend_sq = (uint32_t)(i - jl + 1);
      pend_mul = (int)(d >> 1);
      i = jl - 1;
      continue;
    }
    __builtin_amdgcn_wave_barrier();
    if (sq) lds_put<KD, G>(stream, acc, g);
    else {
#pragma unroll
      for (int j = 0; j < L; ++j) stream[g * L + j] = src[g * L + j];
    }
    __builtin_amdgcn_wave_barrier();
    if constexpr (QS) {
      if (sq) M.sqr_s(acc, acc, stream);
      else M.mul_s(acc, acc, stream);
    } else {
      if (sq) M.sqr(acc, acc, stream);
      else M.mul(acc, acc, stream);
    }
    if (phase == 0) {
      store(T);
      phase = 1;
    } else if (phase == 1) {
      store(T + (size_t)tw * KD);
      load(T);
      phase = tw > 1 ? 2 : 3;
    } else if (phase == 2) {
      store(T + (size_t)jt * KD);
      if (++jt == tw) phase = 3;
    }
    if (phase == 3 && i == top) {   // the first window: its odd power, no squarings of 1
      if (top >= lo) {
        int jl;
        const uint32_t d = window(i, &jl);
        load(T + (size_t)(d >> 1) * KD);
        i = jl - 1;
      } else {   // a head whose bits are all below lo: 1 (the table is built for the tail)
        load(C + KD);
      }
    }
  }
  if (lo) {   // head: hand the accumulator (Montgomery form mod the chain's modulus) to the tail
#pragma unroll
    for (int j = 0; j < L; ++j) a.state[(size_t)inst * KD + g * L + j] = acc[j];
    return;
  }
  // exit: acc * 1 / R, modulo N itself for quotient-scaled chains
  if constexpr (QS) {
#pragma unroll
    for (int j = 0; j < L; ++j) M.n[j] = C0[g * L + j];
    M.ninv = C0[3 * KD];
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = (g == 0 && j == 0) ? 1u : 0u;
  __builtin_amdgcn_wave_barrier();
  M.mul(acc, acc, stream);
  M.carry_exact(acc);
  M.sub_if_ge(acc);
  __builtin_amdgcn_wave_barrier();
  lds_put<KD, G>(stream, acc, g);
  __builtin_amdgcn_wave_barrier();
  uint32_t* O = a.out + (size_t)(a.out_idx ? a.out_idx[inst] : inst) * K32;
  constexpr int LO = K32 / G;
#pragma unroll
  for (int k = 0; k < LO; ++k) O[g * LO + k] = limb_of(stream, KD, g * LO + k);
}

// The tail of a split chain (ModexpArgs lo_bit / tail): resumes the head's
// accumulator x^(E >> lo) and runs the exponent bits below lo with the head's
// sliding windows (wave-uniform E, the head's odd-power table), and with base2 set
// multiplies in base2^exp2 along the same squarings: 4-bit fixed windows of the
// instance's own exp2 (< 2^lo) over a 16-entry table base2^0..15.  GA's joint tail
// (collect_prepare.cpp): s2^N * c^-e_pdl and s^N * c^-e_A mod N^2 in one chain,
// base2 = c^-1, instead of a separate 256-bit chain c^e per proof and its inverse
// (zk_pdl_with_slack.rs:136-142 via commitment_unknown_order :170-188,
// range_proofs.rs:140-148).  QS as the head (the 8 / 16-lane shapes quotient-
// scaled, the 4-lane throughput shape plain).  Exact results.
template <int KD, int G, int K32, bool QS>
__global__ __launch_bounds__(BLOCK, 2) void modexp_tail_kernel(const ModexpArgs a) {
  using MT = Mont29<KD, G>;
  constexpr int L = MT::L;
  constexpr int IPB = BLOCK / G;
  constexpr int STRIDE = cons_stride(KD);
  static_assert(!QS || scaled_ok(KD, K32), "quotient-scaled chains: N' within R/4");
  __shared__ uint32_t lds[IPB * KD];
  const int g = threadIdx.x % G;
  const int li = threadIdx.x / G;
  const uint32_t inst = blockIdx.x * (blockDim.x / G) + li;
  if (inst >= a.count) return;
  if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  uint32_t* stream = lds + li * KD;
  const uint32_t* C0 = a.consts + (size_t)a.mod_idx[inst] * STRIDE;
  const uint32_t* C = QS ? C0 + cons_scaled(KD) : C0;
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = C[g * L + j];
  M.ninv = C[3 * KD];
  auto mulx = [&](uint32_t* x) {
    if constexpr (QS) M.mul_s(x, x, stream);
    else M.mul(x, x, stream);
  };
  const uint32_t w = a.window, tw = 1u << (w - 1);
  const uint32_t* T = a.table + (size_t)inst * (tw + 1) * KD;
  const uint64_t ea = a.exp_ptr[inst];
  const uint32_t* E = reinterpret_cast<const uint32_t*>(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(ea >> 32)) << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ea));
  const int exp_limbs = __builtin_amdgcn_readfirstlane((int)a.exp_len[inst]);
  auto bit = [&](int i) -> uint32_t { return (i >> 5) < exp_limbs ? (E[i >> 5] >> (i & 31)) & 1u : 0u; };
  const int lo = (int)a.lo_bit;
  uint32_t acc[L];
#pragma unroll
  for (int j = 0; j < L; ++j) acc[j] = a.state[(size_t)inst * KD + g * L + j];
  auto put_row = [&](const uint32_t* row) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < L; ++j) stream[g * L + j] = row[g * L + j];
    __builtin_amdgcn_wave_barrier();
  };
  // the joint base's table T2[u] = base2^u (Montgomery form), u < 16
  const bool joint = a.base2_ptr != nullptr;
  uint32_t* T2 = joint ? a.table2 + (size_t)inst * 16 * KD : nullptr;
  const uint32_t* E2 = nullptr;
  uint32_t e2len = 0;
  if (joint) {
    E2 = reinterpret_cast<const uint32_t*>(a.base2_ptr ? a.exp2_ptr[inst] : 0);
    e2len = a.exp2_len[inst];
    const uint32_t* B2 = reinterpret_cast<const uint32_t*>(a.base2_ptr[inst]);
    uint32_t y[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      y[j] = digit_of(B2, K32, g * L + j);
      T2[g * L + j] = C[KD + g * L + j];   // T2[0] = 1 (R mod N')
    }
    put_row(C + 2 * KD);                   // R^2: y -> y R
    mulx(y);
#pragma unroll
    for (int j = 0; j < L; ++j) T2[KD + g * L + j] = y[j];
    __builtin_amdgcn_wave_barrier();
    lds_put<KD, G>(stream, y, g);          // T2[1] streamed for the powers
    __builtin_amdgcn_wave_barrier();
    for (int u = 2; u < 16; ++u) {
      mulx(y);
#pragma unroll
      for (int j = 0; j < L; ++j) T2[(size_t)u * KD + g * L + j] = y[j];
    }
  }
  // bits lo-1 .. 0: square; the sliding window of E that ends at i multiplies
  // T[d >> 1] in; every 4th bit the instance's exp2 digit multiplies T2[digit] in
  int pend_at = -1;
  uint32_t pend_d = 0, ew = 0;
  for (int i = lo - 1; i >= 0; --i) {
    if ((i & 31) == 31 && joint) ew = ((uint32_t)(i >> 5) < e2len) ? E2[i >> 5] : 0u;
    if (pend_at < 0 && bit(i)) {   // a window starts: its lowest set bit jl >= max(i - w + 1, 0)
      int j = max(i - (int)w + 1, 0);
      while (!bit(j)) ++j;
      uint32_t d = 0;
      for (int k = i; k >= j; --k) d = (d << 1) | bit(k);
      pend_at = j;
      pend_d = d;
    }
    __builtin_amdgcn_wave_barrier();
    lds_put<KD, G>(stream, acc, g);
    __builtin_amdgcn_wave_barrier();
    if constexpr (QS) M.sqr_s(acc, acc, stream);
    else M.sqr(acc, acc, stream);
    if (i == pend_at) {
      put_row(T + (size_t)(pend_d >> 1) * KD);
      mulx(acc);
      pend_at = -1;
    }
    if (joint && (i & 3) == 0) {
      put_row(T2 + (size_t)((ew >> (i & 31)) & 15u) * KD);
      mulx(acc);
    }
  }
  // exit: acc * 1 / R modulo N itself
  if constexpr (QS) {
#pragma unroll
    for (int j = 0; j < L; ++j) M.n[j] = C0[g * L + j];
    M.ninv = C0[3 * KD];
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < L; ++j) stream[g * L + j] = (g == 0 && j == 0) ? 1u : 0u;
  __builtin_amdgcn_wave_barrier();
  M.mul(acc, acc, stream);
  M.carry_exact(acc);
  M.sub_if_ge(acc);
  __builtin_amdgcn_wave_barrier();
  lds_put<KD, G>(stream, acc, g);
  __builtin_amdgcn_wave_barrier();
  uint32_t* O = a.out + (size_t)(a.out_idx ? a.out_idx[inst] : inst) * K32;
  constexpr int LO = K32 / G;
#pragma unroll
  for (int k = 0; k < LO; ++k) O[g * LO + k] = limb_of(stream, KD, g * LO + k);
}

// One instance per wave64 (the latency shape of small launches, e.g. a
// multi-GPU rank's GA chains): lane g holds digits gL..gL+L-1 of every operand,
// KR digits in the first KR/L lanes and zeros above; the streamed operand of each
// Montgomery product is read from registers with v_readlane (Mont29::product_w),
// so the row digit and the quotient digit are wave-uniform and the quotient is
// computed on the scalar unit.  Constants are the KR-digit class's (mod_setup).
// Same exponentiation schedule as modexp_kernel; the window table is a global
// slab of KD-word entries; no LDS except the final limb conversion.
template <int KR, int L, int K32>
__global__ __launch_bounds__(64) void modexp_wave_kernel(const ModexpArgs a) {
  constexpr int KD = 64 * L;
  using MT = Mont29<KD, 64, KR>;
  constexpr int STRIDE = cons_stride(KR);
  __shared__ uint32_t lds[KD];
  const int g = threadIdx.x;
  const uint32_t inst = blockIdx.x;
  if (inst >= a.count) return;
  if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  const uint32_t* C = a.consts + (size_t)a.mod_idx[inst] * STRIDE;
  const bool live = g * L < KR;   // lanes holding digits of the KR-digit class
  MT M;
  M.init_lane(g);
#pragma unroll
  for (int j = 0; j < L; ++j) M.n[j] = live ? C[g * L + j] : 0u;
  M.ninv = (uint32_t)__builtin_amdgcn_readfirstlane((int)C[3 * KR]);
  const uint32_t w = a.window;
  const uint32_t tsize = 1u << w;
  uint32_t* T = a.table + (size_t)inst * tsize * KD;
  const uint32_t* E = reinterpret_cast<const uint32_t*>(a.exp_ptr[inst]);
  const uint32_t exp_limbs = a.exp_len[inst];
  uint32_t acc[L], opnd[L];
  const uint32_t* B = reinterpret_cast<const uint32_t*>(a.base_ptr[inst]);
  const int blen = (int)min(a.base_len[inst], (uint32_t)K32);
#pragma unroll
  for (int j = 0; j < L; ++j) acc[j] = digit_of(B, blen, g * L + j);   // 0 past the class's digits
#pragma unroll
  for (int j = 0; j < L; ++j) T[g * L + j] = live ? C[KR + g * L + j] : 0u;   // T[0] = R mod N
  const uint32_t nwin = a.nwin_i ? max(1u, a.nwin_i[inst]) : a.nwin;
  auto digit = [&](uint32_t k) -> uint32_t {
    const uint32_t p = (nwin - 1 - k) * w;
    const uint32_t lo = p >> 5, sh = p & 31;
    const uint32_t v0 = (lo < exp_limbs) ? E[lo] : 0u;
    const uint32_t v1 = (lo + 1 < exp_limbs) ? E[lo + 1] : 0u;
    return (uint32_t)(mk64(v0, v1) >> sh) & (tsize - 1);
  };
  // the schedule of modexp_kernel: R^2, table build, nwin-1 windows, exit by 1
  const uint32_t n_build = tsize - 1;
  const uint32_t n_steps = n_build + (nwin - 1) * (w + 1) + 1;
  uint32_t k = 1, sub = 0;
  for (uint32_t st = 0; st < n_steps; ++st) {
    if (st == n_build) {
      const uint32_t d0 = digit(0);
#pragma unroll
      for (int j = 0; j < L; ++j) acc[j] = T[(size_t)d0 * KD + g * L + j];
    }
    if (st >= n_build && st < n_steps - 1 && sub < w) {
      M.sqr_w(acc, acc);   // the ladder's squarings
    } else {
      const uint32_t* src = (st == 0) ? nullptr : (st < n_build) ? T + KD : (st == n_steps - 1) ? nullptr
                                                                            : T + (size_t)digit(k) * KD;
      if (st == 0) {
#pragma unroll
        for (int j = 0; j < L; ++j) opnd[j] = live ? C[2 * KR + g * L + j] : 0u;   // R^2 mod N
      } else if (!src) {
#pragma unroll
        for (int j = 0; j < L; ++j) opnd[j] = (g == 0 && j == 0) ? 1u : 0u;
      } else {
#pragma unroll
        for (int j = 0; j < L; ++j) opnd[j] = src[g * L + j];
      }
      M.mul_w(acc, acc, opnd);
    }
    if (st < n_build) {
#pragma unroll
      for (int j = 0; j < L; ++j) T[(size_t)(st + 1) * KD + g * L + j] = acc[j];
    } else if (st < n_steps - 1) {
      if (++sub == w + 1) { sub = 0; ++k; }
    }
  }
  M.carry_exact(acc);
  M.sub_if_ge(acc);
  lds_put<KD, 64>(lds, acc, g);
  __builtin_amdgcn_wave_barrier();
  uint32_t* O = a.out + (size_t)(a.out_idx ? a.out_idx[inst] : inst) * K32;
  for (int q = g; q < K32; q += 64) O[q] = limb_of(lds, KR, q);
}

// ---- host-side launchers -------------------------------------------------------
template <int KR, int L, int K32>
static hipError_t launch_setup_wave(const uint32_t* mods, uint32_t n_mod, uint32_t* consts, hipStream_t st) {
  const uint32_t waves = scaled_ok(KR, K32) ? 2 * n_mod : n_mod;
  if (waves == 0) return hipSuccess;
  hipLaunchKernelGGL((mod_setup_wave_kernel<KR, L, K32>), dim3(waves), dim3(64), 0, st, mods, n_mod, consts);
  return hipGetLastError();
}
template <int KD, int G, int K32>
static hipError_t launch_setup(const uint32_t* mods, uint32_t n_mod, uint32_t* consts, hipStream_t st) {
  constexpr int IPB = BLOCK / G;
  const uint32_t inst = scaled_ok(KD, K32) ? 2 * n_mod : n_mod;
  const uint32_t blocks = (inst + IPB - 1) / IPB;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((mod_setup_kernel<KD, G, K32>), dim3(blocks), dim3(BLOCK), 0, st, mods, n_mod, consts);
  return hipGetLastError();
}
// A launch with fewer waves than the chip has SIMDs runs one wave per block,
// so the dispatcher can give every wave its own SIMD (a latency-bound chain
// sharing a SIMD with another wave runs up to 2x slower).
constexpr uint32_t kSmallLaunchLanes = 256u * 4u * 64u;
static inline uint32_t block_threads(uint32_t lanes) { return lanes <= kSmallLaunchLanes ? 64u : (uint32_t)BLOCK; }

template <int KD, int G, int K32, bool CT = false, bool QS = false>
static hipError_t launch_modexp(const ModexpArgs& a, hipStream_t st) {
  const uint32_t bs = block_threads(a.count * G);
  const uint32_t ipb = bs / G;
  const uint32_t blocks = (a.count + ipb - 1) / ipb;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((modexp_kernel<KD, G, K32, CT, QS>), dim3(blocks), dim3(bs), 0, st, a);
  return hipGetLastError();
}

template <int KD, int G, int K32, bool QS>
static hipError_t launch_modexp_slide(const ModexpArgs& a, hipStream_t st) {
  const uint32_t bs = block_threads(a.count * G);
  const uint32_t ipb = bs / G;
  const uint32_t blocks = (a.count + ipb - 1) / ipb;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((modexp_slide_kernel<KD, G, K32, QS>), dim3(blocks), dim3(bs), 0, st, a);
  return hipGetLastError();
}

template <int KD, int G, int K32, bool QS>
static hipError_t launch_modexp_tail(const ModexpArgs& a, hipStream_t st) {
  const uint32_t bs = block_threads(a.count * G);
  const uint32_t ipb = bs / G;
  const uint32_t blocks = (a.count + ipb - 1) / ipb;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((modexp_tail_kernel<KD, G, K32, QS>), dim3(blocks), dim3(bs), 0, st, a);
  return hipGetLastError();
}

template <int KR, int L, int K32>
static hipError_t launch_modexp_wave(const ModexpArgs& a, hipStream_t st) {
  if (a.count == 0) return hipSuccess;
  hipLaunchKernelGGL((modexp_wave_kernel<KR, L, K32>), dim3(a.count), dim3(64), 0, st, a);
  return hipGetLastError();
}

// The same constants from one wave per modulus (mod_setup_wave_kernel) where a
// width has that shape: 3072-bit moduli.  Used for the multi-session prestart's
// table chains, whose setup otherwise waits for a whole free slot beside GA.
hipError_t mod_setup_wave(uint32_t k32, const uint32_t* mods, uint32_t n_mod, uint32_t* consts, hipStream_t st) {
  if (k32 == 96) return launch_setup_wave<108, 2, 96>(mods, n_mod, consts, st);
  return mod_setup(k32, mods, n_mod, consts, st);
}

int shape_digits(uint32_t k32) {
  switch (k32) {
    case 64: return 72;
    case 96: return 108;
    case 128: return 144;
    case 192: return 216;
    default: return 0;
  }
}

int shape_digits_g(uint32_t k32, uint32_t group) {
  if (k32 == kPrimeLimbs) return 36;   // key generation only (1024-bit primes)
  return (k32 == 128 && group == kWideGroup) ? 160 : shape_digits(k32);
}

int table_digits(uint32_t k32, uint32_t group) {
  if (k32 == 128 && group == kWaveGroup) return 192;   // 64 lanes x 3 slots
  return shape_digits_g(k32, group);
}

hipError_t mod_setup_g(uint32_t k32, uint32_t group, const uint32_t* mods, uint32_t n_mod, uint32_t* consts,
                       hipStream_t st) {
  if (k32 == 128 && group == kWideGroup) return launch_setup<160, 8, 128>(mods, n_mod, consts, st);
  return mod_setup(k32, mods, n_mod, consts, st);
}

// The constants depend on KD only (exact values), so the setup runs in a light
// shape: few VGPRs and little LDS, so a setup at the head of a job's chain is
// dispatched beside long-running waves instead of waiting for a whole free slot
// (the 2-lane 2048-bit setup took 222 VGPRs and 36 KB per block and waited up to
// 29 ms behind an 8-way n = 256 rank's GA, profiles/r04/r04ad_*).
hipError_t mod_setup(uint32_t k32, const uint32_t* mods, uint32_t n_mod, uint32_t* consts, hipStream_t st) {
  switch (k32) {
    case 32: return launch_setup<36, 2, 32>(mods, n_mod, consts, st);
    case 64: return launch_setup<72, 8, 64>(mods, n_mod, consts, st);
    case 96: return launch_setup<108, 4, 96>(mods, n_mod, consts, st);
    case 128: return launch_setup<144, 16, 128>(mods, n_mod, consts, st);
    case 192: return launch_setup<216, 8, 192>(mods, n_mod, consts, st);
    default: return hipErrorInvalidValue;
  }
}

// Lanes per instance.  A launch that cannot fill the chip runs with more lanes
// per instance for lower latency: the largest G whose lanes still fit the
// resident-wave capacity.  Past that capacity the throughput shape: 2048-bit
// G = 4 (L = 18: no in-cycle normalisation, profiles/r01_modexp_group_sweep_*),
// 4096-bit G = 4 (L = 36; with squaring rows it edges out L = 18 by 4%,
// profiles/r02h_modexp_sqr.jsonl).  G = 2 (2048-bit) only when forced.
// ModexpArgs.group (fsdkr_ctx_set_modexp_group) forces a group size (tuning, tests).
static int pick_group(uint32_t count, int forced, std::initializer_list<int> allowed, int min_auto) {
  for (int g : allowed)
    if (g == forced) return g;
  constexpr uint64_t kLaneCapacity = 256ull * 4 * 3 * 64;   // CUs x SIMDs x resident waves x lanes
  int best = min_auto;
  for (int g : allowed)
    if (g > best && (uint64_t)count * (uint64_t)g <= kLaneCapacity) best = g;
  return best;
}

hipError_t modexp(uint32_t k32, const ModexpArgs& a, hipStream_t st) {
  if (a.ct) {   // secret exponents: one regular-access shape per width
    if (a.group == kWideGroup) return hipErrorInvalidValue;
    switch (k32) {
      case 32: return launch_modexp<36, 4, 32, true>(a, st);
      case 64: return launch_modexp<72, 8, 64, true>(a, st);   // small launches (decryption): 8 lanes
      case 96: return launch_modexp<108, 4, 96, true>(a, st);
      case 128: return launch_modexp<144, 8, 128, true>(a, st);
      case 192: return launch_modexp<216, 8, 192, true>(a, st);
      default: return hipErrorInvalidValue;
    }
  }
  // public exponents run quotient-scaled chains (modexp_kernel QS: no quotient
  // multiply per row) at every group shape: 8-32 lanes since round 4, the 4-lane
  // throughput shapes since round 5 (metric 2 -1.5 % keyed, -0.9 % per-instance
  // exponents, interleaved, profiles/r05/r05qs4_*)
  if (a.slide) {   // shared exponent per wave: the 4096-bit shapes of GA
    if (k32 != 128 || a.ct || a.group == kWaveGroup) return hipErrorInvalidValue;
    if (a.group == kWideGroup) {   // 32 lanes (KD = 160 constants, the caller's): small launches
      if (a.lo_bit && a.tail)
        return launch_modexp_tail<160, 32, 128, true>(a, st);
      return launch_modexp_slide<160, 32, 128, true>(a, st);
    }
    if (a.lo_bit) {   // split chains: head and tail at the caller's lanes, QS as the full chain's
      switch (a.group) {
        case 16: return a.tail ? launch_modexp_tail<144, 16, 128, true>(a, st)
                               : launch_modexp_slide<144, 16, 128, true>(a, st);
        case 8: return a.tail ? launch_modexp_tail<144, 8, 128, true>(a, st)
                              : launch_modexp_slide<144, 8, 128, true>(a, st);
        case 4: return a.tail ? launch_modexp_tail<144, 4, 128, true>(a, st)
                              : launch_modexp_slide<144, 4, 128, true>(a, st);
        default: return hipErrorInvalidValue;
      }
    }
    switch (pick_group(a.count, (int)a.group, {4, 8, 16}, 4)) {
      case 16: return launch_modexp_slide<144, 16, 128, true>(a, st);
      case 8: return launch_modexp_slide<144, 8, 128, true>(a, st);
      default: return launch_modexp_slide<144, 4, 128, true>(a, st);
    }
  }
  switch (k32) {
    case 32:   // 1024-bit primes of key generation: L = 9 (4 lanes) or 18
      return pick_group(a.count, (int)a.group, {2, 4}, 4) == 2 ? launch_modexp<36, 2, 32>(a, st)
                                                              : launch_modexp<36, 4, 32>(a, st);
    case 64:
      switch (pick_group(a.count, (int)a.group, {2, 4, 8}, 4)) {
        case 8: return launch_modexp<72, 8, 64, false, true>(a, st);
        case 4: return launch_modexp<72, 4, 64, false, true>(a, st);
        default: return launch_modexp<72, 2, 64>(a, st);
      }
    case 96: return launch_modexp<108, 4, 96, false, true>(a, st);
    case 128:
      // 32 lanes only on explicit request: it needs KD = 160 constants (mod_setup_g)
      if (a.group == kWideGroup)
        return launch_modexp<160, 32, 128, false, true>(a, st);
      if (a.group == kWaveGroup) return launch_modexp_wave<144, 3, 128>(a, st);
      // a launch past the resident-lane capacity: 4 lanes (L = 36, squaring rows
      // with 19 + 36 MACs per row) beat 8 (L = 18) by 4% (profiles/r02h_modexp_sqr.jsonl)
      switch (pick_group(a.count, (int)a.group, {4, 8, 16}, 4)) {
        case 16: return launch_modexp<144, 16, 128, false, true>(a, st);
        case 8: return launch_modexp<144, 8, 128, false, true>(a, st);
        default: return launch_modexp<144, 4, 128, false, true>(a, st);
      }
    case 192:
      if (pick_group(a.count, (int)a.group, {4, 8}, 4) == 8)
        return launch_modexp<216, 8, 192, false, true>(a, st);
      return launch_modexp<216, 4, 192, false, true>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace fsdkr
