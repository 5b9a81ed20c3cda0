// Lane-distributed radix-2^29 Montgomery arithmetic for gfx950 (CDNA4, wave64).
//
// Why radix 2^29: on gfx950 v_mad_u64_u32 and every carry-writing add issue at
// half rate (tools/microbench, profiles/r01_intrates.jsonl), so a radix-2^32
// CIOS costs two half-rate instructions per MAC.  With 29-bit digits a product
// is < 2^58 and a 64-bit column accumulator absorbs 31 rows of products, so the
// inner loop is ONE v_mad_u64_u32 per MAC with no carry chain; carries are
// resolved by a cheap parallel normalisation every 18 rows.
//
// Layout: a KD-digit integer is owned by G consecutive lanes (G in {2,4,8,16}:
// one DPP quad or part of one 16-lane DPP row; G = 32: two rows, see below); lane g holds digits
// [g*L, g*L+L), L = KD/G.  Larger G = lower latency per instance (small
// batches), smaller G = fewer cross-lane ops per MAC (full chip).  Row-oriented CIOS:
// row i broadcasts digit a_i of the streamed operand (LDS) to the group, every
// lane adds a_i*b and m_i*n into its L column accumulators, lane 0 folds the
// retired column's carry and the accumulator shifts one digit down (register
// slot rotation inside an L-row unrolled cycle plus one 64-bit DPP move).
//
// Values are kept "almost Montgomery": R = 2^(29*KD) > 4N, operands < 2N with
// digits <= 2^29+127, outputs < 2N; exact reduction happens once per modexp.
//
// This replaces GMP mpz_powm/mpz_mul/mpz_mod behind curv BigInt::mod_pow and
// BigInt::mod_mul (curv-kzen 0.10, /root/reference/Cargo.toml:33,41-44) on the
// collect() hot path (/root/reference/src/refresh_message.rs:321-467).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <utility>

#include "kernels.h"

namespace fsdkr {

constexpr uint32_t M29 = (1u << 29) - 1;
#ifndef FSDKR_ROW_FENCE_MIN_L
#define FSDKR_ROW_FENCE_MIN_L 12
#endif

// ---- intra-group DPP helpers --------------------------------------------------
// G <= 4: quad_perm inside one DPP quad.  G = 8/16: row_shr/row_shl:1 inside a
// 16-lane row (group boundaries masked by the caller), row_newbcast:n for the
// broadcasts (two bank-masked moves for the two 8-lane groups of a row).
// bound_ctrl set: a lane whose source is outside the row reads 0 (the old value
// is undefined for these moves anyway), and the DPP-combine pass may then fold
// the move into the VALU op that consumes it (`dpp(x) & y` as one v_and_b32_dpp)
#define FSDKR_DPP(v, ctrl) ((uint32_t)__builtin_amdgcn_mov_dpp((int)(v), (ctrl), 0xF, 0xF, true))
#define FSDKR_DPP_BANK(old, v, ctrl, bank) \
  ((uint32_t)__builtin_amdgcn_update_dpp((int)(old), (int)(v), (ctrl), 0xF, (bank), false))

// G = 32 (4096-bit latency shape, two instances per wave): the group spans two
// DPP rows, so the carry moves use the GFX9 wavefront shifts (wave_shl/shr:1)
// and the lane-0 broadcast is row_newbcast:0 followed by row_bcast:15 into the
// odd rows.
template <int G>
__device__ __forceinline__ uint32_t bcast_lane0(uint32_t v) {
  if constexpr (G == 1) return v;
  else if constexpr (G == 64) return (uint32_t)__builtin_amdgcn_readlane((int)v, 0);   // wave-uniform (SGPR)
  else if constexpr (G == 32) {
    const uint32_t t = FSDKR_DPP(v, 0x150);                                   // row_newbcast:0
    return (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)t, 0x142, 0xA, 0xF, false);   // row_bcast:15 -> rows 1, 3
  }
  else if constexpr (G == 2) return FSDKR_DPP(v, 0xA0);   // [0,0,2,2]
  else if constexpr (G == 4) return FSDKR_DPP(v, 0x00);   // [0,0,0,0]
  else if constexpr (G == 8) return FSDKR_DPP_BANK(FSDKR_DPP(v, 0x150), v, 0x158, 0xC);   // lane 0, then lane 8 into 8..15
  else return FSDKR_DPP(v, 0x150);                        // row_newbcast:0
}
template <int G>
__device__ __forceinline__ uint32_t bcast_top(uint32_t v) {
  if constexpr (G == 1) return v;
  else if constexpr (G == 64) return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
  else if constexpr (G == 32) return (uint32_t)__shfl((int)v, (int)((__lane_id() & ~31u) + 31u));   // rare: once per modexp
  else if constexpr (G == 2) return FSDKR_DPP(v, 0xF5);   // [1,1,3,3]
  else if constexpr (G == 4) return FSDKR_DPP(v, 0xFF);   // [3,3,3,3]
  else if constexpr (G == 8) return FSDKR_DPP_BANK(FSDKR_DPP_BANK(v, v, 0x157, 0x3), v, 0x15F, 0xC);
  else return FSDKR_DPP(v, 0x15F);                        // row_newbcast:15
}
// raw value of lane g+1 (top lane: caller masks)
template <int G>
__device__ __forceinline__ uint32_t dpp_next(uint32_t v) {
  if constexpr (G == 1) return v;
  else if constexpr (G == 32 || G == 64) return FSDKR_DPP(v, 0x130);   // wave_shl:1 (lane 63 reads 0)
  else if constexpr (G == 2) return FSDKR_DPP(v, 0xF5);   // [1,1,3,3]
  else if constexpr (G == 4) return FSDKR_DPP(v, 0xF9);   // [1,2,3,3]
  else return FSDKR_DPP(v, 0x101);                        // row_shl:1
}
// raw value of lane g-1 (lane 0: caller masks)
template <int G>
__device__ __forceinline__ uint32_t dpp_prev(uint32_t v) {
  if constexpr (G == 1) return v;
  else if constexpr (G == 32 || G == 64) return FSDKR_DPP(v, 0x138);   // wave_shr:1 (lane 0 reads 0)
  else if constexpr (G == 2) return FSDKR_DPP(v, 0xA0);   // [0,0,2,2]
  else if constexpr (G == 4) return FSDKR_DPP(v, 0x90);   // [0,0,1,2]
  else return FSDKR_DPP(v, 0x111);                        // row_shr:1
}
// value of lane g+1, rotating within the group (the top lane reads lane 0), where
// one DPP move does it (G = 2, 4: quad_perm; G = 16: row_ror:15); HAS_ROT<G>
template <int G>
constexpr bool HAS_ROT = G == 2 || G == 4 || G == 16;
template <int G>
__device__ __forceinline__ uint32_t dpp_next_rot(uint32_t v) {
  static_assert(HAS_ROT<G>, "no single-move rotation for this group size");
  if constexpr (G == 2) return FSDKR_DPP(v, 0xB1);        // [1,0,3,2]
  else if constexpr (G == 4) return FSDKR_DPP(v, 0x39);   // [1,2,3,0]
  else return FSDKR_DPP(v, 0x12F);                        // row_ror:15
}
// group-wide max over the G lanes
template <int G>
__device__ __forceinline__ int group_max(int v) {
  if constexpr (G >= 2) v = max(v, (int)FSDKR_DPP(v, 0xB1));   // [1,0,3,2]
  if constexpr (G >= 4) v = max(v, (int)FSDKR_DPP(v, 0x4E));   // [2,3,0,1]
  if constexpr (G >= 8) v = max(v, (int)FSDKR_DPP(v, 0x141));  // row_half_mirror
  if constexpr (G >= 16) v = max(v, (int)FSDKR_DPP(v, 0x140)); // row_mirror
  if constexpr (G >= 32) v = max(v, __shfl_xor(v, 16));
  if constexpr (G >= 64) v = max(v, __shfl_xor(v, 32));
  return v;
}

__device__ __forceinline__ uint64_t mk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

// acc += a * b  -> one v_mad_u64_u32 (callers guarantee acc never exceeds 2^64).
__device__ __forceinline__ void mac(uint64_t& acc, uint32_t a, uint32_t b) {
  acc += (uint64_t)a * b;
}

// Make N register values opaque to the optimiser at this point (no code).  Used
// at the top of each product cycle so LLVM cannot hoist zext(digit) out of the
// cycle loop: a hoisted i64 zext is a cross-block value that ISel materialises
// as a VGPR pair per digit (+2L VGPRs for b and n), instead of folding it into
// each v_mad_u64_u32's 32-bit source operand.
template <int N>
__device__ __forceinline__ void opaque(uint32_t* v) {
#pragma unroll
  for (int j = 0; j + 3 < N; j += 4) asm volatile("" : "+v"(v[j]), "+v"(v[j + 1]), "+v"(v[j + 2]), "+v"(v[j + 3]));
#pragma unroll
  for (int j = N - N % 4; j < N; ++j) asm volatile("" : "+v"(v[j]));
}

// KR: digits of the modulus class (rows of a product, R = 2^(29 KR)); KD >= KR
// register slots over the G lanes.  KD > KR only for G = 64 (one instance per
// wave), whose top lanes hold zero digits.
template <int KD, int G, int KR = KD>
struct Mont29 {
  static constexpr int L = KD / G;
  static_assert(KD % G == 0, "KD must split evenly over the group");
  static_assert(KR == KD || (G == 64 && KR % L == 0 && KR < KD), "spare slots only in the wave shape");
  // A column spends exactly L rows in a lane and leaves it as a 29-bit digit
  // (row(): the retired column's carry stays behind).  Each row adds at most one
  // a*b and one m*n product to it (< 2^58.01 each), so a product cycle adds
  // < L 2^59.01.  A squaring row may add 2 a_r b_j instead (sq_dbl), but over the
  // column's L rows the tournament offset d = (j - r) mod L steps by -2 per row:
  // for odd L it takes every residue once ((L-1)/2 doubled, one raw, (L-1)/2
  // none), for even L one parity class twice (at most L - 2 doubled units and 4
  // raw), so the a*b part stays <= (L + 2) 2^58.01 and the column
  // < (L + 1) 2^59.01 + 2^35 (the carry it receives as the lane's second
  // column).  For L <= 30 that is < 2^64 (2^63.96): no carries inside the cycle,
  // only the final carry passes of mul().  (Round 5 folded from L > 24 on the
  // per-row worst case 2^59.6; profiles/r06/r06n_*.)
  static constexpr bool NORM_IN_CYCLE = L > 30;
  // Longer lanes fold the column at logical position P_k into P_k + 1 once per
  // row (rolling normalisation, roll_norm), so every column is folded once per
  // fold point during its L-row stay and accumulates at most 18 rows between
  // folds (bound: 21 squaring rows).  That is NROLL column folds per row
  // instead of a full L-column carry pass every 18 rows (2L per 36 rows).
  static constexpr int NROLL = NORM_IN_CYCLE ? (L + 17) / 18 - 1 : 0;
  static constexpr int roll_pos(int k) { return (k + 1) * L / (NROLL + 1); }
  // Scheduling fence at the end of each row.  Long lanes (throughput shapes,
  // 3 waves/SIMD) need it to hold VGPRs down; short lanes (latency shapes, one
  // wave per SIMD) drop it so the next row's a*b products can fill the m-digit
  // dependency chain (v_mul_lo -> DPP broadcast -> m*n[0] -> carry).
  static constexpr bool ROW_FENCE = L > FSDKR_ROW_FENCE_MIN_L;

  uint32_t n[L];
  uint32_t ninv;      // -N^-1 mod 2^29
  int g;
  uint32_t m_lane0;   // ~0 in group lane 0
  uint32_t m_first;   // ~0 unless lane 0   (masks dpp_prev)
  uint32_t m_top;     // ~0 unless top lane (masks dpp_next)
  uint32_t eight;     // 8 in an SGPR (roll_fold)
  uint32_t m29;       // M29 in a VGPR: DPP-combined v_and_b32 needs a VGPR operand
  uint32_t m_top29;   // M29 unless top lane (the digit moving down, masked in one v_and_b32_dpp)

  __device__ __forceinline__ void init_lane(int g_) {
    g = g_;
    m_lane0 = (g == 0) ? 0xFFFFFFFFu : 0u;
    m_first = (g == 0) ? 0u : 0xFFFFFFFFu;
    m_top = (g == G - 1) ? 0u : 0xFFFFFFFFu;
    // keep the masks as plain values so `x & mask` stays one full-rate v_and
    // (the optimiser otherwise rewrites it into v_cndmask on a lane predicate)
    asm volatile("" : "+v"(m_lane0), "+v"(m_first), "+v"(m_top));
    eight = 8u;
    m29 = M29;
    m_top29 = m_top & M29;
    asm volatile("" : "+s"(eight), "+v"(m29), "+v"(m_top29));
  }

  __device__ __forceinline__ uint64_t prev64(uint64_t v) const {
    return mk64(dpp_prev<G>((uint32_t)v) & m_first, dpp_prev<G>((uint32_t)(v >> 32)) & m_first);
  }
  __device__ __forceinline__ uint64_t next64(uint64_t v) const {
    return mk64(dpp_next<G>((uint32_t)v) & m_top, dpp_next<G>((uint32_t)(v >> 32)) & m_top);
  }

  // one parallel carry step over the logical columns (slot of logical j = (j+RHO)%L)
  template <int RHO>
  __device__ __forceinline__ void norm_step(uint64_t* acc) const {
    const uint64_t cin = prev64(acc[(L - 1 + RHO) % L] >> 29);
    // descending so each column reads its lower neighbour before that one is
    // rewritten; sched barriers every 6 columns stop the scheduler from
    // hoisting all L shifts at once (that alone costs 2L VGPRs)
#pragma unroll
    for (int j = L - 1; j > 0; --j) {
      const int s = (j + RHO) % L, sp = (j - 1 + RHO) % L;
      acc[s] = (uint64_t)((uint32_t)acc[s] & M29) + (acc[sp] >> 29);
      if (j % 6 == 0) __builtin_amdgcn_sched_barrier(0);
    }
    acc[RHO % L] = (uint64_t)((uint32_t)acc[RHO % L] & M29) + cin;
    __builtin_amdgcn_sched_barrier(0);
  }

  // Rolling normalisation at rotation R: the column at logical position P moves
  // its high word into position P + 1 (same lane: P + 1 < L), one v_mad_u64_u32
  // by 8 (2^32 = 8 * 2^29) and one move that clears the high word.  The folded
  // column keeps < 2^32, the receiving one gains < 2^35; values are unchanged.
  template <int R, int K>
  __device__ __forceinline__ void roll_fold(uint64_t* acc) const {
    constexpr int P = roll_pos(K);
    static_assert(P >= 2 && P + 1 < L, "fold points stay inside the lane, clear of the retiring column");
    constexpr int sp = (P + R) % L, sn = (P + 1 + R) % L;
    const uint32_t hi = (uint32_t)(acc[sp] >> 32);
    acc[sp] = (uint64_t)(uint32_t)acc[sp];
    mac(acc[sn], hi, eight);   // a v_mad_u64_u32 by an opaque 8, not a 64-bit shift-add
  }
  template <int R, int... Ks>
  __device__ __forceinline__ void roll_norm(uint64_t* acc, std::integer_sequence<int, Ks...>) const {
    (roll_fold<R, Ks>(acc), ...);
  }

  // Squaring rows (SQ): of the pair products a_r a_p (p = g L + j) a row issues
  // only the slots of a cyclic tournament over d = (j - r) mod L, uniform across
  // the group's lanes (r mod L = R is a compile-time row of the cycle):
  //   d = 0                        a_r   * a_p   (the diagonal, and the pairs
  //                                               p = r mod L of other lanes,
  //                                               issued from both rows)
  //   1 <= d < L/2 (L odd: <= L/2)  2 a_r * a_p   (row p skips this pair)
  //   d = L/2 (L even)             a_r   * a_p   (both rows issue it)
  // so every unordered pair is counted twice and every a_r^2 once: (L+1)/2
  // (L odd) or L/2 + 1 (L even) MACs per row instead of L.  A pair {r, p} is
  // issued in a row <= r + p, so the column a row retires holds the same value
  // as in the plain product: identical m digits, bit-identical results.  A
  // column gains < 2^59.6 in one row (2 a_r < 2^30.01), but < (L + 1) 2^59.01
  // over its L-row stay in a lane (NORM_IN_CYCLE), as in the plain product.
  static constexpr bool sq_raw(int d) { return d == 0 || (L % 2 == 0 && d == L / 2); }
  static constexpr bool sq_dbl(int d) { return d > 0 && (L % 2 == 1 ? d <= L / 2 : d < L / 2); }
  // Short-lane group shapes (8-32 lanes) keep the doubled digits 2 b_j of a
  // squaring in registers for the whole product (L shifts per product instead
  // of one per row); the long-lane shapes cannot spare the L VGPRs, and the
  // wave shape doubles its SGPR row digit on the scalar unit.
  static constexpr bool USE_B2 = G >= 8 && G < 64;
  static constexpr int NB2 = USE_B2 ? L : 1;

  // a_r * b_j into slot (j + R) % L (squaring rows: the tournament slots only;
  // 2 a_r b_j as a_r * (2 b_j) when the doubled digits are held, USE_B2)
  template <int R, bool SQ, int J>
  __device__ __forceinline__ void mac_ab(uint64_t* acc, const uint32_t* b, const uint32_t* b2, uint32_t ai,
                                         uint32_t a2) const {
    if constexpr (SQ) {
      constexpr int d = (J - R % L + L) % L;
      if constexpr (sq_raw(d)) mac(acc[(J + R) % L], ai, b[J]);
      else if constexpr (sq_dbl(d)) {
        if constexpr (USE_B2) mac(acc[(J + R) % L], ai, b2[J]);
        else mac(acc[(J + R) % L], a2, b[J]);
      }
    } else {
      mac(acc[(J + R) % L], ai, b[J]);
    }
  }
  template <int R, bool SQ, int... Js>
  __device__ __forceinline__ void mac_ab_rest(uint64_t* acc, const uint32_t* b, const uint32_t* b2, uint32_t ai,
                                              uint32_t a2, std::integer_sequence<int, Js...>) const {
    (mac_ab<R, SQ, Js + 1>(acc, b, b2, ai, a2), ...);
  }

  // One CIOS row at rotation R (logical column j lives in slot (j+R)%L).  For
  // the long-lane throughput shapes (ORDERED: L > FSDKR_ROW_FENCE_MIN_L with a
  // rotating DPP move, i.e. G = 2 / 4) the order is fixed by scheduling barriers
  // so every dependent step has independent MACs between it and its producer (no
  // s_nop before the DPP moves, the quotient's v_mul_lo latency hidden):
  //   a_r*b_0 (the retiring column s0), m = s0 * n' (lane-local), a_r*b_1..L-1,
  //   broadcast m, m*n_0, carry/digit of s0, m*n_1, carry into s1, m*n_2..L-1,
  //   the retired digit moves down one lane.
  // Short lanes (latency shapes) keep the compiler's order, which interleaves
  // consecutive rows (measured: the fixed order cost 4-8 % at 8 lanes,
  // profiles/r03d_row_order_ab.txt).
  static constexpr bool ORDERED = HAS_ROT<G> && L > FSDKR_ROW_FENCE_MIN_L;
  // QS (quotient-scaled rows): the modulus is N' = N (-N^-1 mod 2^29), so
  // -N'^-1 = 1 mod 2^29 and the quotient digit is the retiring column itself:
  // no v_mul_lo_u32 on the row's dependency chain, and its mask folds into the
  // broadcast (mul_s / sqr_s; the group shapes only).
  template <int R, bool SQ, bool QS = false>
  __device__ __forceinline__ void row(uint64_t* acc, const uint32_t* b, const uint32_t* b2, const uint32_t* n,
                                      uint32_t ai) const {
    constexpr int s0 = R % L, s1 = (R + 1) % L;
    const uint32_t a2 = (SQ && !USE_B2) ? ai << 1 : 0u;
    if constexpr (ORDERED) {
      mac_ab<R, SQ, 0>(acc, b, b2, ai, a2);
      // QS: the retiring column is the quotient (no v_mul_lo_u32)
      uint32_t m = QS ? (uint32_t)acc[s0] : (uint32_t)acc[s0] * ninv;
      __builtin_amdgcn_sched_barrier(0);
      mac_ab_rest<R, SQ>(acc, b, b2, ai, a2, std::make_integer_sequence<int, L - 1>{});
      __builtin_amdgcn_sched_barrier(0);
      m = bcast_lane0<G>(m) & m29;   // one v_and_b32 with the DPP broadcast folded in
      mac(acc[s0], m, n[0]);
      uint64_t carry = acc[s0] >> 29;
      uint32_t digit = (uint32_t)acc[s0];
      asm volatile("" : "+v"(digit), "+v"(carry));   // computed here, not sunk to their uses
      __builtin_amdgcn_sched_barrier(0);
      mac(acc[s1], m, n[1]);
      acc[s1] += carry;
#pragma unroll
      for (int j = 2; j < L; ++j) mac(acc[(j + R) % L], m, n[j]);
      roll_norm<R>(acc, std::make_integer_sequence<int, NROLL>{});
      __builtin_amdgcn_sched_barrier(0);
      acc[s0] = (uint64_t)(dpp_next_rot<G>(digit) & m29);   // lane 0's digit is 0: the top lane gets the 0 it needs
    } else {
      static_assert(!QS || G < 64, "quotient-scaled rows: group shapes of 8-32 lanes");
      mac_ab<R, SQ, 0>(acc, b, b2, ai, a2);
      mac_ab_rest<R, SQ>(acc, b, b2, ai, a2, std::make_integer_sequence<int, L - 1>{});
      // G = 64: the instance is the wave, so m is computed on the scalar unit
      // from lane 0's column (ninv is an SGPR there)
      const uint32_t m = (G == 64) ? ((bcast_lane0<G>((uint32_t)acc[s0]) * ninv) & M29)
                         : QS      ? (bcast_lane0<G>((uint32_t)acc[s0]) & m29)
                                   : (bcast_lane0<G>((uint32_t)acc[s0] * ninv) & m29);
#pragma unroll
      for (int j = 0; j < L; ++j) mac(acc[(j + R) % L], m, n[j]);
      roll_norm<R>(acc, std::make_integer_sequence<int, NROLL>{});
      // every lane carries its lowest column into the next one (value-preserving;
      // in lane 0 that column is 0 mod 2^29 after m*n), so the digit that moves
      // down to lane g-1 fits 29 bits: one 32-bit DPP move
      acc[s1] += acc[s0] >> 29;
      if constexpr (HAS_ROT<G>) acc[s0] = (uint64_t)(dpp_next_rot<G>((uint32_t)acc[s0]) & m29);
      else acc[s0] = (uint64_t)(dpp_next<G>((uint32_t)acc[s0]) & m_top29);
    }
    if constexpr (ROW_FENCE) __builtin_amdgcn_sched_barrier(0);
  }

  // row R with its streamed digit already in `cur`; first issues the LDS read of
  // the next row's digit (the next cycle's first digit after the last row), so
  // the read's latency hides behind this row's MACs instead of stalling the
  // next row (one wave per SIMD in latency-bound launches has no other wave
  // to cover it).  arow[L] past the last cycle reads a harmless in-range word.
  // Short lanes (latency shapes) carry the next cycle's first NXT digits in
  // registers from the top of the cycle (product(), cycle_c)
  static constexpr int NXT = L <= 12 ? 1 : 0;
  template <int R, bool SQ, bool QS>
  __device__ __forceinline__ void row_pf(uint64_t* acc, const uint32_t* b, const uint32_t* b2, const uint32_t* n,
                                         const uint32_t* arow, uint32_t& cur, uint32_t next_off) const {
    const uint32_t ai = cur;
    cur = (R + 1 < L) ? arow[R + 1] : arow[next_off];
    row<R, SQ, QS>(acc, b, b2, n, ai);
  }
  // row R of a carried-digit cycle: its digit is carried (R < NXT) or read here
  template <int R, bool SQ, bool QS>
  __device__ __forceinline__ void row_c(uint64_t* acc, const uint32_t* b, const uint32_t* b2, const uint32_t* n,
                                        const uint32_t* arow, const uint32_t* carried) const {
    row<R, SQ, QS>(acc, b, b2, n, R < NXT ? carried[R < NXT ? R : 0] : arow[R]);
  }
  template <bool SQ, bool QS, int... Rs>
  __device__ __forceinline__ void cycle_c(uint64_t* acc, const uint32_t* b, const uint32_t* b2, const uint32_t* n,
                                          const uint32_t* arow, const uint32_t* carried,
                                          std::integer_sequence<int, Rs...>) const {
    (row_c<Rs, SQ, QS>(acc, b, b2, n, arow, carried), ...);
  }

  template <bool SQ, bool QS, int... Rs>
  __device__ __forceinline__ void cycle(uint64_t* acc, const uint32_t* b, const uint32_t* b2, const uint32_t* n,
                                        const uint32_t* arow, uint32_t& cur, uint32_t next_off,
                                        std::integer_sequence<int, Rs...>) const {
    (row_pf<Rs, SQ, QS>(acc, b, b2, n, arow, cur, next_off), ...);
  }

  // out = a * b / R  (almost Montgomery, < 2N), b = this lane's L digits (regs),
  // a = full KD-digit operand in LDS.  out may alias b.  (Non-const: b and n
  // pass through opaque(), which leaves their values unchanged.)
  __device__ __forceinline__ void mul(uint32_t* out, uint32_t* b, const uint32_t* a_lds) { product<false, false>(out, b, a_lds); }
  // out = a^2 / R where a_lds holds the same value as b (squaring rows above)
  __device__ __forceinline__ void sqr(uint32_t* out, uint32_t* b, const uint32_t* a_lds) { product<true, false>(out, b, a_lds); }
  // the same products with quotient-scaled rows (n holds N' = N (-N^-1 mod 2^29), see row())
  __device__ __forceinline__ void mul_s(uint32_t* out, uint32_t* b, const uint32_t* a_lds) { product<false, true>(out, b, a_lds); }
  __device__ __forceinline__ void sqr_s(uint32_t* out, uint32_t* b, const uint32_t* a_lds) { product<true, true>(out, b, a_lds); }

  template <bool SQ, bool QS>
  __device__ __forceinline__ void product(uint32_t* out, uint32_t* b, const uint32_t* a_lds) {
    static_assert(NORM_IN_CYCLE || L <= 30, "column bound of a product cycle (NORM_IN_CYCLE)");
    static_assert(G != 64, "the wave shape streams from registers: product_w");
    uint64_t acc[L];
#pragma unroll
    for (int j = 0; j < L; ++j) acc[j] = 0;
    uint32_t b2[NB2];
    if constexpr (SQ && USE_B2) {
#pragma unroll
      for (int j = 0; j < L; ++j) b2[j] = b[j] << 1;   // digits <= 2^29 + 127: fits
    }
    if constexpr (NXT) {
      // the next cycle's first NXT digits are read at the top of this cycle and
      // held in registers to its end (left to itself the compiler issued every
      // cycle's reads at its top and waited there for the first one: one LDS
      // round trip per cycle, 16 per 16-lane product); the later rows' reads are
      // then done before those rows
      uint32_t car[NXT];
#pragma unroll
      for (int k = 0; k < NXT; ++k) car[k] = a_lds[k];
#pragma unroll 1
      for (int cyc = 0; cyc < G; ++cyc) {
        uint32_t nx[NXT];
#pragma unroll
        for (int k = 0; k < NXT; ++k) nx[k] = a_lds[(cyc + 1 < G ? cyc + 1 : 0) * L + k];
        opaque<L>(b);
        if constexpr (!(SQ && USE_B2)) opaque<L>(n);
        if constexpr (SQ && USE_B2) opaque<L>(b2);
        cycle_c<SQ, QS>(acc, b, b2, n, a_lds + cyc * L, car, std::make_integer_sequence<int, L>{});
#pragma unroll
        for (int k = 0; k < NXT; ++k) {
          asm volatile("" : "+v"(nx[k]));
          car[k] = nx[k];
        }
      }
      finish(out, acc);
      return;
    }
    uint32_t cur = a_lds[0];
#pragma unroll 1
    for (int cyc = 0; cyc < G; ++cyc) {
      // values unchanged; only the optimiser's view of them is reset (see opaque)
      opaque<L>(b);
      // not n in the short-lane squarings (b2 held): there the per-cycle
      // barrier made the register allocator rotate the modulus digits through
      // copies every cycle (16 lanes: 183 -> 171 VALU per 9-row squaring cycle
      // of the sliding-window kernel, 8 lanes: 649 -> 625 per 18 rows, and
      // 4 fewer VGPRs); their zext is not hoisted there either
      if constexpr (!(SQ && USE_B2)) opaque<L>(n);
      if constexpr (SQ && USE_B2) opaque<L>(b2);
      cycle<SQ, QS>(acc, b, b2, n, a_lds + cyc * L, cur, cyc + 1 < G ? (uint32_t)L : 0u,
                    std::make_integer_sequence<int, L>{});
    }
    finish(out, acc);
  }

  // G = 64 (one instance per wave): the streamed operand is held in registers
  // like b (lane g: digits gL..gL+L-1) and each row's digit is read with
  // v_readlane, so it is wave-uniform: the a*b MACs take it from an SGPR and
  // the quotient digit is computed on the scalar unit (row()).  No LDS.  Only
  // the first KR/L lanes' digits are streamed (R = 2^(29 KR)).  a may alias b.
  __device__ __forceinline__ void mul_w(uint32_t* out, uint32_t* b, const uint32_t* a) { product_w<false>(out, b, a); }
  __device__ __forceinline__ void sqr_w(uint32_t* out, uint32_t* b) { product_w<true>(out, b, b); }

  template <int R, bool SQ>
  __device__ __forceinline__ void row_w(uint64_t* acc, const uint32_t* b, const uint32_t* n, const uint32_t* a,
                                        uint32_t& cur, int cyc) const {
    const uint32_t ai = cur;   // next row's digit first: the readlane latency hides behind this row
    cur = (R + 1 < L) ? (uint32_t)__builtin_amdgcn_readlane((int)a[R + 1], cyc)
                      : (uint32_t)__builtin_amdgcn_readlane((int)a[0], cyc + 1);   // lane KR/L past the end: unused
    row<R, SQ>(acc, b, nullptr, n, ai);
  }
  template <bool SQ, int... Rs>
  __device__ __forceinline__ void cycle_w(uint64_t* acc, const uint32_t* b, const uint32_t* n, const uint32_t* a,
                                          uint32_t& cur, int cyc, std::integer_sequence<int, Rs...>) const {
    (row_w<Rs, SQ>(acc, b, n, a, cur, cyc), ...);
  }
  template <bool SQ>
  __device__ __forceinline__ void product_w(uint32_t* out, uint32_t* b, const uint32_t* a) {
    static_assert(G == 64 && (!SQ || L <= 21), "wave shape");
    uint64_t acc[L];
#pragma unroll
    for (int j = 0; j < L; ++j) acc[j] = 0;
    uint32_t cur = (uint32_t)__builtin_amdgcn_readlane((int)a[0], 0);
#pragma unroll 1
    for (int cyc = 0; cyc < KR / L; ++cyc) {
      opaque<L>(b);
      opaque<L>(n);
      cycle_w<SQ>(acc, b, n, a, cur, cyc, std::make_integer_sequence<int, L>{});
    }
    finish(out, acc);
  }

  // carries of a finished product: digits <= 2^29+127
  __device__ __forceinline__ void finish(uint32_t* out, uint64_t* acc) const {
    // rotation is back to identity; two more carry steps give digits <= 2^29+127
    norm_step<0>(acc);
    const uint32_t cin = dpp_prev<G>((uint32_t)(acc[L - 1] >> 29)) & m_first;
#pragma unroll
    for (int j = L - 1; j > 0; --j) out[j] = ((uint32_t)acc[j] & M29) + (uint32_t)(acc[j - 1] >> 29);
    out[0] = ((uint32_t)acc[0] & M29) + cin;
  }

  // Exact normalisation of lazy digits (value < 2^(29*KD)) to digits < 2^29.
  __device__ __forceinline__ void carry_exact(uint32_t* d) const {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) { uint32_t v = d[j] + c; d[j] = v & M29; c = v >> 29; }
#pragma unroll 1
    for (int round = 0; round < G - 1; ++round) {
      uint32_t in = dpp_prev<G>(c) & m_first;
      c = 0;
#pragma unroll
      for (int j = 0; j < L; ++j) { uint32_t v = d[j] + in; d[j] = v & M29; in = v >> 29; }
      c = in;
    }
  }

  // n <- N' = N k with k = ninv = -N^-1 mod 2^29 (exact digits in, exact out), so
  // N' = -1 mod 2^29: the modulus of the quotient-scaled rows.  The caller
  // guarantees N' < 2^(29 KD) (SCALED_OK).
  __device__ __forceinline__ void scale_modulus() {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint64_t t = (uint64_t)n[j] * ninv + c;   // < 2^58 + 2^30
      n[j] = (uint32_t)t & M29;
      c = (uint32_t)(t >> 29);
    }
#pragma unroll 1
    for (int round = 0; round < G - 1; ++round) {   // each lane's carry into the next lane's digits
      uint32_t in = dpp_prev<G>(c) & m_first;
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const uint32_t v = n[j] + in;
        n[j] = v & M29;
        in = v >> 29;
      }
      c = in;
    }
    ninv = 1u;
  }

  // d (exact digits, value < 2N) -> d mod N
  __device__ __forceinline__ void sub_if_ge(uint32_t* d) const {
    uint32_t t[L];
    uint32_t bin = 0;
#pragma unroll 1
    for (int round = 0; round < G; ++round) {
      uint32_t bw = (round == 0) ? 0u : (dpp_prev<G>(bin) & m_first);
#pragma unroll
      for (int j = 0; j < L; ++j) {
        uint32_t v = d[j] - n[j] - bw;
        t[j] = v & M29;
        bw = v >> 31;
      }
      bin = bw;
    }
    const uint32_t ge = bcast_top<G>(bin == 0u ? 1u : 0u);
#pragma unroll
    for (int j = 0; j < L; ++j) d[j] = ge ? t[j] : d[j];
  }

  // d (exact, < N) -> 2d mod N, exact
  __device__ __forceinline__ void dbl(uint32_t* d) const {
    const uint32_t in = dpp_prev<G>(d[L - 1] >> 28) & m_first;
#pragma unroll
    for (int j = L - 1; j > 0; --j) d[j] = ((d[j] << 1) & M29) | (d[j - 1] >> 28);
    d[0] = ((d[0] << 1) & M29) | in;
    sub_if_ge(d);
  }
};

// ---- radix conversion helpers (global u32 limbs <-> 29-bit digits) -----------
// digit j of a K32-limb little-endian integer
__device__ __forceinline__ uint32_t digit_of(const uint32_t* __restrict__ x, int K32, int j) {
  const int bit = 29 * j;
  const int w = bit >> 5, sh = bit & 31;
  const uint32_t lo = (w < K32) ? x[w] : 0u;
  const uint32_t hi = (w + 1 < K32) ? x[w + 1] : 0u;
  return (uint32_t)(mk64(lo, hi) >> sh) & M29;
}
// limb k (32-bit) of an exact-digit integer stored in LDS
__device__ __forceinline__ uint32_t limb_of(const uint32_t* d, int KD, int k) {
  const int bit = 32 * k;
  const int j = bit / 29, sh = bit % 29;
  uint64_t v = (j < KD) ? d[j] : 0u;
  if (j + 1 < KD) v |= (uint64_t)d[j + 1] << 29;
  if (j + 2 < KD) v |= (uint64_t)d[j + 2] << 58;
  return (uint32_t)(v >> sh);
}

}  // namespace fsdkr
