// One-wave cooperative modular exponentiation for latency-bound launches (a
// multi-GPU rank's slice: ~1 000 chains on 1 024 SIMDs).  The CIOS shapes of
// modexp.hip spend one dependent row per digit of the streamed operand (144
// rows of a 4096-bit product), and a 16-lane group issues each row's 19
// instructions itself: ~7 us per product when the chip is otherwise idle.  Here
// the whole wave (64 lanes) owns ONE chain and a product has no row chain:
//
//   separated Montgomery, R = 2^(28 K):
//     T = a * b                    (2K columns)
//     m = (T mod R) * N'' mod R    (N'' = -N^-1 mod R: the low K columns)
//     U = T + m * N,   out = U / R (U = 0 mod R)
//
// Each product is an 8 x 8 grid of TD x TD digit tiles, one tile per lane
// (TD^2 MACs, v_mad_u64_u32 into 2TD-1 column accumulators); the tiles' column
// partials are added into LDS column sums (ds_add_u64) and each lane takes ~5.  28-bit digits keep a
// whole column (K products < 2^56.0001) below 2^64, so the sums need no carry
// handling; two carry-save passes then leave digits < 2^28 + 2^8, which the
// next product accepts as they are.  The division by R needs no carry chain
// through the low half: it holds 0 or exactly R (a multiple of R below 2R), so
// out = U's high half + [any low digit != 0].  Outputs stay below 2N ("almost
// Montgomery", like mont29.hpp); one exact reduction at the exit.
//
// Exponent schedule: sliding windows over the instance's own exponent (one
// instance per wave, so the schedule is wave-uniform) -- the same windows as
// modexp_slide_kernel.  Used for the GA chains s^N mod N^2 of a shard's slice
// (refresh_message.rs:330-350 via zk_pdl_with_slack.rs:136-142 and
// range_proofs.rs:140-148) and exposed through fsdkr_modexp_batch with the
// context's modexp group set to FSDKR_COOP_GROUP.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"
#include "verify.h"

namespace fsdkr {

constexpr uint32_t M28 = (1u << 28) - 1;

template <int K, int TD>
struct CoopShape {
  static constexpr int P = K / TD;          // tiles per side
  static constexpr int NC = 2 * TD - 1;     // column partials per tile
  static constexpr int NCOL = 2 * K;        // columns of a full product
  static constexpr int R = (NCOL + 63) / 64;   // columns per lane (c = lane + 64 r)
  static constexpr int NCP = 64 * R;        // padded: every lane handles R columns, branch-free
  static_assert(P * P == 64 && P * TD == K, "one tile per lane of one wave");
};

// LDS of one chain (one wave per block)
template <int K, int TD>
struct CoopSmem {
  using S = CoopShape<K, TD>;
  uint64_t col[S::NCP];       // column sums: every tile's partials added in (ds_add_u64)
  uint32_t A[S::NCP - K], B[S::NCP - K];   // operands (K digits < 2^28 + 2^9; the rest scratch)
  uint32_t T[S::NCP];         // a * b (columns past 2K stay 0)
  uint32_t Mq[S::NCP];        // m (K digits)
  uint32_t Nd[K], Ni[K];      // N, N''
};

template <int K, int TD>
__device__ __forceinline__ void tile_product(const uint32_t* X, const uint32_t* Y, int p, int q, uint64_t* acc) {
  using S = CoopShape<K, TD>;
  uint32_t x[TD], y[TD];
#pragma unroll
  for (int i = 0; i < TD; ++i) {
    x[i] = X[p * TD + i];
    y[i] = Y[q * TD + i];
  }
#pragma unroll
  for (int k = 0; k < S::NC; ++k) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < TD; ++i)
#pragma unroll
    for (int j = 0; j < TD; ++j) acc[i + j] += (uint64_t)x[i] * y[j];
}

// a tile's partials into the column sums (the columns start zeroed)
template <int K, int TD>
__device__ __forceinline__ void add_partials(CoopSmem<K, TD>& s, int d, const uint64_t* acc) {
  using S = CoopShape<K, TD>;
  unsigned long long* c0 = reinterpret_cast<unsigned long long*>(s.col) + d * TD;
#pragma unroll
  for (int k = 0; k < S::NC; ++k) atomicAdd(c0 + k, (unsigned long long)acc[k]);
}

// The lane's columns c = lane + 64 r: v[r] = column sum (+ add[c]), every column
// zeroed for the next product's sums.  Padded columns (>= 2K) hold 0.
template <int K, int TD>
__device__ __forceinline__ void take_columns(CoopSmem<K, TD>& s, const uint32_t* add, uint64_t* v) {
  using S = CoopShape<K, TD>;
  const int lane = threadIdx.x;
#pragma unroll
  for (int r = 0; r < S::R; ++r) {
    const int c = lane + 64 * r;
    v[r] = s.col[c] + (add ? add[c] : 0u);
    s.col[c] = 0;
  }
}

// the value of lane - 1 (lane 0: `first`, uniform)
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t x, uint32_t first, bool lane0) {
  const uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x138, 0xF, 0xF, true);   // wave_shr:1
  return lane0 ? first : t;
}

// two carry-save passes over all columns: < 2^28 + 2^35.3, then < 2^28 + 2^8.
// Column c = lane + 64 r takes the carry of c - 1 from the previous lane (wave_shr
// DPP; lane 0 from lane 63 of r - 1), no LDS round trip.  Carries only move up,
// so the low columns do not depend on the high ones (the reduction mod R ignores
// them); nothing leaves the top (the values fit 2K columns).
template <int K, int TD>
__device__ __forceinline__ void normalise(uint64_t* v) {
  using S = CoopShape<K, TD>;
  const bool lane0 = threadIdx.x == 0;
  {   // pass 0: 36-bit carries
    uint32_t lo[S::R], hi[S::R];
#pragma unroll
    for (int r = 0; r < S::R; ++r) {
      const uint64_t c = v[r] >> 28;
      lo[r] = (uint32_t)c;
      hi[r] = (uint32_t)(c >> 32);
    }
#pragma unroll
    for (int r = 0; r < S::R; ++r) {
      const uint32_t plo = r ? (uint32_t)__builtin_amdgcn_readlane((int)lo[r - 1], 63) : 0u;
      const uint32_t phi = r ? (uint32_t)__builtin_amdgcn_readlane((int)hi[r - 1], 63) : 0u;
      const uint64_t in = ((uint64_t)from_prev_lane(hi[r], phi, lane0) << 32) | from_prev_lane(lo[r], plo, lane0);
      v[r] = (v[r] & M28) + in;
    }
  }
  {   // pass 1: carries < 2^8
    uint32_t cr[S::R];
#pragma unroll
    for (int r = 0; r < S::R; ++r) cr[r] = (uint32_t)(v[r] >> 28);
#pragma unroll
    for (int r = 0; r < S::R; ++r) {
      const uint32_t prv = r ? (uint32_t)__builtin_amdgcn_readlane((int)cr[r - 1], 63) : 0u;
      v[r] = (v[r] & M28) + from_prev_lane(cr[r], prv, lane0);
    }
  }
}

// out = a * b / R mod N (almost: < 2N).  a, b, out: K-digit LDS arrays (out may
// alias a or b).  s.col is zero on entry and on exit.
template <int K, int TD>
__device__ __forceinline__ void coop_mont(CoopSmem<K, TD>& s, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  using S = CoopShape<K, TD>;
  const int lane = threadIdx.x;
  const int p = lane / S::P, q = lane % S::P;
  uint64_t acc[S::NC];
  uint64_t v[S::R];
  // T = a * b
  tile_product<K, TD>(a, b, p, q, acc);
  add_partials<K, TD>(s, p + q, acc);
  __syncthreads();
  take_columns<K, TD>(s, nullptr, v);
  normalise<K, TD>(v);
#pragma unroll
  for (int r = 0; r < S::R; ++r) s.T[lane + 64 * r] = (uint32_t)v[r];
  __syncthreads();
  // m = (T mod R) * N'' mod R: the tiles on diagonals < P; the columns >= K they
  // also reach are normalised with the rest and not read
  if (p + q < S::P) {
    tile_product<K, TD>(s.T, s.Ni, p, q, acc);
    add_partials<K, TD>(s, p + q, acc);
  }
  __syncthreads();
  take_columns<K, TD>(s, nullptr, v);
  normalise<K, TD>(v);
#pragma unroll
  for (int r = 0; r < S::R; ++r) s.Mq[lane + 64 * r] = (uint32_t)v[r];
  __syncthreads();
  // U = T + m * N; its low half is 0 or R
  tile_product<K, TD>(s.Mq, s.Nd, p, q, acc);
  add_partials<K, TD>(s, p + q, acc);
  __syncthreads();
  take_columns<K, TD>(s, s.T, v);
  normalise<K, TD>(v);
  bool low_nz = false;
#pragma unroll
  for (int r = 0; r < S::R; ++r) low_nz |= (lane + 64 * r < K) & (v[r] != 0);
  const uint32_t any = __any(low_nz ? 1 : 0) ? 1u : 0u;
#pragma unroll
  for (int r = 0; r < S::R; ++r) {
    const int c = lane + 64 * r;
    if (64 * r + 63 >= K) {   // (compile time per r) rows of the high half
      if (c >= K) out[c - K] = (uint32_t)v[r] + (c == K ? any : 0u);
    }
  }
  __syncthreads();
}

// digit j (28-bit) of a little-endian u32-limb integer of n limbs
__device__ __forceinline__ uint32_t digit28(const uint32_t* x, int n, int j) {
  const int bit = 28 * j;
  const int w = bit >> 5, sh = bit & 31;
  const uint32_t lo = w < n ? x[w] : 0u;
  const uint32_t hi = w + 1 < n ? x[w + 1] : 0u;
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & M28;
}

template <int K, int TD, int K32>
__global__ __launch_bounds__(64) void modexp_coop_kernel(const CoopArgs a) {
  __shared__ CoopSmem<K, TD> s;
  const uint32_t inst = blockIdx.x;
  if (inst >= a.count) return;
  const int lane = threadIdx.x;
  if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  const uint32_t* C = a.consts + (size_t)a.mod_idx[inst] * 4 * K;   // N | R mod N | R^2 mod N | N''
  for (int j = lane; j < K; j += 64) {
    s.Nd[j] = C[j];
    s.Ni[j] = C[3 * K + j];
  }
  for (int j = lane; j < CoopShape<K, TD>::NCP; j += 64) s.col[j] = 0;
  const uint32_t* Bp = reinterpret_cast<const uint32_t*>(a.base_ptr[inst]);
  const int blen = (int)min(a.base_len[inst], (uint32_t)K32);
  for (int j = lane; j < K; j += 64) {
    s.A[j] = digit28(Bp, blen, j);
    s.B[j] = C[2 * K + j];   // R^2 mod N
  }
  const uint64_t ea = a.exp_ptr[inst];
  const uint32_t* E = reinterpret_cast<const uint32_t*>(
      ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(ea >> 32)) << 32) |
      (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)ea));
  const int exp_limbs = __builtin_amdgcn_readfirstlane((int)a.exp_len[inst]);
  auto bit = [&](int i) -> uint32_t { return (E[i >> 5] >> (i & 31)) & 1u; };
  int top = 32 * exp_limbs - 1;
  while (top >= 0 && E[top >> 5] == 0) top = (top & ~31) - 1;
  while (top >= 0 && !bit(top)) --top;
  const uint32_t w = a.window, tw = 1u << (w - 1);   // odd powers T[0..tw), x^2 at T[tw]
  uint32_t* Tab = a.table + (size_t)inst * (tw + 1) * K;
  auto store = [&](uint32_t* row, const uint32_t* src) {
    for (int j = lane; j < K; j += 64) row[j] = src[j];
  };
  auto load = [&](uint32_t* dst, const uint32_t* row) {
    for (int j = lane; j < K; j += 64) dst[j] = row[j];
  };
  auto window = [&](int i, int* jl) -> uint32_t {   // the window ending the run of bits at i (bit i set)
    int j = max(i - (int)w + 1, 0);
    while (!bit(j)) ++j;
    uint32_t d = 0;
    for (int k = i; k >= j; --k) d = (d << 1) | bit(k);
    *jl = j;
    return d;   // odd
  };
  __syncthreads();
  // Every product is issued from ONE site (coop_mont inlined once: the operands
  // are known LDS arrays, no generic-pointer conversions, one copy in the I-cache):
  //   phase 0: A = x R (B = R^2);  1: B = x^2 R;  2: A = T[jt] = T[jt-1] x^2;
  //   3: the windows (squarings of A, then A * T[d] through B);  4: A * 1
  int phase = top < 0 ? 4 : 0, i = top, pend_mul = -1;
  uint32_t jt = 1, pend_sq = 0;
  if (top < 0) {   // exponent 0: the Montgomery one
    load(s.A, C + K);
    for (int j = lane; j < K; j += 64) s.B[j] = j == 0 ? 1u : 0u;
    __syncthreads();
  }
  while (phase < 5) {
    bool sq = false, to_b = false;
    if (phase == 1) {
      sq = to_b = true;
    } else if (phase == 3) {
      if (pend_sq) {
        sq = true;
        --pend_sq;
      } else if (pend_mul >= 0) {
        load(s.B, Tab + (size_t)pend_mul * K);
        pend_mul = -1;
        __syncthreads();
      } else if (i < 0) {   // exit product: A * 1
        for (int j = lane; j < K; j += 64) s.B[j] = j == 0 ? 1u : 0u;
        phase = 4;
        __syncthreads();
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
    }
    coop_mont<K, TD>(s, s.A, sq ? s.A : s.B, to_b ? s.B : s.A);
    if (phase == 0) {
      store(Tab, s.A);
      phase = 1;
    } else if (phase == 1) {
      store(Tab + (size_t)tw * K, s.B);
      phase = tw > 1 ? 2 : 3;
    } else if (phase == 2) {
      store(Tab + (size_t)jt * K, s.A);
      if (++jt == tw) phase = 3;
    } else if (phase == 4) {
      phase = 5;
    }
    if (phase == 3 && i == top) {   // entering the windows: the first window's odd power, no squarings of 1
      __syncthreads();   // the table rows are read back by other lanes
      int jl;
      const uint32_t d = window(i, &jl);
      load(s.A, Tab + (size_t)(d >> 1) * K);
      i = jl - 1;
      __syncthreads();
    }
  }
  // exit: A = x^e R / R (< N + 1): exact digits, then mod N
  if (lane == 0) {
    uint32_t c = 0;
    for (int j = 0; j < K; ++j) {
      const uint32_t v = s.A[j] + c;
      s.A[j] = v & M28;
      c = v >> 28;
    }
    // v >= N ?  (v < 2N: one subtraction)
    int ge = 1;
    for (int j = K - 1; j >= 0; --j)
      if (s.A[j] != s.Nd[j]) {
        ge = s.A[j] > s.Nd[j];
        break;
      }
    if (c || ge) {
      uint32_t bw = 0;
      for (int j = 0; j < K; ++j) {
        const uint32_t v = s.A[j] - s.Nd[j] - bw;
        s.A[j] = v & M28;
        bw = v >> 31;
      }
    }
  }
  __syncthreads();
  uint32_t* O = a.out + (size_t)(a.out_idx ? a.out_idx[inst] : inst) * K32;
  for (int q = lane; q < K32; q += 64) {   // limb q = bits [32q, 32q + 32)
    const int bit0 = 32 * q;
    const int j = bit0 / 28, sh = bit0 % 28;
    uint64_t v = (uint64_t)s.A[j] >> sh;
    if (j + 1 < K) v |= (uint64_t)s.A[j + 1] << (28 - sh);
    if (j + 2 < K) v |= (uint64_t)s.A[j + 2] << (56 - sh);
    O[q] = (uint32_t)v;
  }
}

template <int K, int TD, int K32>
static hipError_t launch_coop(const CoopArgs& a, hipStream_t st) {
  if (a.count == 0) return hipSuccess;
  hipLaunchKernelGGL((modexp_coop_kernel<K, TD, K32>), dim3(a.count), dim3(64), 0, st, a);
  return hipGetLastError();
}

uint32_t coop_digits(uint32_t k32) {
  switch (k32) {
    case 64: return 80;     // 8 x 10: R = 2^2240
    case 128: return 152;   // 8 x 19: R = 2^4256
    default: return 0;
  }
}

hipError_t launch_modexp_coop(uint32_t k32, const CoopArgs& a, hipStream_t st) {
  switch (k32) {
    case 64: return launch_coop<80, 10, 64>(a, st);
    case 128: return launch_coop<152, 19, 128>(a, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace fsdkr
