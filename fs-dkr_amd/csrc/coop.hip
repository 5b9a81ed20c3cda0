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
// partials meet in LDS and each lane sums ~5 columns.  28-bit digits keep a
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
  static_assert(P * P == 64 && P * TD == K, "one tile per lane of one wave");
};

// LDS of one chain (one wave per block)
template <int K, int TD>
struct CoopSmem {
  using S = CoopShape<K, TD>;
  uint64_t part[64][S::NC];   // column partials of the lanes' tiles
  uint64_t car[S::NCOL];      // carries of the normalisation passes
  uint32_t A[K], B[K];        // operands (digits < 2^28 + 2^9)
  uint32_t T[S::NCOL];        // a * b
  uint32_t Mq[K];             // m
  uint32_t Nd[K], Ni[K];      // N, N''
  uint32_t flag;
};

// sum of column c over the tiles of diagonals c / TD and c / TD - 1: 2P
// predicated reads, all independent (a loop over the valid range would wait out
// each read's LDS latency in turn)
template <int K, int TD>
__device__ __forceinline__ uint64_t column_sum(const CoopSmem<K, TD>& s, int c, int dmax) {
  using S = CoopShape<K, TD>;
  uint64_t v = 0;
  const int d1 = c / TD;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int d = d1 - e;
    const int k = c - d * TD;
    const bool okd = d >= 0 && d <= dmax && k < S::NC;
#pragma unroll
    for (int p = 0; p < S::P; ++p) {
      const int q = d - p;
      const bool ok = okd && q >= 0 && q < S::P;
      const uint64_t x = s.part[ok ? p * S::P + q : 0][ok ? k : 0];
      v += ok ? x : 0u;
    }
  }
  return v;
}

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

// Columns [0, ncol) of the partials in s.part (diagonals 0..dmax) plus `add`
// (ncol words or null) -> lazy 28-bit digits in dst.  Carries out of column
// ncol-1 are dropped (callers: they are zero, or the reduction is mod R).
template <int K, int TD>
__device__ __forceinline__ void columns_to_digits(CoopSmem<K, TD>& s, int ncol, int dmax, const uint32_t* add,
                                                  uint32_t* dst) {
  constexpr int R = (2 * K + 63) / 64;   // columns per lane (strided by 64)
  const int lane = threadIdx.x;
  uint64_t v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int c = lane + 64 * r;
    v[r] = 0;
    if (c < ncol) {
      v[r] = column_sum<K, TD>(s, c, dmax);
      if (add) v[r] += add[c];
    }
  }
  // two carry-save passes: < 2^28 + 2^35.3, then < 2^28 + 2^8
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int c = lane + 64 * r;
      if (c < ncol) s.car[c] = v[r] >> 28;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int c = lane + 64 * r;
      if (c < ncol) v[r] = (v[r] & M28) + (c > 0 ? s.car[c - 1] : 0u);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int c = lane + 64 * r;
    if (c < ncol) dst[c] = (uint32_t)v[r];
  }
}

// out = a * b / R mod N (almost: < 2N).  a, b, out: K-digit LDS arrays (out may
// alias a or b).
template <int K, int TD>
__device__ void coop_mont(CoopSmem<K, TD>& s, const uint32_t* a, const uint32_t* b, uint32_t* out) {
  using S = CoopShape<K, TD>;
  const int lane = threadIdx.x;
  const int p = lane / S::P, q = lane % S::P;
  uint64_t acc[S::NC];
  // T = a * b
  tile_product<K, TD>(a, b, p, q, acc);
#pragma unroll
  for (int k = 0; k < S::NC; ++k) s.part[lane][k] = acc[k];
  __syncthreads();
  columns_to_digits<K, TD>(s, S::NCOL, 2 * S::P - 2, nullptr, s.T);
  __syncthreads();
  // m = (T mod R) * N'' mod R: the tiles on diagonals < P
  if (p + q < S::P) {
    tile_product<K, TD>(s.T, s.Ni, p, q, acc);
#pragma unroll
    for (int k = 0; k < S::NC; ++k) s.part[lane][k] = acc[k];
  }
  __syncthreads();
  columns_to_digits<K, TD>(s, K, S::P - 1, nullptr, s.Mq);
  __syncthreads();
  // U = T + m * N; its low half is 0 or R
  tile_product<K, TD>(s.Mq, s.Nd, p, q, acc);
#pragma unroll
  for (int k = 0; k < S::NC; ++k) s.part[lane][k] = acc[k];
  if (lane == 0) s.flag = 0;
  __syncthreads();
  {
    constexpr int R = (2 * K + 63) / 64;
    uint64_t v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int c = lane + 64 * r;
      v[r] = 0;
      if (c < S::NCOL) v[r] = column_sum<K, TD>(s, c, 2 * S::P - 2) + s.T[c];
    }
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int c = lane + 64 * r;
        if (c < S::NCOL) s.car[c] = v[r] >> 28;
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int c = lane + 64 * r;
        if (c < S::NCOL) v[r] = (v[r] & M28) + (c > 0 ? s.car[c - 1] : 0u);
      }
      __syncthreads();
    }
    bool low_nz = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int c = lane + 64 * r;
      if (c < K && v[r] != 0) low_nz = true;
    }
    const bool any = __any(low_nz ? 1 : 0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int c = lane + 64 * r;
      if (c >= K && c < S::NCOL) out[c - K] = (uint32_t)v[r] + ((c == K && any) ? 1u : 0u);
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
  const uint32_t* C = a.consts + (size_t)a.mod_idx[inst] * 4 * K;   // N | R mod N | R^2 mod N | N''
  for (int j = lane; j < K; j += 64) {
    s.Nd[j] = C[j];
    s.Ni[j] = C[3 * K + j];
  }
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
  __syncthreads();
  if (top < 0) {   // exponent 0: the Montgomery one
    load(s.A, C + K);
    __syncthreads();
  } else {
    coop_mont<K, TD>(s, s.A, s.B, s.A);   // x R
    store(Tab, s.A);
    coop_mont<K, TD>(s, s.A, s.A, s.B);   // x^2 R
    store(Tab + (size_t)tw * K, s.B);
    for (uint32_t jt = 1; jt < tw; ++jt) {   // odd powers
      coop_mont<K, TD>(s, s.A, s.B, s.A);
      store(Tab + (size_t)jt * K, s.A);
    }
    __syncthreads();   // the table rows are read back by other lanes
    // the first window: its odd power, no squarings of 1
    auto window = [&](int i, int* jl) -> uint32_t {
      int j = max(i - (int)w + 1, 0);
      while (!bit(j)) ++j;
      uint32_t d = 0;
      for (int k = i; k >= j; --k) d = (d << 1) | bit(k);
      *jl = j;
      return d;
    };
    int jl;
    uint32_t d = window(top, &jl);
    load(s.A, Tab + (size_t)(d >> 1) * K);
    __syncthreads();
    int i = jl - 1;
    while (i >= 0) {
      if (!bit(i)) {
        coop_mont<K, TD>(s, s.A, s.A, s.A);
        --i;
        continue;
      }
      d = window(i, &jl);
      for (int k = i; k >= jl; --k) coop_mont<K, TD>(s, s.A, s.A, s.A);
      load(s.B, Tab + (size_t)(d >> 1) * K);
      __syncthreads();
      coop_mont<K, TD>(s, s.A, s.B, s.A);
      i = jl - 1;
    }
  }
  // exit: acc * 1 / R  (< N + 1), exact digits, then mod N
  for (int j = lane; j < K; j += 64) s.B[j] = j == 0 ? 1u : 0u;
  __syncthreads();
  coop_mont<K, TD>(s, s.A, s.B, s.A);
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
