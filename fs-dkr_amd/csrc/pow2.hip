// 2-adic half of the equality checks modulo an EVEN modulus (gfx950).
//
// The reference exponentiates with GMP mpz_powm, which accepts any modulus:
// RingPedersenProof::verify (ring_pedersen_proof.rs:144-148) checks
// T^Z_i == A_i * S^e_i (mod N) for the prover-chosen N, and zk-paillier's
// CompositeDLogProof::verify checks x == g^y * ni^e (mod N) for the joiner's N.
// An odd N runs entirely in the Montgomery kernels.  For N = 2^k * m (m odd)
// the congruence holds iff it holds modulo m (Montgomery kernels, modulus m)
// and modulo 2^k (this kernel), by the Chinese remainder theorem.
//
// Only adversarial messages have even moduli, so this is one thread per check
// with truncated schoolbook products (k <= 3072 bits); exponents are first
// shortened with the structure of (Z/2^k)^*: an odd base has order dividing
// 2^max(k-2,1), an even base to a power >= k vanishes.
#include "verify.h"

namespace fsdkr {

namespace {

constexpr int P2_MAX = 96;   // limbs of 2^k (k <= 3072)

__device__ __forceinline__ const uint32_t* P32(uint64_t a) { return reinterpret_cast<const uint32_t*>(a); }

// r = x * y mod 2^(32 K)
__device__ void mul_trunc(uint32_t* r, const uint32_t* x, const uint32_t* y, int K) {
  uint32_t t[P2_MAX];
  for (int i = 0; i < K; ++i) t[i] = 0;
  for (int i = 0; i < K; ++i) {
    const uint32_t xi = x[i];
    if (!xi) continue;
    uint64_t c = 0;
    for (int j = 0; i + j < K; ++j) {
      c += (uint64_t)xi * y[j] + t[i + j];
      t[i + j] = (uint32_t)c;
      c >>= 32;
    }
  }
  for (int i = 0; i < K; ++i) r[i] = t[i];
}

__device__ void load_mod2k(uint32_t* d, uint64_t addr, uint32_t len, int K, uint32_t topmask) {
  const uint32_t* x = P32(addr);
  for (int i = 0; i < K; ++i) d[i] = (addr && (uint32_t)i < len) ? x[i] : 0u;
  if (!addr) d[0] = 1;   // null operand = 1
  d[K - 1] &= topmask;
}

__device__ uint32_t bitlen(const uint32_t* e, uint32_t len) {
  for (int k = (int)len - 1; k >= 0; --k)
    if (e[k]) return 32u * (uint32_t)k + 32u - (uint32_t)__builtin_clz(e[k]);
  return 0;
}

// out = b^e mod 2^kbits  (b already reduced: K limbs, masked)
__device__ void pow_mod2k(uint32_t* out, const uint32_t* b, uint64_t eaddr, uint32_t elen, uint32_t kbits, int K,
                          uint32_t topmask) {
  const uint32_t* e = P32(eaddr);
  const uint32_t eb = eaddr ? bitlen(e, elen) : 0u;
  for (int i = 0; i < K; ++i) out[i] = 0;
  out[0] = 1;
  if (eb == 0) {               // x^0 = 1 (GMP: 0^0 = 1)
    out[K - 1] &= topmask;
    return;
  }
  bool zero = true;
  int tz = 0;
  for (int i = 0; i < K; ++i)
    if (b[i]) {
      zero = false;
      tz = 32 * i + __builtin_ctz(b[i]);
      break;
    }
  uint32_t limit;
  if (zero) {
    out[0] = 0;
    return;
  }
  if (tz > 0) {                // even base: b^e == 0 once e * tz >= k
    if (eb > 13 || (uint64_t)e[0] * (uint32_t)tz >= kbits) {
      out[0] = 0;
      return;
    }
    limit = eb;
  } else {                     // odd base: order divides 2^max(k-2, 1)
    const uint32_t ord = kbits > 3 ? kbits - 2 : 1u;
    limit = eb < ord ? eb : ord;
  }
  uint32_t t[P2_MAX];
  for (int bit = (int)limit - 1; bit >= 0; --bit) {
    mul_trunc(out, out, out, K);
    if ((e[bit >> 5] >> (bit & 31)) & 1u) {
      mul_trunc(t, out, b, K);
      for (int i = 0; i < K; ++i) out[i] = t[i];
    }
    out[K - 1] &= topmask;
  }
}

__global__ __launch_bounds__(64) void pow2_check_kernel(const Pow2Args a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.count) return;
  const Pow2Op op = a.ops[i];
  const uint32_t kbits = op.kbits;
  if (kbits == 0 || kbits > 32u * P2_MAX) {   // host never emits these
    a.out[i] = 0;
    return;
  }
  const int K = (int)((kbits + 31) / 32);
  const uint32_t topmask = (kbits % 32) ? ((1u << (kbits % 32)) - 1u) : 0xFFFFFFFFu;
  uint32_t x[P2_MAX], y[P2_MAX], b[P2_MAX];
  // lhs = a^ea * b^eb
  load_mod2k(b, op.a, op.a_len, K, topmask);
  pow_mod2k(x, b, op.ea, op.ea_len, kbits, K, topmask);
  load_mod2k(b, op.b, op.b_len, K, topmask);
  pow_mod2k(y, b, op.eb, op.eb_len, kbits, K, topmask);
  mul_trunc(x, x, y, K);
  x[K - 1] &= topmask;
  // rhs = c * d^[bit]
  bool use_d = op.d != 0;
  if (use_d && op.sel != 0xFFFFFFFFu) use_d = ((a.sel_bits[op.sel >> 5] >> (op.sel & 31)) & 1u) != 0;
  load_mod2k(y, op.c, op.c_len, K, topmask);
  if (use_d) {
    load_mod2k(b, op.d, op.d_len, K, topmask);
    mul_trunc(y, y, b, K);
    y[K - 1] &= topmask;
  }
  uint32_t diff = 0;
  for (int k = 0; k < K; ++k) diff |= x[k] ^ y[k];
  a.out[i] = diff == 0 ? 1u : 0u;
}

}  // namespace

hipError_t launch_pow2_check(const Pow2Args& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  hipLaunchKernelGGL(pow2_check_kernel, dim3((a.count + 63) / 64), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace fsdkr
