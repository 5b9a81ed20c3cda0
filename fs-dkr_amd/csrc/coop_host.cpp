// Host constants of the one-wave cooperative modexp (coop.hip): per odd modulus
// N, in 28-bit digits, N | R mod N | R^2 mod N | N'' = -N^-1 mod R with
// R = 2^(28 K).  O(K^2) each (Newton's iteration doubles the precision of the
// 2-adic inverse: 32, 64, ..., 28 K bits).
#include <cstdint>
#include <vector>

#include "hostbn.hpp"
#include "verify.h"

namespace fsdkr {

namespace {

// low `bits` bits of a
hbn::Limbs trunc(hbn::Limbs a, uint32_t bits) {
  const size_t words = (bits + 31) / 32;
  if (a.size() > words) a.resize(words);
  if (bits % 32 && a.size() == words) a[words - 1] &= (1u << (bits % 32)) - 1u;
  hbn::trim(a);
  return a;
}

void to_digits28(const hbn::Limbs& a, uint32_t K, uint32_t* out) {
  for (uint32_t j = 0; j < K; ++j) {
    const uint32_t bit = 28 * j, w = bit / 32, sh = bit % 32;
    const uint64_t lo = w < a.size() ? a[w] : 0u;
    const uint64_t hi = w + 1 < a.size() ? a[w + 1] : 0u;
    out[j] = (uint32_t)(((hi << 32) | lo) >> sh) & ((1u << 28) - 1u);
  }
}

}  // namespace

void coop_constants(const uint32_t* n, uint32_t k32, uint32_t K, uint32_t* out) {
  const hbn::Limbs N = hbn::from(n, k32);
  const uint32_t rbits = 28 * K;
  const hbn::Limbs Rm = hbn::mod(hbn::shl(hbn::Limbs{1}, rbits), N);
  const hbn::Limbs R2 = hbn::mulmod(Rm, Rm, N);
  // N^-1 mod 2^32 (Newton over u32), then doubling precision
  uint32_t x0 = n[0];
  for (int i = 0; i < 5; ++i) x0 *= 2u - n[0] * x0;
  hbn::Limbs x{x0};
  for (uint32_t bits = 64;; bits *= 2) {
    const uint32_t b = bits < rbits ? bits : rbits;
    const hbn::Limbs t = trunc(hbn::mul(trunc(N, b), x), b);   // N x mod 2^b (= 1 mod 2^(b/2))
    const hbn::Limbs two_minus = trunc(hbn::sub(hbn::add(hbn::shl(hbn::Limbs{1}, b), hbn::Limbs{2}), t), b);
    x = trunc(hbn::mul(x, two_minus), b);
    if (b == rbits) break;
  }
  // N'' = R - x  (x != 0: N is odd)
  const hbn::Limbs ninv = hbn::sub(hbn::shl(hbn::Limbs{1}, rbits), x);
  to_digits28(N, K, out);
  to_digits28(Rm, K, out + K);
  to_digits28(R2, K, out + 2 * K);
  to_digits28(ninv, K, out + 3 * K);
}

}  // namespace fsdkr
