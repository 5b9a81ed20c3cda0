// Minimal host big-integer helpers (little-endian u32 limbs) for the O(1)- or
// O(n)-per-collect host logic around the GPU batch: N^2, bit lengths,
// comparisons, the correct-key rho reduction, small-prime trial division,
// gcd tests of DLog statements and the Paillier L-function.  Not on the
// O(n^2) verification path (that is all GPU).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

namespace fsdkr {
namespace hbn {

using Limbs = std::vector<uint32_t>;

inline void trim(Limbs& a) {
  while (!a.empty() && a.back() == 0) a.pop_back();
}
inline Limbs from(const uint32_t* p, size_t n) {
  Limbs a(p, p + n);
  trim(a);
  return a;
}
inline uint32_t bitlen(const Limbs& a) {
  if (a.empty()) return 0;
  return (uint32_t)(a.size() - 1) * 32 + 32 - __builtin_clz(a.back());
}
inline uint32_t bitlen(const uint32_t* p, size_t n) {
  for (size_t k = n; k-- > 0;)
    if (p[k]) return (uint32_t)k * 32 + 32 - __builtin_clz(p[k]);
  return 0;
}
inline int cmp(const Limbs& a, const Limbs& b) {
  if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
  for (size_t k = a.size(); k-- > 0;)
    if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
  return 0;
}
inline Limbs add(const Limbs& a, const Limbs& b) {
  Limbs r(std::max(a.size(), b.size()) + 1, 0);
  uint64_t c = 0;
  for (size_t k = 0; k < r.size(); ++k) {
    c += (uint64_t)(k < a.size() ? a[k] : 0) + (k < b.size() ? b[k] : 0);
    r[k] = (uint32_t)c;
    c >>= 32;
  }
  trim(r);
  return r;
}
inline Limbs add_small(const Limbs& a, uint32_t v) { return add(a, Limbs{v}); }
// a - b, requires a >= b
inline Limbs sub(const Limbs& a, const Limbs& b) {
  Limbs r(a.size(), 0);
  int64_t br = 0;
  for (size_t k = 0; k < a.size(); ++k) {
    int64_t d = (int64_t)a[k] - (k < b.size() ? b[k] : 0) + br;
    r[k] = (uint32_t)d;
    br = d >> 32;
  }
  trim(r);
  return r;
}
inline Limbs mul(const Limbs& a, const Limbs& b) {
  if (a.empty() || b.empty()) return {};
  Limbs r(a.size() + b.size(), 0);
  for (size_t i = 0; i < a.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.size(); ++j) {
      c += (uint64_t)a[i] * b[j] + r[i + j];
      r[i + j] = (uint32_t)c;
      c >>= 32;
    }
    r[i + b.size()] = (uint32_t)c;
  }
  trim(r);
  return r;
}
inline Limbs shl(const Limbs& a, uint32_t s) {
  if (a.empty()) return {};
  const uint32_t w = s / 32, b = s % 32;
  Limbs r(a.size() + w + 1, 0);
  for (size_t k = 0; k < a.size(); ++k) {
    r[k + w] |= a[k] << b;
    if (b) r[k + w + 1] |= a[k] >> (32 - b);
  }
  trim(r);
  return r;
}
inline Limbs shr1(const Limbs& a) {
  Limbs r(a.size(), 0);
  for (size_t k = 0; k < a.size(); ++k) r[k] = (a[k] >> 1) | (k + 1 < a.size() ? a[k + 1] << 31 : 0);
  trim(r);
  return r;
}
// remainder modulo a small word
inline uint32_t mod_small(const Limbs& a, uint32_t m) {
  uint64_t r = 0;
  for (size_t k = a.size(); k-- > 0;) r = ((r << 32) | a[k]) % m;
  return (uint32_t)r;
}
// (q, r) = a / b, bit-serial long division (inputs are a few thousand bits)
inline void divmod(const Limbs& a, const Limbs& b, Limbs* q, Limbs* r) {
  Limbs rem;
  Limbs quo(a.size(), 0);
  const uint32_t nb = bitlen(a);
  for (uint32_t i = nb; i-- > 0;) {
    rem = shl(rem, 1);
    if ((a[i / 32] >> (i % 32)) & 1u) {
      if (rem.empty()) rem.push_back(1);
      else rem[0] |= 1u;
    }
    if (cmp(rem, b) >= 0) {
      rem = sub(rem, b);
      quo[i / 32] |= 1u << (i % 32);
    }
  }
  trim(quo);
  if (q) *q = quo;
  if (r) *r = rem;
}
// Knuth algorithm D (TAOCP 4.3.1) for larger operands
inline void divmod_knuth(const Limbs& a, const Limbs& b, Limbs* q, Limbs* r) {
  if (cmp(a, b) < 0) {
    if (q) q->clear();
    if (r) *r = a;
    return;
  }
  if (b.size() == 1) {
    Limbs quo(a.size(), 0);
    uint64_t rem = 0;
    for (size_t k = a.size(); k-- > 0;) {
      const uint64_t cur = (rem << 32) | a[k];
      quo[k] = (uint32_t)(cur / b[0]);
      rem = cur % b[0];
    }
    trim(quo);
    if (q) *q = quo;
    if (r) *r = rem ? Limbs{(uint32_t)rem} : Limbs{};
    return;
  }
  const uint32_t s = __builtin_clz(b.back());
  Limbs v = shl(b, s), u = shl(a, s);
  const size_t n = v.size();
  if (u.size() == a.size() + (s ? 0 : 0)) u.push_back(0);
  while (u.size() < a.size() + 1) u.push_back(0);
  const size_t m = u.size() - n - 1 + 1;
  Limbs quo(m, 0);
  for (size_t j = m; j-- > 0;) {
    const uint64_t num = ((uint64_t)u[j + n] << 32) | u[j + n - 1];
    uint64_t qhat = num / v[n - 1], rhat = num % v[n - 1];
    while (qhat > 0xFFFFFFFFull || qhat * v[n - 2] > ((rhat << 32) | u[j + n - 2])) {
      --qhat;
      rhat += v[n - 1];
      if (rhat > 0xFFFFFFFFull) break;
    }
    int64_t borrow = 0;
    uint64_t carry = 0;
    for (size_t i = 0; i < n; ++i) {
      const uint64_t p = qhat * v[i] + carry;
      carry = p >> 32;
      const int64_t t = (int64_t)u[i + j] - (int64_t)(uint32_t)p + borrow;
      u[i + j] = (uint32_t)t;
      borrow = t >> 32;
    }
    const int64_t t = (int64_t)u[j + n] - (int64_t)carry + borrow;
    u[j + n] = (uint32_t)t;
    if (t < 0) {  // add back
      --qhat;
      uint64_t c = 0;
      for (size_t i = 0; i < n; ++i) {
        c += (uint64_t)u[i + j] + v[i];
        u[i + j] = (uint32_t)c;
        c >>= 32;
      }
      u[j + n] += (uint32_t)c;
    }
    quo[j] = (uint32_t)qhat;
  }
  trim(quo);
  if (q) *q = quo;
  if (r) {
    u.resize(n);
    trim(u);
    // unnormalise
    Limbs rr(u.size(), 0);
    for (size_t k = 0; k < u.size(); ++k) rr[k] = (s ? (u[k] >> s) | (k + 1 < u.size() ? u[k + 1] << (32 - s) : 0) : u[k]);
    trim(rr);
    *r = rr;
  }
}
inline Limbs mod(const Limbs& a, const Limbs& m) {
  Limbs r;
  divmod_knuth(a, m, nullptr, &r);
  return r;
}
inline Limbs mulmod(const Limbs& a, const Limbs& b, const Limbs& m) { return mod(mul(a, b), m); }
inline Limbs div_exact(const Limbs& a, const Limbs& b) {
  Limbs q;
  divmod_knuth(a, b, &q, nullptr);
  return q;
}
inline bool is_even(const Limbs& a) { return a.empty() || (a[0] & 1u) == 0; }
// binary gcd
inline Limbs gcd(Limbs a, Limbs b) {
  if (a.empty()) return b;
  if (b.empty()) return a;
  uint32_t shift = 0;
  while (is_even(a) && is_even(b)) {
    a = shr1(a);
    b = shr1(b);
    ++shift;
  }
  while (is_even(a)) a = shr1(a);
  while (!b.empty()) {
    while (is_even(b)) b = shr1(b);
    if (cmp(a, b) > 0) std::swap(a, b);
    b = sub(b, a);
  }
  return shl(a, shift);
}
inline bool is_one(const Limbs& a) { return a.size() == 1 && a[0] == 1; }
// modular inverse by the extended binary method (m odd), false if none
inline bool modinv(const Limbs& y, const Limbs& m, Limbs* out) {
  Limbs a = mod(y, m), b = m, u{1}, v{};
  auto half = [&](Limbs& x) {  // x/2 mod m
    if (is_even(x)) x = shr1(x);
    else x = shr1(add(x, m));
  };
  while (!a.empty()) {
    if (is_even(a)) {
      a = shr1(a);
      half(u);
    } else {
      if (cmp(a, b) < 0) {
        std::swap(a, b);
        std::swap(u, v);
      }
      a = shr1(sub(a, b));
      Limbs d = cmp(u, v) >= 0 ? sub(u, v) : sub(add(u, m), v);
      half(d);
      u = d;
    }
  }
  if (!is_one(b)) return false;
  *out = v;
  return true;
}
inline void store(const Limbs& a, uint32_t* out, size_t n) {
  for (size_t k = 0; k < n; ++k) out[k] = k < a.size() ? a[k] : 0u;
}

// ---- allocation-free helpers on raw limb arrays (the per-pair / per-message
//      scans of the collect() pre-pass run these thousands of times)
// compare a (an limbs) with b (bn limbs)
inline int cmp_raw(const uint32_t* a, size_t an, const uint32_t* b, size_t bn) {
  const size_t n = std::max(an, bn);
  for (size_t k = n; k-- > 0;) {
    const uint32_t x = k < an ? a[k] : 0u, y = k < bn ? b[k] : 0u;
    if (x != y) return x < y ? -1 : 1;
  }
  return 0;
}
inline bool is_zero_raw(const uint32_t* a, size_t n) {
  for (size_t k = 0; k < n; ++k)
    if (a[k]) return false;
  return true;
}
inline uint32_t ctz_raw(const uint32_t* a, size_t n) {
  for (size_t k = 0; k < n; ++k)
    if (a[k]) return 32u * (uint32_t)k + (uint32_t)__builtin_ctz(a[k]);
  return 32u * (uint32_t)n;
}
// a >>= s (in place, n limbs)
inline void shr_raw(uint32_t* a, size_t n, uint32_t s) {
  const size_t w = s / 32;
  const uint32_t b = s % 32;
  for (size_t k = 0; k < n; ++k) {
    const uint32_t lo = k + w < n ? a[k + w] : 0u;
    const uint32_t hi = k + w + 1 < n ? a[k + w + 1] : 0u;
    a[k] = b ? (lo >> b) | (hi << (32 - b)) : lo;
  }
}
// gcd(a, b) == 1, binary gcd in place on copies (no allocation per step)
inline bool gcd_is_one(const uint32_t* a, size_t an, const uint32_t* b, size_t bn) {
  const size_t n = std::max(an, bn);
  std::vector<uint32_t> u(n, 0), v(n, 0);
  std::copy(a, a + an, u.begin());
  std::copy(b, b + bn, v.begin());
  const bool uz = is_zero_raw(u.data(), n), vz = is_zero_raw(v.data(), n);
  if (uz || vz) {   // gcd(0, x) = x
    const uint32_t* x = uz ? v.data() : u.data();
    if (uz && vz) return false;
    if (x[0] != 1) return false;
    return is_zero_raw(x + 1, n - 1);
  }
  if (!(u[0] & 1u) && !(v[0] & 1u)) return false;   // both even: 2 | gcd
  shr_raw(u.data(), n, ctz_raw(u.data(), n));
  size_t len = n;
  for (;;) {
    while (len > 1 && u[len - 1] == 0 && v[len - 1] == 0) --len;
    shr_raw(v.data(), len, ctz_raw(v.data(), len));
    if (cmp_raw(u.data(), len, v.data(), len) > 0) std::swap(u, v);
    // v -= u  (v >= u)
    int64_t br = 0;
    for (size_t k = 0; k < len; ++k) {
      const int64_t d = (int64_t)v[k] - u[k] + br;
      v[k] = (uint32_t)d;
      br = d >> 32;
    }
    if (is_zero_raw(v.data(), len)) break;
  }
  return u[0] == 1 && is_zero_raw(u.data() + 1, len - 1);
}
// true iff some prime in `primes` divides a (primes < 2^13, paired into
// products < 2^26 so one 64-bit remainder chain serves two primes)
inline bool has_small_factor(const uint32_t* a, size_t n, const std::vector<uint32_t>& primes) {
  for (size_t j = 0; j < primes.size(); j += 2) {
    const uint64_t p1 = primes[j], p2 = j + 1 < primes.size() ? primes[j + 1] : 1u;
    const uint64_t m = p1 * p2;
    uint64_t r = 0;
    for (size_t k = n; k-- > 0;) r = ((r << 32) | a[k]) % m;
    if (r % p1 == 0 || (p2 > 1 && r % p2 == 0)) return true;
  }
  return false;
}

// Trial division by a fixed prime list, several primes per pass: a mod M for
// M = p_1 ... p_k < 2^63 (k <= 4) as sum_j a_j (2^(32 j) mod M), independent
// 64 x 64 -> 128-bit products and one 128-bit reduction per M, then r mod p_i.
// Same answer as has_small_factor (2 primes per pass, a dependent 64-bit
// division per limb), ~10x fewer cycles: the correct-key primorial check of
// 3 072 keys was most of prepare's 29 ms "ck" phase at configs[4].
class SmallFactorSieve {
 public:
  SmallFactorSieve(const std::vector<uint32_t>& primes, size_t max_limbs) : L_(max_limbs) {
    for (size_t i = 0; i < primes.size();) {
      Group g;
      while (i < primes.size() && g.np < 4 && (unsigned __int128)g.m * primes[i] < ((unsigned __int128)1 << 63)) {
        g.m *= primes[i];
        g.p[g.np++] = primes[i++];
      }
      groups_.push_back(g);
    }
    pw_.resize(groups_.size() * L_);
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
      const uint64_t m = groups_[gi].m;
      uint64_t v = 1 % m;
      for (size_t k = 0; k < L_; ++k) {
        pw_[gi * L_ + k] = v;
        v = (uint64_t)(((unsigned __int128)v << 32) % m);
      }
    }
  }
  size_t max_limbs() const { return L_; }
  // does a prime of the list divide a (n <= max_limbs limbs; a = 0: yes)?
  bool divides(const uint32_t* a, size_t n) const {
    for (size_t gi = 0; gi < groups_.size(); ++gi) {
      const Group& g = groups_[gi];
      const uint64_t* pw = pw_.data() + gi * L_;
      unsigned __int128 acc = 0;
      for (size_t k = 0; k < n; ++k) acc += (unsigned __int128)a[k] * pw[k];
      const uint64_t r = (uint64_t)(acc % g.m);
      for (uint32_t t = 0; t < g.np; ++t)
        if (r % g.p[t] == 0) return true;
    }
    return false;
  }

 private:
  struct Group {
    uint64_t m = 1;
    uint32_t p[4] = {0, 0, 0, 0};
    uint32_t np = 0;
  };
  size_t L_;
  std::vector<Group> groups_;
  std::vector<uint64_t> pw_;
};

}  // namespace hbn
}  // namespace fsdkr
