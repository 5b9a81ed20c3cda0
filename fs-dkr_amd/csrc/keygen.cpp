// Key generation entry points: batched Miller–Rabin.
//
// fsdkr_miller_rabin replaces the primality test of kzen-paillier 0.4.3
// Paillier::keypair_with_modulus_size (refresh_message.rs:118,
// ring_pedersen_proof.rs:50, add_party_message.rs:51; a dependency, not
// vendored).  The host splits c - 1 = d 2^s; the GPU computes b^d mod c with
// the batched modexp engine (each candidate its own modulus) and the witness
// tail (prime.hip).
#include "fsdkr/fsdkr.h"

#include <hip/hip_runtime.h>
#include <openssl/evp.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "evp_sha.hpp"
#include "hostbn.hpp"
#include "kernels.h"

using namespace fsdkr;

extern "C" int fsdkr_miller_rabin(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* cand,
                                  const uint32_t* bases, uint32_t* verdict) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!cand || !bases || !verdict) {
    c->fail("fsdkr_miller_rabin: null pointer");
    return FSDKR_E_ARG;
  }
  if (mod_limbs != kPrimeLimbs && mod_limbs != 64 && mod_limbs != 96) {
    c->fail("fsdkr_miller_rabin: unsupported candidate width %u limbs", mod_limbs);
    return FSDKR_E_UNSUPPORTED;
  }
  const size_t K = mod_limbs;
  std::vector<uint32_t> d((size_t)count * K, 0u), s(count);
  uint32_t s_max = 0;
  for (uint32_t i = 0; i < count; ++i) {
    const uint32_t* x = cand + (size_t)i * K;
    bool big = false;
    for (size_t k = 1; k < K; ++k) big = big || x[k] != 0;
    if ((x[0] & 1u) == 0 || (!big && x[0] < 5)) {
      c->fail("fsdkr_miller_rabin: candidate %u is even or below 5", i);
      return FSDKR_E_ARG;
    }
    // c - 1 = d 2^s  (c odd: c - 1 only clears bit 0)
    uint32_t tz = 1;
    size_t w = 0;
    uint32_t lo = x[0] & ~1u;
    while (lo == 0) lo = x[++w];   // c - 1 > 0, so some limb is non-zero
    tz = 32u * (uint32_t)w + (uint32_t)__builtin_ctz(lo);
    s[i] = tz;
    s_max = std::max(s_max, tz);
    uint32_t* di = d.data() + (size_t)i * K;
    const uint32_t ws = tz >> 5, bs = tz & 31;
    for (size_t k = 0; k + ws < K; ++k) {
      const uint32_t a0 = (k + ws == 0) ? (x[0] & ~1u) : x[k + ws];
      const uint32_t a1 = (k + ws + 1 < K) ? x[k + ws + 1] : 0u;
      di[k] = bs ? (a0 >> bs) | (a1 << (32 - bs)) : a0;
    }
  }
  const size_t nb = sizeof(uint32_t) * (size_t)count * K;
  uint32_t* d_cand = (uint32_t*)c->buf("mr_cand", nb);
  uint32_t* d_base = (uint32_t*)c->buf("mr_base", nb);
  uint32_t* d_exp = (uint32_t*)c->buf("mr_exp", nb);
  uint32_t* d_x = (uint32_t*)c->buf("mr_x", nb);
  uint32_t* d_s = (uint32_t*)c->buf("mr_s", 4 * (size_t)count);
  uint32_t* d_v = (uint32_t*)c->buf("mr_v", 4 * (size_t)count);
  if (!d_cand || !d_base || !d_exp || !d_x || !d_s || !d_v) {
    c->fail("fsdkr_miller_rabin: device allocation failed");
    return FSDKR_E_OOM;
  }
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_cand, cand, nb, hipMemcpyHostToDevice, c->stream), "H2D cand")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_base, bases, nb, hipMemcpyHostToDevice, c->stream), "H2D bases")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_exp, d.data(), nb, hipMemcpyHostToDevice, c->stream), "H2D d")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_s, s.data(), 4 * (size_t)count, hipMemcpyHostToDevice, c->stream), "H2D s")))
    return rc;
  uint32_t* d_consts = nullptr;
  if ((rc = setup_moduli(c, mod_limbs, d_cand, count, &d_consts, "mr"))) return rc;
  ModexpJob job;
  job.k32 = mod_limbs;
  for (uint32_t i = 0; i < count; ++i) {
    const uint32_t* di = d.data() + (size_t)i * K;
    int top = (int)K - 1;
    while (top > 0 && di[top] == 0) --top;
    const uint32_t eb = di[top] ? 32u * (uint32_t)top + 32u - (uint32_t)__builtin_clz(di[top]) : 1u;
    job.add((uint64_t)(uintptr_t)(d_base + (size_t)i * K), mod_limbs, (uint64_t)(uintptr_t)(d_exp + (size_t)i * K),
            mod_limbs, eb, i);
  }
  {   // the candidates are secret (the accepted one is a prime factor of a key)
    CtScope ct(c);
    if ((rc = launch_modexp_job(c, job, d_consts, d_x, "mr"))) return rc;
  }
  MrTailArgs a{d_x, d_consts, d_s, s_max, d_v, count};
  c->mark("mr_tail", true);
  rc = c->hip_check(mr_tail(mod_limbs, a, c->stream), "mr_tail launch");
  c->mark("mr_tail", false);
  if (rc) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(verdict, d_v, 4 * (size_t)count, hipMemcpyDeviceToHost, c->stream),
                         "D2H verdict")))
    return rc;
  return c->sync();
}

// ---- the prime walk (fsdkr_sample_primes) -------------------------------------
namespace {

constexpr uint32_t kSieveLimit = 2000;
constexpr uint32_t kMrRounds = 8;
constexpr uint32_t kMaxPasses = 1000;

struct SmallPrimes {
  std::vector<uint32_t> p, half;   // odd primes below 2000 and 2^-1 mod p
  SmallPrimes() {
    std::vector<bool> comp(kSieveLimit, false);
    for (uint32_t i = 2; i < kSieveLimit; ++i) {
      if (comp[i]) continue;
      for (uint32_t j = i * i; j < kSieveLimit; j += i) comp[j] = true;
      if (i > 2) {
        p.push_back(i);
        half.push_back((i + 1) / 2);
      }
    }
  }
};
const SmallPrimes& small_primes() {
  static const SmallPrimes sp;
  return sp;
}

uint32_t mr_limbs(uint32_t bits) {
  for (uint32_t w : {32u, 64u, 96u})
    if (bits <= 32 * w) return w;
  return 0;
}

// offsets k in [0, span) with start + 2k divisible by no odd prime below 2000
std::vector<uint32_t> sieve(const hbn::Limbs& start, uint32_t span) {
  const SmallPrimes& sp = small_primes();
  std::vector<uint8_t> keep(span, 1);
  for (size_t i = 0; i < sp.p.size(); ++i) {
    const uint64_t p = sp.p[i];
    const uint64_t first = ((p - hbn::mod_small(start, (uint32_t)p)) % p) * sp.half[i] % p;
    for (uint64_t k = first; k < span; k += p) keep[k] = 0;
  }
  std::vector<uint32_t> out;
  for (uint32_t k = 0; k < span; ++k)
    if (keep[k]) out.push_back(k);
  return out;
}

// 2 + (SHA-256("fsdkr-mr" | c | j | ctr) stream, nb + 8 bytes, big-endian) mod (c - 3)
bool witness_bases(const hbn::Limbs& c, std::vector<hbn::Limbs>* out) {
  const uint32_t nb = (hbn::bitlen(c) + 7) / 8;
  std::vector<uint8_t> cb(nb);
  for (uint32_t i = 0; i < nb; ++i) {
    const uint32_t byte = nb - 1 - i;   // big-endian position i holds little-endian byte nb-1-i
    cb[i] = (uint8_t)(c[byte / 4] >> (8 * (byte % 4)));
  }
  const hbn::Limbs cm3 = hbn::sub(c, hbn::Limbs{3});
  EVP_MD_CTX* md = EVP_MD_CTX_new();
  if (!md) return false;
  bool ok = true;
  out->clear();
  for (uint32_t j = 0; j < kMrRounds && ok; ++j) {
    std::vector<uint8_t> stream;
    for (uint32_t ctr = 0; stream.size() < nb + 8; ++ctr) {
      uint8_t le[8] = {(uint8_t)j, (uint8_t)(j >> 8), (uint8_t)(j >> 16), (uint8_t)(j >> 24),
                       (uint8_t)ctr, (uint8_t)(ctr >> 8), (uint8_t)(ctr >> 16), (uint8_t)(ctr >> 24)};
      uint8_t d[32];
      unsigned int len = 0;
      ok = ok && EVP_DigestInit_ex(md, sha256_md(), nullptr) == 1 &&
           EVP_DigestUpdate(md, "fsdkr-mr", 8) == 1 && EVP_DigestUpdate(md, cb.data(), nb) == 1 &&
           EVP_DigestUpdate(md, le, 8) == 1 && EVP_DigestFinal_ex(md, d, &len) == 1;
      stream.insert(stream.end(), d, d + 32);
    }
    const size_t L = nb + 8;
    std::vector<uint32_t> w((L + 3) / 4, 0u);
    for (size_t i = 0; i < L; ++i) {
      const size_t byte = L - 1 - i;
      w[byte / 4] |= (uint32_t)stream[i] << (8 * (byte % 4));
    }
    out->push_back(hbn::add(hbn::mod(hbn::from(w.data(), w.size()), cm3), hbn::Limbs{2}));
  }
  EVP_MD_CTX_free(md);
  return ok;
}

struct Walk {
  hbn::Limbs start;
  std::vector<uint32_t> offs;
  size_t pos = 0;
  std::vector<hbn::Limbs> passers;   // base-2 passers of the current window, in walk order
};

}  // namespace

extern "C" int fsdkr_sample_primes(fsdkr_ctx* ctx, uint32_t bits, uint32_t count, uint32_t window, uint32_t span,
                                   fsdkr_draw_bits_fn draw, void* user, uint32_t* out, uint32_t limbs) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  const uint32_t K = mr_limbs(bits);
  if (bits < 64 || !K || !draw || !out || limbs < (bits + 31) / 32) {
    c->fail("fsdkr_sample_primes: bad argument (bits %u, limbs %u)", bits, limbs);
    return bits < 64 || !K ? FSDKR_E_UNSUPPORTED : FSDKR_E_ARG;
  }
  if (!window) window = std::max(32u, bits / 8);
  if (!span) span = 4 * bits;
  const uint32_t dl = (bits + 31) / 32;
  auto new_walk = [&](Walk& w) -> int {
    std::vector<uint32_t> r(dl, 0u);
    if (draw(user, bits, r.data(), dl) != 0) {
      c->fail("fsdkr_sample_primes: the draw callback failed");
      return FSDKR_E_ARG;
    }
    if (bits % 32) r[dl - 1] &= (1u << (bits % 32)) - 1;
    r[(bits - 1) / 32] |= 1u << ((bits - 1) % 32);
    r[(bits - 2) / 32] |= 1u << ((bits - 2) % 32);
    r[0] |= 1u;
    w = Walk();
    w.start = hbn::from(r.data(), dl);
    // the walk stays below 2^bits (a `bits`-bit prime): start + 2k < 2^bits
    uint32_t wspan = span;
    const hbn::Limbs room = hbn::sub(hbn::shl(hbn::Limbs{1}, bits), w.start);   // > 0: start < 2^bits
    // (in 64 bits: room = 0xFFFFFFFF is odd and reachable, room + 1 must not wrap)
    if (hbn::bitlen(room) <= 32)
      wspan = (uint32_t)std::min<uint64_t>(span, (room.empty() ? 0ull : (uint64_t)room[0] + 1ull) / 2ull);
    w.offs = sieve(w.start, wspan);
    return FSDKR_OK;
  };
  auto run_mr = [&](const std::vector<hbn::Limbs>& cands, const std::vector<hbn::Limbs>& bases,
                    std::vector<uint32_t>* v) -> int {
    v->assign(cands.size(), 0u);
    if (cands.empty()) return FSDKR_OK;
    std::vector<uint32_t> C(cands.size() * K, 0u), B(cands.size() * K, 0u);
    for (size_t i = 0; i < cands.size(); ++i) {
      hbn::store(cands[i], C.data() + i * K, K);
      hbn::store(bases[i], B.data() + i * K, K);
    }
    return fsdkr_miller_rabin(ctx, K, (uint32_t)cands.size(), C.data(), B.data(), v->data());
  };
  std::vector<Walk> walks(count);
  std::vector<hbn::Limbs> res(count);
  std::vector<uint8_t> done(count, 0);
  int rc;
  for (uint32_t w = 0; w < count; ++w)
    if ((rc = new_walk(walks[w]))) return rc;
  uint32_t passes = 0;
  for (;;) {
    std::vector<uint32_t> active;
    for (uint32_t w = 0; w < count; ++w)
      if (!done[w] && walks[w].pos < walks[w].offs.size()) active.push_back(w);
    if (active.empty()) {
      std::vector<uint32_t> failed;
      for (uint32_t w = 0; w < count; ++w)
        if (!done[w]) failed.push_back(w);
      if (failed.empty()) break;
      if (++passes > kMaxPasses) {
        c->fail("fsdkr_sample_primes: no prime after %u walk passes", kMaxPasses);
        return FSDKR_E_ARG;
      }
      for (uint32_t w : failed)   // a new pass, in walk order
        if ((rc = new_walk(walks[w]))) return rc;
      continue;
    }
    // base 2 on the next window of every unsettled walk
    std::vector<hbn::Limbs> cands, bases;
    std::vector<uint32_t> owner;
    for (uint32_t w : active) {
      Walk& wk = walks[w];
      const size_t end = std::min(wk.offs.size(), wk.pos + window);
      for (size_t k = wk.pos; k < end; ++k) {
        cands.push_back(hbn::add(wk.start, hbn::Limbs{2 * wk.offs[k]}));
        bases.push_back(hbn::Limbs{2});
        owner.push_back(w);
      }
      wk.pos += window;
    }
    std::vector<uint32_t> v;
    if ((rc = run_mr(cands, bases, &v))) return rc;
    for (size_t i = 0; i < cands.size(); ++i)
      if (v[i]) walks[owner[i]].passers.push_back(cands[i]);
    // the extra rounds on each walk's first passer; a failure tries the next
    for (;;) {
      std::vector<uint32_t> head;
      for (uint32_t w : active)
        if (!walks[w].passers.empty() && !done[w]) head.push_back(w);
      if (head.empty()) break;
      cands.clear();
      bases.clear();
      owner.clear();
      std::vector<hbn::Limbs> wb;
      for (uint32_t w : head) {
        const hbn::Limbs& cand = walks[w].passers.front();
        if (!witness_bases(cand, &wb)) {
          c->fail("fsdkr_sample_primes: SHA-256 (OpenSSL EVP) failed");
          return FSDKR_E_ARG;
        }
        for (const hbn::Limbs& b : wb) {
          cands.push_back(cand);
          bases.push_back(b);
          owner.push_back(w);
        }
      }
      if ((rc = run_mr(cands, bases, &v))) return rc;
      std::vector<uint8_t> pass(count, 1);
      for (size_t i = 0; i < cands.size(); ++i)
        if (!v[i]) pass[owner[i]] = 0;
      for (uint32_t w : head) {
        hbn::Limbs cand = walks[w].passers.front();
        walks[w].passers.erase(walks[w].passers.begin());
        if (pass[w]) {
          res[w] = cand;
          done[w] = 1;
          walks[w].passers.clear();
        }
      }
    }
  }
  for (uint32_t w = 0; w < count; ++w) {
    std::fill(out + (size_t)w * limbs, out + (size_t)(w + 1) * limbs, 0u);
    hbn::store(res[w], out + (size_t)w * limbs, limbs);
  }
  return FSDKR_OK;
}
