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

#include <algorithm>
#include <vector>

#include "ctx.hpp"
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
