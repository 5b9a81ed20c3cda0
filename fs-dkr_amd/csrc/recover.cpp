// Share recovery building blocks of collect() (refresh_message.rs:367-373,
// 439-464): Paillier decryption of the homomorphically summed share and the
// secp256k1 multi-scalar multiplications that rebuild pk_vec and y.  The
// exponentiation and EC work run on the GPU; the O(1) L-function / mu
// arithmetic of kzen-paillier decrypt runs on the host.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "fsdkr/fsdkr.h"
#include "hostbn.hpp"
#include "kernels.h"
#include "verify.h"

using namespace fsdkr;

extern "C" {

int fsdkr_paillier_decrypt(fsdkr_ctx* ctx, uint32_t nl, const uint32_t* c, const uint32_t* p, const uint32_t* q,
                           uint32_t* m_out) {
  Ctx* cx = reinterpret_cast<Ctx*>(ctx);
  if (!cx || !c || !p || !q || !m_out) return FSDKR_E_ARG;
  const uint32_t nn = 2 * nl;
  if (!shape_digits(nn)) {
    cx->fail("fsdkr_paillier_decrypt: unsupported width %u", nl);
    return FSDKR_E_UNSUPPORTED;
  }
  const hbn::Limbs P = hbn::from(p, nl), Q = hbn::from(q, nl);
  const hbn::Limbs N = hbn::mul(P, Q), NN = hbn::mul(N, N);
  const hbn::Limbs lam = hbn::mul(hbn::sub(P, hbn::Limbs{1}), hbn::sub(Q, hbn::Limbs{1}));
  if (hbn::bitlen(NN) > 32 * nn || hbn::is_even(N)) {
    cx->fail("fsdkr_paillier_decrypt: bad key");
    return FSDKR_E_ARG;
  }
  // u = c^lambda mod N^2 on the GPU
  std::vector<uint32_t> cb(nn), eb(nl), mb(nn), ub(nn);
  hbn::store(hbn::mod(hbn::from(c, nn), NN), cb.data(), nn);
  hbn::store(lam, eb.data(), nl);
  hbn::store(NN, mb.data(), nn);
  const uint32_t idx = 0;
  int rc = fsdkr_modexp_batch(ctx, nn, 1, cb.data(), eb.data(), nl, &idx, mb.data(), 1, ub.data());
  if (rc) return rc;
  // m = L(u) * lambda^-1 mod N,  L(u) = (u - 1) / N
  hbn::Limbs Lq, r;
  hbn::divmod(hbn::sub(hbn::from(ub.data(), nn), hbn::Limbs{1}), N, &Lq, &r);
  hbn::Limbs mu;
  if (!hbn::modinv(lam, N, &mu)) {
    cx->fail("fsdkr_paillier_decrypt: lambda not invertible mod N");
    return FSDKR_E_ARG;
  }
  hbn::store(hbn::mulmod(Lq, mu, N), m_out, nl);
  return FSDKR_OK;
}

int fsdkr_ec_msm(fsdkr_ctx* ctx, uint32_t count, uint32_t terms, const uint32_t* points, const uint32_t* scalars,
                 uint32_t* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c || !points || !scalars || !out || terms == 0) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  const size_t np = (size_t)count * terms;
  uint8_t* d = (uint8_t*)c->buf("msm", np * 16 * 4 + np * 8 * 4 + np * 8 + (size_t)count * 16 * 4 + 1024);
  if (!d) return FSDKR_E_OOM;
  uint32_t* d_pts = (uint32_t*)d;
  uint32_t* d_sc = d_pts + np * 16;
  uint64_t* d_ptr = (uint64_t*)(d_sc + np * 8);
  uint32_t* d_out = (uint32_t*)(d_ptr + np);
  std::vector<uint64_t> ptrs(np);
  for (size_t k = 0; k < np; ++k) ptrs[k] = (uint64_t)(uintptr_t)(d_pts + k * 16);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_pts, points, np * 64, hipMemcpyHostToDevice, c->stream), "H2D pts")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_sc, scalars, np * 32, hipMemcpyHostToDevice, c->stream), "H2D sc")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_ptr, ptrs.data(), np * 8, hipMemcpyHostToDevice, c->stream), "H2D ptr")))
    return rc;
  EcMsmArgs a{d_ptr, d_sc, terms, d_out, count};
  c->mark("ec", true);
  rc = c->hip_check(launch_ec_msm(a, c->stream), "ec_msm");
  c->mark("ec", false);
  if (rc) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(out, d_out, (size_t)count * 64, hipMemcpyDeviceToHost, c->stream), "D2H")))
    return rc;
  return c->sync();
}

}  // extern "C"
