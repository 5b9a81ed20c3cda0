// Share recovery building blocks of collect() (refresh_message.rs:367-373,
// 439-464): Paillier decryption of the homomorphically summed share and the
// secp256k1 multi-scalar multiplications that rebuild pk_vec and y.  The
// exponentiation and EC work run on the GPU; the O(1) L-function / mu
// arithmetic of kzen-paillier decrypt runs on the host.
#include <hip/hip_runtime.h>
#include <openssl/bn.h>
#include <openssl/crypto.h>
#include <openssl/ec.h>
#include <openssl/obj_mac.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <cstring>
#include <thread>
#include <vector>

#include "ctx.hpp"
#include "fsdkr/fsdkr.h"
#include "hostbn.hpp"
#include "kernels.h"
#include "verify.h"

using namespace fsdkr;

namespace {
// f(begin, end) over [0, n) on the host worker threads
template <class F>
void parallel_for_host(size_t n, size_t grain, F&& f) {
  const size_t chunks = std::min<size_t>(host_threads(), (n + grain - 1) / grain);
  if (chunks <= 1) {
    f((size_t)0, n);
    return;
  }
  struct Part {
    F* f;
    size_t n, chunks;
  } part{&f, n, chunks};
  host_pool_run(chunks, [](void* a, size_t c) {
    const Part& x = *static_cast<const Part*>(a);
    (*x.f)(x.n * c / x.chunks, x.n * (c + 1) / x.chunks);
  }, &part);
}
}  // namespace

extern "C" {

int fsdkr_paillier_decrypt_multi(fsdkr_ctx* ctx, uint32_t nl, uint32_t count, const uint32_t* c,
                                 const uint32_t* key_idx, const uint32_t* p, const uint32_t* q, uint32_t n_keys,
                                 uint32_t* m_out) {
  Ctx* cx = reinterpret_cast<Ctx*>(ctx);
  if (!cx || !c || !key_idx || !p || !q || !m_out || n_keys == 0) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  const uint32_t nn = 2 * nl;
  if (!shape_digits(nl)) {
    cx->fail("fsdkr_paillier_decrypt: unsupported width %u", nl);
    return FSDKR_E_UNSUPPORTED;
  }
  for (uint32_t k = 0; k < count; ++k)
    if (key_idx[k] >= n_keys) {
      cx->fail("fsdkr_paillier_decrypt: key_idx[%u] out of range", k);
      return FSDKR_E_ARG;
    }
  StreamScope scope(cx, cx->aux_stream());   // overlaps a launched collect batch
  PrioScope prio(cx, 3);                      // few waves on the critical path: win issue arbitration
  // kzen-paillier CRT decryption with g = N + 1.  Its constants have closed forms:
  // (1+N)^(p-1) = 1 + (p-1)N mod p^2 and (p-1)N = -q p mod p^2, so
  // h_p = L_p(g^(p-1) mod p^2)^-1 = (-q)^-1 mod p = p - q^-1 mod p (likewise h_q);
  // the two inverses per key run on the GPU (lane-cooperative inverse kernel).
  struct Key {
    hbn::Limbs P, Q, PP, QQ, pm1, qm1;
    bool ok;
  };
  std::vector<Key> keys(n_keys);
  std::vector<uint32_t> invy((size_t)2 * n_keys * nl, 0u), invm((size_t)2 * n_keys * nl, 0u);
  std::vector<uint8_t> bad(n_keys, 0);
  for (uint32_t k = 0; k < n_keys; ++k) {
    Key& K = keys[k];
    K.P = hbn::from(p + (size_t)k * nl, nl);
    K.Q = hbn::from(q + (size_t)k * nl, nl);
    K.PP = hbn::mul(K.P, K.P);
    K.QQ = hbn::mul(K.Q, K.Q);
    const hbn::Limbs N = hbn::mul(K.P, K.Q);
    K.ok = !hbn::is_even(K.P) && !hbn::is_even(K.Q) && hbn::bitlen(K.PP) <= 32 * nl &&
           hbn::bitlen(K.QQ) <= 32 * nl && hbn::bitlen(N) <= 32 * nl && !(K.P.size() == 1 && K.P[0] == 1) &&
           !(K.Q.size() == 1 && K.Q[0] == 1);
    if (!K.ok) {
      cx->fail("fsdkr_paillier_decrypt: bad key %u", k);
      return FSDKR_E_ARG;
    }
    K.pm1 = hbn::sub(K.P, hbn::Limbs{1});
    K.qm1 = hbn::sub(K.Q, hbn::Limbs{1});
    hbn::store(hbn::mod(K.Q, K.P), invy.data() + (size_t)(2 * k) * nl, nl);      // q^-1 mod p
    hbn::store(K.P, invm.data() + (size_t)(2 * k) * nl, nl);
    hbn::store(hbn::mod(K.P, K.Q), invy.data() + (size_t)(2 * k + 1) * nl, nl);  // p^-1 mod q
    hbn::store(K.Q, invm.data() + (size_t)(2 * k + 1) * nl, nl);
  }
  std::vector<uint32_t> invo((size_t)2 * n_keys * nl), unit(2 * (size_t)n_keys);
  int rc = fsdkr_mod_inverse(ctx, nl, 2 * n_keys, invy.data(), invm.data(), invo.data(), unit.data());
  if (rc) return rc;
  for (uint32_t k = 0; k < n_keys; ++k)
    if (!unit[2 * k] || !unit[2 * k + 1]) {
      cx->fail("fsdkr_paillier_decrypt: degenerate key %u", k);
      return FSDKR_E_ARG;
    }
  // 2*count GPU exponentiations: (c mod p^2)^(p-1) mod p^2, (c mod q^2)^(q-1) mod q^2
  std::vector<uint32_t> base((size_t)2 * count * nl), ex((size_t)2 * count * nl), idx(2 * count),
      mods((size_t)2 * n_keys * nl), outv((size_t)2 * count * nl);
  for (uint32_t k = 0; k < n_keys; ++k) {
    hbn::store(keys[k].PP, mods.data() + (size_t)(2 * k) * nl, nl);
    hbn::store(keys[k].QQ, mods.data() + (size_t)(2 * k + 1) * nl, nl);
  }
  parallel_for_host(count, 16, [&](size_t b0, size_t b1) {
    for (size_t i = b0; i < b1; ++i) {
      const Key& K = keys[key_idx[i]];
      const hbn::Limbs ck = hbn::from(c + i * nn, nn);
      hbn::store(hbn::mod(ck, K.PP), base.data() + (2 * i) * nl, nl);
      hbn::store(hbn::mod(ck, K.QQ), base.data() + (2 * i + 1) * nl, nl);
      hbn::store(K.pm1, ex.data() + (2 * i) * nl, nl);
      hbn::store(K.qm1, ex.data() + (2 * i + 1) * nl, nl);
      idx[2 * i] = 2 * key_idx[i];
      idx[2 * i + 1] = 2 * key_idx[i] + 1;
    }
  });
  // secret exponents p - 1, q - 1: regular-access modexp
  rc = fsdkr_modexp_batch_ct(ctx, nl, 2 * count, base.data(), ex.data(), nl, idx.data(), mods.data(), 2 * n_keys,
                             outv.data());
  if (rc) return rc;
  const hbn::Limbs one{1};
  parallel_for_host(count, 16, [&](size_t b0, size_t b1) {
    for (size_t i = b0; i < b1; ++i) {
      const uint32_t k = key_idx[i];
      const Key& K = keys[k];
      const hbn::Limbs qinv = hbn::from(invo.data() + (size_t)(2 * k) * nl, nl);
      const hbn::Limbs pinv = hbn::from(invo.data() + (size_t)(2 * k + 1) * nl, nl);
      const hbn::Limbs hp = hbn::sub(K.P, qinv), hq = hbn::sub(K.Q, pinv);
      const hbn::Limbs up = hbn::from(outv.data() + (2 * i) * nl, nl);
      const hbn::Limbs uq = hbn::from(outv.data() + (2 * i + 1) * nl, nl);
      const hbn::Limbs mp = hbn::mulmod(hbn::div_exact(hbn::sub(up.empty() ? one : up, one), K.P), hp, K.P);
      const hbn::Limbs mq = hbn::mulmod(hbn::div_exact(hbn::sub(uq.empty() ? one : uq, one), K.Q), hq, K.Q);
      // m = mq + q * ((mp - mq) q^-1 mod p)
      const hbn::Limbs mqp = hbn::mod(mq, K.P);
      const hbn::Limbs d = hbn::cmp(mp, mqp) >= 0 ? hbn::sub(mp, mqp) : hbn::sub(hbn::add(mp, K.P), mqp);
      const hbn::Limbs m = hbn::add(mq, hbn::mul(K.Q, hbn::mulmod(d, qinv, K.P)));
      hbn::store(m, m_out + i * nl, nl);
    }
  });
  return FSDKR_OK;
}

int fsdkr_paillier_decrypt(fsdkr_ctx* ctx, uint32_t nl, uint32_t count, const uint32_t* c, const uint32_t* p,
                           const uint32_t* q, uint32_t* m_out) {
  if (count == 0) return ctx ? FSDKR_OK : FSDKR_E_ARG;   // an empty batch: nothing to decrypt
  std::vector<uint32_t> key_idx(count, 0u);
  return fsdkr_paillier_decrypt_multi(ctx, nl, count, c, key_idx.data(), p, q, 1, m_out);
}

// Job 1 (refresh_message.rs:72-84): c_k = (1 + m_k N) * r_k^N mod N^2 for the
// n shares of distribute(), each under its receiver's key ns[n_idx[k]].
int fsdkr_paillier_encrypt(fsdkr_ctx* ctx, uint32_t nl, uint32_t count, const uint32_t* m, uint32_t ml,
                           const uint32_t* r, const uint32_t* n_idx, const uint32_t* ns, uint32_t n_keys,
                           uint32_t* out) {
  Ctx* cx = reinterpret_cast<Ctx*>(ctx);
  if (!cx || !m || !r || !n_idx || !ns || !out || ml == 0 || n_keys == 0) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  const uint32_t nn = 2 * nl;
  if (!shape_digits(nn)) return FSDKR_E_UNSUPPORTED;
  std::vector<uint32_t> NNs((size_t)n_keys * nn);
  for (uint32_t k = 0; k < n_keys; ++k) {
    const hbn::Limbs N = hbn::from(ns + (size_t)k * nl, nl);
    if (hbn::is_even(N)) {
      cx->fail("fsdkr_paillier_encrypt: even modulus");
      return FSDKR_E_ARG;
    }
    hbn::store(hbn::mul(N, N), NNs.data() + (size_t)k * nn, nn);
  }
  for (uint32_t k = 0; k < count; ++k)
    if (n_idx[k] >= n_keys) return FSDKR_E_ARG;
  // device image: ns | NNs | m | r | one | outputs | descriptors
  const size_t b_ns = 0, b_nns = b_ns + (size_t)n_keys * nl * 4, b_m = b_nns + NNs.size() * 4;
  const size_t b_r = b_m + (size_t)count * ml * 4, b_one = b_r + (size_t)count * nl * 4;
  const size_t b_gm = b_one + (size_t)nn * 4, b_rn = b_gm + (size_t)count * nn * 4;
  const size_t b_out = b_rn + (size_t)count * nn * 4, b_desc = b_out + (size_t)count * nn * 4;
  // r^N mod N^2: every share under key k has exponent N_k.  At 4096 bits the job is
  // regrouped by key so every wave shares its exponent and runs sliding windows
  // (modexp_slide_kernel, as fsdkr_modexp_keyed_device: metric 2); pads rewrite
  // their own chain's row.  Other widths keep fixed windows.  The base r and the
  // exponent schedule's memory accesses depend on N only (public).
  ModexpJob job;
  job.k32 = nn;
  auto A0 = [](size_t off) { return (uint64_t)off; };   // offsets until the buffer exists
  for (uint32_t k = 0; k < count; ++k)
    job.add(A0(b_r + (size_t)k * nl * 4), nl, A0(b_ns + (size_t)n_idx[k] * nl * 4), nl, 32 * nl, n_idx[k]);
  uint32_t G = 0, flags = 0;
  if (nn == 128 && !cx->ct) {
    G = keyed_lanes(count);
    if (group_by_exponent(job, 64 / G, kPadSelf)) flags = kDescOutIdx | kDescSlide;
    else G = 0;
  }
  const size_t total = b_desc + job.desc_bytes() + (size_t)count * (16 + sizeof(Prod3Operand) + 4) + 8 * 256 + 4096;
  uint8_t* d = (uint8_t*)cx->buf("enc", total);
  if (!d) return FSDKR_E_OOM;
  for (size_t i = 0; i < job.size(); ++i) {   // offsets -> device addresses
    job.base_ptr[i] += (uint64_t)(uintptr_t)d;
    job.exp_ptr[i] += (uint64_t)(uintptr_t)d;
  }
  std::vector<uint8_t> img(b_desc, 0);
  memcpy(img.data() + b_ns, ns, (size_t)n_keys * nl * 4);
  memcpy(img.data() + b_nns, NNs.data(), NNs.size() * 4);
  memcpy(img.data() + b_m, m, (size_t)count * ml * 4);
  memcpy(img.data() + b_r, r, (size_t)count * nl * 4);
  ((uint32_t*)(img.data() + b_one))[0] = 1;
  auto A = [&](size_t off) { return (uint64_t)(uintptr_t)(d + off); };
  // binom: gm = 1 + m*N  (m < N for a share; reduced mod N^2 by prod3 anyway)
  std::vector<uint64_t> s_ptr(count), n_ptr(count);
  std::vector<Prod3Operand> ops(count);
  std::vector<uint32_t> midx(count);
  for (uint32_t k = 0; k < count; ++k) {
    s_ptr[k] = A(b_m + (size_t)k * ml * 4);
    n_ptr[k] = A(b_ns + (size_t)n_idx[k] * nl * 4);
    ops[k] = {A(b_gm + (size_t)k * nn * 4), A(b_rn + (size_t)k * nn * 4), A(b_one), nn, nn, nn, 0};
    midx[k] = n_idx[k];
  }
  auto app = [&](const void* src, size_t bytes) {
    const size_t o = (img.size() + 255) & ~(size_t)255;
    img.resize(o + bytes);
    memcpy(img.data() + o, src, bytes);
    return o;
  };
  const size_t o_s = app(s_ptr.data(), count * 8), o_n = app(n_ptr.data(), count * 8);
  const size_t o_ops = app(ops.data(), count * sizeof(Prod3Operand)), o_midx = app(midx.data(), count * 4);
  std::vector<uint8_t> jd;
  job.pack(jd);
  const size_t o_job = app(jd.data(), jd.size());
  if (img.size() > total) return FSDKR_E_ARG;
  int rc = cx->hip_check(hipMemcpyAsync(d, img.data(), img.size(), hipMemcpyHostToDevice, cx->stream), "H2D enc");
  if (rc) return rc;
  uint32_t* consts = nullptr;
  if ((rc = setup_moduli(cx, nn, (const uint32_t*)(d + b_nns), n_keys, &consts, "enc"))) return rc;
  BinomArgs ba{(const uint64_t*)(d + o_s), (const uint64_t*)(d + o_n), ml, nl, nn, (uint32_t*)(d + b_gm), count};
  if ((rc = cx->hip_check(launch_binom(ba, cx->stream), "binom"))) return rc;
  if ((rc = launch_modexp_desc(cx, nn, (uint32_t)job.size(), 32 * nl, d + o_job, consts, (uint32_t*)(d + b_rn),
                                nullptr, "mxtable", cx->prio, G, flags)))
    return rc;
  Prod3Args pa{(const Prod3Operand*)(d + o_ops), (const uint32_t*)(d + o_midx), consts, (uint32_t*)(d + b_out), count};
  // prod3 computes a*b*c mod N^2 exactly: (1+mN) * r^N * 1
  if ((rc = cx->hip_check(launch_prod3(nn, pa, cx->stream), "prod3"))) return rc;
  if ((rc = cx->hip_check(hipMemcpyAsync(out, d + b_out, (size_t)count * nn * 4, hipMemcpyDeviceToHost, cx->stream),
                          "D2H enc")))
    return rc;
  return cx->sync();
}

int fsdkr_ec_msm(fsdkr_ctx* ctx, uint32_t count, uint32_t terms, const uint32_t* points, const uint32_t* scalars,
                 uint32_t* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c || !points || !scalars || !out || terms == 0) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  StreamScope scope(c, c->aux_stream());   // overlaps a launched collect batch
  PrioScope prio(c, 3);
  const size_t np = (size_t)count * terms;
  uint8_t* d = (uint8_t*)c->buf("msm", np * 16 * 4 + np * 8 * 4 + np * 8 + (size_t)count * 16 * 4 + np * 96 + 1024);
  if (!d) return FSDKR_E_OOM;
  uint32_t* d_pts = (uint32_t*)d;
  uint32_t* d_sc = d_pts + np * 16;
  uint64_t* d_ptr = (uint64_t*)(d_sc + np * 8);
  uint32_t* d_out = (uint32_t*)(d_ptr + np);
  uint32_t* d_scr = d_out + (size_t)count * 16;
  std::vector<uint64_t> ptrs(np);
  for (size_t k = 0; k < np; ++k) ptrs[k] = (uint64_t)(uintptr_t)(d_pts + k * 16);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_pts, points, np * 64, hipMemcpyHostToDevice, c->stream), "H2D pts")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_sc, scalars, np * 32, hipMemcpyHostToDevice, c->stream), "H2D sc")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_ptr, ptrs.data(), np * 8, hipMemcpyHostToDevice, c->stream), "H2D ptr")))
    return rc;
  EcMsmArgs a{d_ptr, d_sc, terms, d_out, count, d_scr, c->prio};
  c->mark("ec", true);
  rc = c->hip_check(launch_ec_msm(a, c->stream), "ec_msm");
  c->mark("ec", false);
  if (rc) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(out, d_out, (size_t)count * 64, hipMemcpyDeviceToHost, c->stream), "D2H")))
    return rc;
  return c->sync();
}

}  // extern "C"

namespace {
const uint32_t SECP_Q[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                            0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
const uint32_t SECP_G[16] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu, 0xCE870B07u, 0x55A06295u,
                             0xF9DCBBACu, 0x79BE667Eu, 0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                             0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};

// curv VerifiableSS::map_share_to_new_params: the Lagrange weight at 0 of point
// x_j = old_index[j] over the set, prod_{x_k != x_j} x_k / (x_k - x_j) mod q
// (entries equal to x_j are skipped, as the reference skips index == j)
hbn::Limbs lagrange(const uint32_t* x, uint32_t cnt, uint32_t j, const hbn::Limbs& Q) {
  hbn::Limbs num{1}, den{1};
  for (uint32_t k = 0; k < cnt; ++k) {
    if (x[k] == x[j]) continue;
    num = hbn::mulmod(num, hbn::Limbs{x[k]}, Q);
    const hbn::Limbs d = x[k] > x[j] ? hbn::Limbs{x[k] - x[j]} : hbn::sub(Q, hbn::Limbs{x[j] - x[k]});
    den = hbn::mulmod(den, d, Q);
  }
  hbn::Limbs inv;
  if (!hbn::modinv(den, Q, &inv)) return hbn::Limbs{};   // unreachable for indices < q
  return hbn::mulmod(num, inv, Q);
}

// secp256k1 group of the host-side y = G * share (OpenSSL; one scalar
// multiplication per job, off the GPU's latency-bound MSM path)
const EC_GROUP* secp_group() {
  static const EC_GROUP* g = EC_GROUP_new_by_curve_name(NID_secp256k1);
  return g;
}

// out16 = G * k (affine x | y as 8 little-endian u32 limbs each; (0, 0) = infinity)
bool g_mul(const hbn::Limbs& k, uint32_t* out16) {
  std::memset(out16, 0, 64);
  uint8_t kb[32] = {0};
  for (size_t i = 0; i < k.size() && i < 8; ++i)
    for (int b = 0; b < 4; ++b) kb[4 * i + b] = (uint8_t)(k[i] >> (8 * b));
  BN_CTX* bc = BN_CTX_new();
  BIGNUM* bk = BN_lebin2bn(kb, 32, nullptr);
  BIGNUM *x = BN_new(), *y = BN_new();
  EC_POINT* R = EC_POINT_new(secp_group());
  bool ok = bc && bk && x && y && R;
  if (ok) BN_set_flags(bk, BN_FLG_CONSTTIME);
  ok = ok && EC_POINT_mul(secp_group(), R, bk, nullptr, nullptr, bc) == 1;
  if (ok && !EC_POINT_is_at_infinity(secp_group(), R)) {
    ok = EC_POINT_get_affine_coordinates(secp_group(), R, x, y, bc) == 1;
    uint8_t xb[32], yb[32];
    ok = ok && BN_bn2lebinpad(x, xb, 32) == 32 && BN_bn2lebinpad(y, yb, 32) == 32;
    if (ok) {
      std::memcpy(out16, xb, 32);
      std::memcpy(out16 + 8, yb, 32);
    }
  }
  EC_POINT_free(R);
  BN_free(x);
  BN_free(y);
  BN_clear_free(bk);
  BN_CTX_free(bc);
  OPENSSL_cleanse(kb, sizeof kb);
  return ok;
}

// a^-1 mod m for a secret odd m (OpenSSL, constant-time flag); false if not a unit
bool inv_secret(const hbn::Limbs& a, const hbn::Limbs& m, hbn::Limbs* out) {
  auto to_bn = [](const hbn::Limbs& v) {
    std::vector<uint8_t> b(4 * std::max<size_t>(v.size(), 1), 0);
    for (size_t i = 0; i < v.size(); ++i)
      for (int k = 0; k < 4; ++k) b[4 * i + k] = (uint8_t)(v[i] >> (8 * k));
    BIGNUM* r = BN_lebin2bn(b.data(), (int)b.size(), nullptr);
    OPENSSL_cleanse(b.data(), b.size());
    return r;
  };
  BN_CTX* bc = BN_CTX_new();
  BIGNUM *ba = to_bn(a), *bm = to_bn(m), *br = BN_new();
  bool ok = bc && ba && bm && br;
  if (ok) {
    BN_set_flags(ba, BN_FLG_CONSTTIME);
    BN_set_flags(bm, BN_FLG_CONSTTIME);
    ok = BN_mod_inverse(br, ba, bm, bc) != nullptr;
  }
  if (ok) {
    const int nb = BN_num_bytes(br);
    std::vector<uint8_t> b((size_t)std::max(nb, 1) + 3, 0);
    BN_bn2lebinpad(br, b.data(), (int)b.size());
    hbn::Limbs r((b.size() + 3) / 4, 0u);
    for (size_t i = 0; i < b.size(); ++i) r[i / 4] |= (uint32_t)b[i] << (8 * (i % 4));
    hbn::trim(r);
    *out = r;
    OPENSSL_cleanse(b.data(), b.size());
  }
  BN_clear_free(ba);
  BN_clear_free(bm);
  BN_clear_free(br);
  BN_CTX_free(bc);
  return ok;
}

// grow-only pinned host buffer (the async D2H targets of a launched recovery)
struct Pinned {
  void* p = nullptr;
  size_t bytes = 0;
  uint32_t* get(size_t want) {
    if (want > bytes) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      bytes = 0;
      if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess) return nullptr;
      bytes = want;
    }
    return reinterpret_cast<uint32_t*>(p);
  }
  ~Pinned() {
    if (p) (void)hipHostFree(p);
  }
};
}  // namespace

namespace fsdkr {

// A launched share recovery (fsdkr_collect_recover_launch): the GPU work (CRT
// decryption exponentiations, the pk_vec MSM) is enqueued on the recovery
// stream; finish() waits for it and does the O(1) host arithmetic.  Every input
// is copied at launch, so the caller's arrays may go away in between.
struct RecoverPending {
  struct Job {
    uint32_t nl = 0, T = 0, t_key = 0, t_vss = 0, n_new = 0, tp = 0;
    std::vector<hbn::Limbs> li;
    hbn::Limbs P, Q, qinv, pinv;
    bool dec_ok = false;
    bool no_dec = false;     // FSDKR_RECOVER_NO_DECRYPT: pk_vec rows only
    uint32_t width = 0;      // decryption batch (index into widths)
    size_t dec_at = 0;       // its first decryption in that batch
    size_t row = ~(size_t)0; // its first pk_vec row of the MSM
  };
  struct Width {
    uint32_t nl = 0, total = 0, keys = 0, exp_bits = 0;
    std::vector<uint32_t> base, ex, idx, mods;
    std::vector<uint8_t> desc;
    uint32_t* out = nullptr;   // pinned, dec_out[class]
  };
  std::vector<Job> jobs;
  std::vector<Width> widths;
  uint32_t rows = 0, terms = 1;
  std::vector<uint32_t> pts, scs;
  std::vector<uint64_t> ptrs;
  // pinned D2H targets, kept across calls (allocating or freeing pinned memory
  // synchronises the device, which would wait for a running pipeline)
  Pinned dec_out[4], msm_out;
  hipEvent_t done = nullptr;
  bool in_flight = false;

  ~RecoverPending() {
    if (done) (void)hipEventDestroy(done);
  }
  int launch(Ctx* c, const fsdkr_recover_job* in, uint32_t count);
  int finish(Ctx* c, fsdkr_recovered* out);
};

RecoverPending* recover_state(Ctx* c) {
  if (!c->recover) c->recover = new RecoverPending();
  return reinterpret_cast<RecoverPending*>(c->recover);
}

void free_recover(Ctx* c) {
  delete reinterpret_cast<RecoverPending*>(c->recover);
  c->recover = nullptr;
}

int RecoverPending::launch(Ctx* c, const fsdkr_recover_job* in, uint32_t count) {
  const hbn::Limbs Qs = hbn::from(SECP_Q, 8);
  jobs.assign(count, Job{});
  widths.clear();
  rows = 0;
  terms = 1;
  pts.clear();
  scs.clear();
  // per job: Lagrange weights, the key's CRT constants (a degenerate key panics in
  // Paillier::decrypt: p or q even or 1, p == q, p^2 / q^2 / N wider than the class)
  parallel_for_host(count, 1, [&](size_t b0, size_t b1) {
    for (size_t j = b0; j < b1; ++j) {
      const fsdkr_recover_job& J = in[j];
      Job& X = jobs[j];
      X.nl = J.nl;
      X.T = J.t_vss + 1;
      X.t_key = J.t_key;
      X.t_vss = J.t_vss;
      X.n_new = J.n_new;
      X.tp = std::min(J.t_key, J.t_vss) + 1;
      X.li.resize(X.T);
      for (uint32_t k = 0; k < X.T; ++k) X.li[k] = lagrange(J.old_index, X.T, k, Qs);
      X.no_dec = (J.flags & FSDKR_RECOVER_NO_DECRYPT) != 0;
      if (X.no_dec) {   // the Lagrange weights of the pk_vec rows; the key is not read
        X.dec_ok = true;
        continue;
      }
      X.P = hbn::from(J.p, J.nl);
      X.Q = hbn::from(J.q, J.nl);
      const hbn::Limbs PP = hbn::mul(X.P, X.P), QQ = hbn::mul(X.Q, X.Q), N = hbn::mul(X.P, X.Q);
      X.dec_ok = !hbn::is_even(X.P) && !hbn::is_even(X.Q) && hbn::bitlen(PP) <= 32 * J.nl &&
                 hbn::bitlen(QQ) <= 32 * J.nl && hbn::bitlen(N) <= 32 * J.nl && !hbn::is_one(X.P) &&
                 !hbn::is_one(X.Q) && inv_secret(hbn::mod(X.Q, X.P), X.P, &X.qinv) &&
                 inv_secret(hbn::mod(X.P, X.Q), X.Q, &X.pinv);
    }
  });
  // decryption batches, one per key width: (c mod p^2)^(p-1), (c mod q^2)^(q-1)
  for (uint32_t wc = 0; wc < 4; ++wc) {
    const uint32_t nl = 64u + 32u * wc + (wc == 3 ? 32u : 0u);   // 64, 96, 128, 192
    Width W;
    W.nl = nl;
    std::vector<uint32_t> owners;
    for (uint32_t j = 0; j < count; ++j)
      if (jobs[j].nl == nl && jobs[j].dec_ok && !jobs[j].no_dec) {
        jobs[j].width = (uint32_t)widths.size();
        jobs[j].dec_at = W.total;
        W.total += jobs[j].T;
        owners.push_back(j);
      }
    if (!W.total) continue;
    W.keys = (uint32_t)owners.size();
    W.base.assign((size_t)2 * W.total * nl, 0u);
    W.ex.assign((size_t)2 * W.total * nl, 0u);
    W.idx.resize(2 * (size_t)W.total);
    W.mods.assign((size_t)2 * W.keys * nl, 0u);
    parallel_for_host(owners.size(), 1, [&](size_t b0, size_t b1) {
      for (size_t o = b0; o < b1; ++o) {
        const uint32_t j = owners[o];
        const Job& X = jobs[j];
        const hbn::Limbs PP = hbn::mul(X.P, X.P), QQ = hbn::mul(X.Q, X.Q);
        const hbn::Limbs pm1 = hbn::sub(X.P, hbn::Limbs{1}), qm1 = hbn::sub(X.Q, hbn::Limbs{1});
        hbn::store(PP, W.mods.data() + (2 * o) * nl, nl);
        hbn::store(QQ, W.mods.data() + (2 * o + 1) * nl, nl);
        for (uint32_t k = 0; k < X.T; ++k) {
          const size_t i = X.dec_at + k;
          const hbn::Limbs ck = hbn::from(in[j].cts + (size_t)k * 2 * nl, 2 * nl);
          hbn::store(hbn::mod(ck, PP), W.base.data() + (2 * i) * nl, nl);
          hbn::store(hbn::mod(ck, QQ), W.base.data() + (2 * i + 1) * nl, nl);
          hbn::store(pm1, W.ex.data() + (2 * i) * nl, nl);
          hbn::store(qm1, W.ex.data() + (2 * i + 1) * nl, nl);
          W.idx[2 * i] = (uint32_t)(2 * o);
          W.idx[2 * i + 1] = (uint32_t)(2 * o + 1);
        }
      }
    });
    for (uint32_t j : owners) W.exp_bits = std::max({W.exp_bits, hbn::bitlen(jobs[j].P), hbn::bitlen(jobs[j].Q)});
    widths.push_back(std::move(W));
  }
  // pk_vec rows: new party i's sum over k < tp of li[k] * points_committed_vec[i] of message k
  for (uint32_t j = 0; j < count; ++j)
    if (jobs[j].dec_ok && jobs[j].n_new) terms = std::max(terms, jobs[j].tp);
  for (uint32_t j = 0; j < count; ++j) {
    Job& X = jobs[j];
    if (!X.dec_ok || !X.n_new) continue;
    X.row = rows;
    for (uint32_t i = 0; i < X.n_new; ++i)
      for (uint32_t k = 0; k < terms; ++k) {
        const size_t at = pts.size();
        pts.resize(at + 16, 0u);
        scs.resize(scs.size() + 8, 0u);
        if (k < X.tp) {
          std::memcpy(pts.data() + at, in[j].points + ((size_t)i * X.tp + k) * 16, 64);
          hbn::store(X.li[k], scs.data() + scs.size() - 8, 8);
        }
      }
    rows += X.n_new;
  }
  // enqueue: recovery stream, issue priority 3 (few waves beside a launched pipeline)
  StreamScope scope(c, c->aux_stream());
  PrioScope prio(c, 3);
  int rc;
  for (Width& W : widths) {
    const uint32_t nl = W.nl, n = 2 * W.total, nm = 2 * W.keys;
    const std::string tag = "rc" + std::to_string(nl);
    const size_t nb = (size_t)n * nl * 4;
    uint8_t* d = (uint8_t*)c->buf((tag + "_io").c_str(), 3 * nb + (size_t)nm * nl * 4 + 1024);
    const uint32_t wc = nl == 64 ? 0 : nl == 96 ? 1 : nl == 128 ? 2 : 3;
    uint32_t* h_out = W.out = dec_out[wc].get(nb);
    if (!d || !h_out) {
      c->fail("fsdkr_collect_recover: allocation failed");
      return FSDKR_E_OOM;
    }
    uint32_t *d_base = (uint32_t*)d, *d_ex = d_base + (size_t)n * nl, *d_out = d_ex + (size_t)n * nl;
    uint32_t* d_mods = d_out + (size_t)n * nl;
    if ((rc = c->hip_check(hipMemcpyAsync(d_base, W.base.data(), nb, hipMemcpyHostToDevice, c->stream), "H2D rc")) ||
        (rc = c->hip_check(hipMemcpyAsync(d_ex, W.ex.data(), nb, hipMemcpyHostToDevice, c->stream), "H2D rc")) ||
        (rc = c->hip_check(hipMemcpyAsync(d_mods, W.mods.data(), (size_t)nm * nl * 4, hipMemcpyHostToDevice, c->stream),
                           "H2D rc")))
      return rc;
    uint32_t* consts = nullptr;
    if ((rc = setup_moduli(c, nl, d_mods, nm, &consts, tag.c_str()))) return rc;
    ModexpJob job;
    job.k32 = nl;
    for (uint32_t i = 0; i < n; ++i)
      job.add((uint64_t)(uintptr_t)(d_base + (size_t)i * nl), nl, (uint64_t)(uintptr_t)(d_ex + (size_t)i * nl), nl,
              W.exp_bits, W.idx[i]);
    W.desc.clear();
    job.pack(W.desc);
    uint8_t* d_desc = (uint8_t*)c->buf((tag + "_desc").c_str(), W.desc.size());
    if (!d_desc) return FSDKR_E_OOM;
    if ((rc = c->hip_check(hipMemcpyAsync(d_desc, W.desc.data(), W.desc.size(), hipMemcpyHostToDevice, c->stream),
                           "H2D rc desc")))
      return rc;
    {
      CtScope ct(c);   // secret exponents p - 1, q - 1: regular-access modexp
      if ((rc = launch_modexp_desc(c, nl, n, W.exp_bits, d_desc, consts, d_out, c->stream, (tag + "_tab").c_str(),
                                   c->prio, 0)))
        return rc;
    }
    if ((rc = c->hip_check(hipMemcpyAsync(h_out, d_out, nb, hipMemcpyDeviceToHost, c->stream), "D2H rc"))) return rc;
  }
  if (rows) {
    const size_t np = (size_t)rows * terms;
    uint8_t* d = (uint8_t*)c->buf("rc_msm", np * 16 * 4 + np * 8 * 4 + np * 8 + (size_t)rows * 16 * 4 + np * 96 + 1024);
    uint32_t* h_out = msm_out.get((size_t)rows * 64);
    if (!d || !h_out) return FSDKR_E_OOM;
    uint32_t* d_pts = (uint32_t*)d;
    uint32_t* d_sc = d_pts + np * 16;
    uint64_t* d_ptr = (uint64_t*)(d_sc + np * 8);
    uint32_t* d_o = (uint32_t*)(d_ptr + np);
    uint32_t* d_scr = d_o + (size_t)rows * 16;
    ptrs.resize(np);
    for (size_t k = 0; k < np; ++k) ptrs[k] = (uint64_t)(uintptr_t)(d_pts + k * 16);
    if ((rc = c->hip_check(hipMemcpyAsync(d_pts, pts.data(), np * 64, hipMemcpyHostToDevice, c->stream), "H2D pts")) ||
        (rc = c->hip_check(hipMemcpyAsync(d_sc, scs.data(), np * 32, hipMemcpyHostToDevice, c->stream), "H2D sc")) ||
        (rc = c->hip_check(hipMemcpyAsync(d_ptr, ptrs.data(), np * 8, hipMemcpyHostToDevice, c->stream), "H2D ptr")))
      return rc;
    EcMsmArgs a{d_ptr, d_sc, terms, d_o, rows, d_scr, c->prio};
    c->mark("ec", true);
    rc = c->hip_check(launch_ec_msm(a, c->stream), "ec_msm");
    c->mark("ec", false);
    if (rc) return rc;
    if ((rc = c->hip_check(hipMemcpyAsync(h_out, d_o, (size_t)rows * 64, hipMemcpyDeviceToHost, c->stream), "D2H msm")))
      return rc;
  }
  if (!done && (rc = c->hip_check(hipEventCreateWithFlags(&done, hipEventDisableTiming), "event"))) return rc;
  if ((rc = c->hip_check(hipEventRecord(done, c->stream), "event record"))) return rc;
  in_flight = true;
  return FSDKR_OK;
}

int RecoverPending::finish(Ctx* c, fsdkr_recovered* out) {
  in_flight = false;
  int rc = c->hip_check(hipEventSynchronize(done), "recovery wait");
  if (rc) return rc;
  const hbn::Limbs Qs = hbn::from(SECP_Q, 8), one{1};
  std::atomic<bool> ec_ok{true};
  parallel_for_host(jobs.size(), 1, [&](size_t b0, size_t b1) {
    for (size_t j = b0; j < b1; ++j) {
      const Job& X = jobs[j];
      fsdkr_recovered& O = out[j];
      std::memset(O.share, 0, sizeof O.share);
      std::memset(O.y, 0, sizeof O.y);
      if (!X.dec_ok) {
        O.status = FSDKR_RECOVER_PANIC_DECRYPT;
        continue;
      }
      O.status = X.t_key > X.t_vss ? FSDKR_RECOVER_PANIC_LI : FSDKR_RECOVER_OK;
      if (X.n_new) {
        const uint32_t* r = reinterpret_cast<const uint32_t*>(msm_out.p) + X.row * 16;
        std::memcpy(O.pk_vec, r, (size_t)X.n_new * 64);
      }
      if (X.no_dec) continue;
      const uint32_t nl = X.nl;
      const uint32_t* h = widths[X.width].out;
      // kzen-paillier CRT decryption with g = N + 1: h_p = L_p(g^(p-1) mod p^2)^-1 = p - q^-1 mod p.
      // The reference decrypts C = Enc(0) prod_k c_k^l_k once; per CRT half that is
      // sum_k l_k L_p(c_k^(p-1)) h_p mod p (L_p is a homomorphism on units), and 0
      // when p divides some c_k (then p | C, C^(p-1) = 0 mod p^2 and L_p(0) =
      // (0 - 1) / p truncates to 0).  Units give (sum_k l_k m_k) mod N exactly.
      const hbn::Limbs hp = hbn::sub(X.P, X.qinv), hq = hbn::sub(X.Q, X.pinv);
      hbn::Limbs acc_p, acc_q;
      bool zero_p = false, zero_q = false;
      for (uint32_t k = 0; k < X.T; ++k) {
        const size_t i = X.dec_at + k;
        const hbn::Limbs up = hbn::from(h + (2 * i) * nl, nl), uq = hbn::from(h + (2 * i + 1) * nl, nl);
        zero_p = zero_p || up.empty();
        zero_q = zero_q || uq.empty();
        const hbn::Limbs mp = hbn::mulmod(hbn::div_exact(hbn::sub(up.empty() ? one : up, one), X.P), hp, X.P);
        const hbn::Limbs mq = hbn::mulmod(hbn::div_exact(hbn::sub(uq.empty() ? one : uq, one), X.Q), hq, X.Q);
        acc_p = hbn::add(acc_p, hbn::mul(X.li[k], mp));
        acc_q = hbn::add(acc_q, hbn::mul(X.li[k], mq));
      }
      const hbn::Limbs mp = zero_p ? hbn::Limbs{} : hbn::mod(acc_p, X.P);
      const hbn::Limbs mq = zero_q ? hbn::Limbs{} : hbn::mod(acc_q, X.Q);
      // m = mq + q * ((mp - mq) q^-1 mod p)
      const hbn::Limbs mqp = hbn::mod(mq, X.P);
      const hbn::Limbs d = hbn::cmp(mp, mqp) >= 0 ? hbn::sub(mp, mqp) : hbn::sub(hbn::add(mp, X.P), mqp);
      const hbn::Limbs m = hbn::add(mq, hbn::mul(X.Q, hbn::mulmod(d, X.qinv, X.P)));
      // new share = the decrypted sum (in [0, N)) mod q
      const hbn::Limbs share = hbn::mod(m, Qs);
      hbn::store(share, O.share, 8);
      if (!g_mul(share, O.y)) ec_ok = false;
    }
  });
  if (!ec_ok) {
    c->fail("fsdkr_collect_recover: OpenSSL secp256k1 scalar multiplication failed");
    return FSDKR_E_ARG;
  }
  return FSDKR_OK;
}

}  // namespace fsdkr

extern "C" {

int fsdkr_collect_recover_launch(fsdkr_ctx* ctx, const fsdkr_recover_job* jobs, uint32_t count) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count && !jobs) {
    c->fail("fsdkr_collect_recover: null jobs");
    return FSDKR_E_ARG;
  }
  for (uint32_t j = 0; j < count; ++j) {
    const fsdkr_recover_job& J = jobs[j];
    const bool dec = !(J.flags & FSDKR_RECOVER_NO_DECRYPT);   // a rows-only job reads no key or ciphertext
    if (!shape_digits(J.nl) || !J.old_index || (dec && (!J.cts || !J.p || !J.q)) || (J.n_new && !J.points)) {
      c->fail("fsdkr_collect_recover: job %u: bad shape or null array (nl=%u)", j, J.nl);
      return FSDKR_E_ARG;
    }
  }
  RecoverPending* R = recover_state(c);
  if (R->in_flight) {
    c->fail("fsdkr_collect_recover_launch: a recovery is in flight (call fsdkr_collect_recover_finish)");
    return FSDKR_E_ARG;
  }
  return R->launch(c, jobs, count);
}

int fsdkr_collect_recover_finish(fsdkr_ctx* ctx, fsdkr_recovered* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  RecoverPending* R = reinterpret_cast<RecoverPending*>(c->recover);
  if (!R || !R->in_flight) {
    c->fail("fsdkr_collect_recover_finish: no recovery launched");
    return FSDKR_E_ARG;
  }
  if (!out && !R->jobs.empty()) {
    c->fail("fsdkr_collect_recover_finish: null out");
    return FSDKR_E_ARG;
  }
  for (size_t j = 0; j < R->jobs.size(); ++j)
    if (R->jobs[j].n_new && !out[j].pk_vec) {
      c->fail("fsdkr_collect_recover_finish: job %zu: null pk_vec", j);
      return FSDKR_E_ARG;
    }
  return R->finish(c, out);
}

int fsdkr_collect_recover(fsdkr_ctx* ctx, const fsdkr_recover_job* jobs, uint32_t count, fsdkr_recovered* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!jobs || !out) {
    c->fail("fsdkr_collect_recover: null jobs / out");
    return FSDKR_E_ARG;
  }
  int rc = fsdkr_collect_recover_launch(ctx, jobs, count);
  return rc ? rc : fsdkr_collect_recover_finish(ctx, out);
}

}  // extern "C"
