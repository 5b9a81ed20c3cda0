// Share recovery building blocks of collect() (refresh_message.rs:367-373,
// 439-464): Paillier decryption of the homomorphically summed share and the
// secp256k1 multi-scalar multiplications that rebuild pk_vec and y.  The
// exponentiation and EC work run on the GPU; the O(1) L-function / mu
// arithmetic of kzen-paillier decrypt runs on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
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
  std::vector<std::thread> th;
  for (size_t k = 1; k < chunks; ++k) th.emplace_back([&, k] { f(n * k / chunks, n * (k + 1) / chunks); });
  f((size_t)0, n / chunks);
  for (auto& t : th) t.join();
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
  // device image: ns | NNs | m | r | one | outputs
  const size_t b_ns = 0, b_nns = b_ns + (size_t)n_keys * nl * 4, b_m = b_nns + NNs.size() * 4;
  const size_t b_r = b_m + (size_t)count * ml * 4, b_one = b_r + (size_t)count * nl * 4;
  const size_t b_gm = b_one + (size_t)nn * 4, b_rn = b_gm + (size_t)count * nn * 4;
  const size_t b_out = b_rn + (size_t)count * nn * 4, b_desc = b_out + (size_t)count * nn * 4;
  const size_t total = b_desc + (size_t)count * (16 + 32 + sizeof(Prod3Operand) + 4) + 8 * 256 + 4096;
  uint8_t* d = (uint8_t*)cx->buf("enc", total);
  if (!d) return FSDKR_E_OOM;
  std::vector<uint8_t> img(b_desc, 0);
  memcpy(img.data() + b_ns, ns, (size_t)n_keys * nl * 4);
  memcpy(img.data() + b_nns, NNs.data(), NNs.size() * 4);
  memcpy(img.data() + b_m, m, (size_t)count * ml * 4);
  memcpy(img.data() + b_r, r, (size_t)count * nl * 4);
  ((uint32_t*)(img.data() + b_one))[0] = 1;
  auto A = [&](size_t off) { return (uint64_t)(uintptr_t)(d + off); };
  // binom: gm = 1 + m*N  (m < N for a share; reduced mod N^2 by prod3 anyway)
  std::vector<uint64_t> s_ptr(count), n_ptr(count);
  ModexpJob job;
  job.k32 = nn;
  std::vector<Prod3Operand> ops(count);
  std::vector<uint32_t> midx(count);
  for (uint32_t k = 0; k < count; ++k) {
    s_ptr[k] = A(b_m + (size_t)k * ml * 4);
    n_ptr[k] = A(b_ns + (size_t)n_idx[k] * nl * 4);
    job.add(A(b_r + (size_t)k * nl * 4), nl, A(b_ns + (size_t)n_idx[k] * nl * 4), nl, 32 * nl, n_idx[k]);
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
  if ((rc = launch_modexp_desc(cx, nn, count, 32 * nl, d + o_job, consts, (uint32_t*)(d + b_rn)))) return rc;
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
}  // namespace

extern "C" {

int fsdkr_collect_recover(fsdkr_ctx* ctx, const fsdkr_recover_job* jobs, uint32_t count, fsdkr_recovered* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!jobs || !out) {
    c->fail("fsdkr_collect_recover: null jobs / out");
    return FSDKR_E_ARG;
  }
  for (uint32_t j = 0; j < count; ++j) {
    const fsdkr_recover_job& J = jobs[j];
    if (!shape_digits(J.nl) || !J.old_index || !J.cts || !J.p || !J.q || (J.n_new && (!J.points || !out[j].pk_vec))) {
      c->fail("fsdkr_collect_recover: job %u: bad shape or null array (nl=%u)", j, J.nl);
      return FSDKR_E_ARG;
    }
  }
  const hbn::Limbs Q = hbn::from(SECP_Q, 8);
  // Lagrange weights (host; t_vss+1 small integers per job)
  std::vector<std::vector<hbn::Limbs>> li(count);
  for (uint32_t j = 0; j < count; ++j) {
    const uint32_t T = jobs[j].t_vss + 1;
    li[j].resize(T);
    for (uint32_t k = 0; k < T; ++k) li[j][k] = lagrange(jobs[j].old_index, T, k, Q);
    out[j].status = FSDKR_RECOVER_OK;
  }
  // decryptions: one batched call per key width; a width whose batch the
  // decryption refuses (a degenerate key) is retried job by job
  std::vector<std::vector<uint32_t>> plain(count);
  for (uint32_t nl : {64u, 96u, 128u, 192u}) {
    std::vector<uint32_t> cts, kidx, ps, qs, owners;
    for (uint32_t j = 0; j < count; ++j) {
      const fsdkr_recover_job& J = jobs[j];
      if (J.nl != nl) continue;
      const uint32_t T = J.t_vss + 1;
      cts.insert(cts.end(), J.cts, J.cts + (size_t)T * 2 * nl);
      for (uint32_t k = 0; k < T; ++k) kidx.push_back((uint32_t)owners.size());
      ps.insert(ps.end(), J.p, J.p + nl);
      qs.insert(qs.end(), J.q, J.q + nl);
      owners.push_back(j);
    }
    if (owners.empty()) continue;
    const uint32_t total = (uint32_t)kidx.size();
    std::vector<uint32_t> m((size_t)total * nl);
    int rc = fsdkr_paillier_decrypt_multi(ctx, nl, total, cts.data(), kidx.data(), ps.data(), qs.data(),
                                          (uint32_t)owners.size(), m.data());
    if (rc == FSDKR_OK) {
      size_t at = 0;
      for (uint32_t j : owners) {
        const size_t T = jobs[j].t_vss + 1;
        plain[j].assign(m.begin() + at * nl, m.begin() + (at + T) * nl);
        at += T;
      }
      continue;
    }
    if (rc != FSDKR_E_ARG) return rc;
    for (uint32_t j : owners) {
      const fsdkr_recover_job& J = jobs[j];
      const uint32_t T = J.t_vss + 1;
      plain[j].resize((size_t)T * nl);
      if (fsdkr_paillier_decrypt(ctx, nl, T, J.cts, J.p, J.q, plain[j].data()) != FSDKR_OK) {
        out[j].status = FSDKR_RECOVER_PANIC_DECRYPT;
        plain[j].clear();
      }
    }
  }
  // new share = (sum_k l_k m_k mod N) mod q, then one MSM launch for every y and pk_vec row
  uint32_t terms = 1;
  for (uint32_t j = 0; j < count; ++j)
    terms = std::max(terms, std::min(jobs[j].t_key, jobs[j].t_vss) + 1);
  std::vector<uint32_t> pts, scs;
  std::vector<uint32_t> row_of(count, ~0u);
  auto add_row = [&](const uint32_t* p16, size_t n_pts, const std::vector<hbn::Limbs>& sc) {
    for (size_t k = 0; k < terms; ++k) {
      const size_t at = pts.size();
      pts.resize(at + 16, 0u);
      scs.resize(scs.size() + 8, 0u);
      if (k < n_pts) {
        memcpy(pts.data() + at, p16 + k * 16, 64);
        hbn::store(sc[k], scs.data() + scs.size() - 8, 8);
      }
    }
  };
  uint32_t rows = 0;
  for (uint32_t j = 0; j < count; ++j) {
    const fsdkr_recover_job& J = jobs[j];
    if (out[j].status == FSDKR_RECOVER_PANIC_DECRYPT) continue;
    const uint32_t T = J.t_vss + 1, nl = J.nl;
    const hbn::Limbs N = hbn::mul(hbn::from(J.p, nl), hbn::from(J.q, nl));
    hbn::Limbs acc;
    for (uint32_t k = 0; k < T; ++k) acc = hbn::add(acc, hbn::mul(li[j][k], hbn::from(plain[j].data() + (size_t)k * nl, nl)));
    const hbn::Limbs share = hbn::mod(hbn::mod(acc, N), Q);
    memset(out[j].share, 0, sizeof out[j].share);
    hbn::store(share, out[j].share, 8);
    row_of[j] = rows;
    add_row(SECP_G, 1, std::vector<hbn::Limbs>{share});
    const uint32_t tp = std::min(J.t_key, J.t_vss) + 1;
    for (uint32_t i = 0; i < J.n_new; ++i) add_row(J.points + (size_t)i * tp * 16, tp, li[j]);
    rows += 1 + J.n_new;
    if (J.t_key > J.t_vss) out[j].status = FSDKR_RECOVER_PANIC_LI;
  }
  if (!rows) return FSDKR_OK;
  std::vector<uint32_t> res((size_t)rows * 16);
  int rc = fsdkr_ec_msm(ctx, rows, terms, pts.data(), scs.data(), res.data());
  if (rc) return rc;
  for (uint32_t j = 0; j < count; ++j) {
    if (row_of[j] == ~0u) continue;
    const uint32_t* r = res.data() + (size_t)row_of[j] * 16;
    memcpy(out[j].y, r, 64);
    if (jobs[j].n_new) memcpy(out[j].pk_vec, r + 16, (size_t)jobs[j].n_new * 64);
  }
  return FSDKR_OK;
}

}  // extern "C"
