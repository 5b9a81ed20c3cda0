// Stand-alone verification entry points of the C ABI (include/fsdkr/fsdkr.h):
//   fsdkr_feldman_check          validate_collect's Feldman loop (refresh_message.rs:177-188)
//   fsdkr_ring_pedersen_verify   RingPedersenProof::verify (ring_pedersen_proof.rs:126-157)
// JoinMessage::collect (add_party_message.rs:136-175) needs exactly these two
// checks and none of the pair proofs, so it calls them instead of the whole
// fsdkr_verify_collect pipeline.  Both run on the context stream; the ring-
// Pedersen challenge hash overlaps the T^Z exponentiations (the challenge bits
// are only needed by the final equality check).
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "ctx.hpp"
#include "fbjob.hpp"
#include "fsdkr/fsdkr.h"
#include "kernels.h"
#include "verify.h"

using namespace fsdkr;

namespace {

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

uint32_t bit_len(const uint32_t* x, uint32_t limbs) {
  for (int k = (int)limbs - 1; k >= 0; --k)
    if (x[k]) return 32u * (uint32_t)k + 32u - (uint32_t)__builtin_clz(x[k]);
  return 0;
}

}  // namespace

extern "C" {

int fsdkr_feldman_check(fsdkr_ctx* ctx, uint32_t n_msgs, uint32_t n, uint32_t t, const uint32_t* vss,
                        const uint32_t* commit, uint8_t* verdict) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  const size_t P = (size_t)n_msgs * n;
  if (P == 0) return FSDKR_OK;
  if (!vss || !commit || !verdict) {
    c->fail("fsdkr_feldman_check: null pointer");
    return FSDKR_E_ARG;
  }
  const size_t vb = (size_t)n_msgs * (t + 1) * 16 * 4, cb = P * 16 * 4;
  uint8_t* d = (uint8_t*)c->buf("fel_io", al256(vb) + al256(cb) + P);
  if (!d) {
    c->fail("fsdkr_feldman_check: device allocation failed");
    return FSDKR_E_OOM;
  }
  uint32_t* d_vss = (uint32_t*)d;
  uint32_t* d_com = (uint32_t*)(d + al256(vb));
  uint8_t* d_out = d + al256(vb) + al256(cb);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_vss, vss, vb, hipMemcpyHostToDevice, c->stream), "H2D vss")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_com, commit, cb, hipMemcpyHostToDevice, c->stream), "H2D commit")))
    return rc;
  FeldmanArgs f{d_vss, d_com, n, t, d_out, (uint32_t)P};
  c->mark("ec", true);
  rc = c->hip_check(launch_feldman(f, c->stream), "feldman");
  c->mark("ec", false);
  if (rc) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(verdict, d_out, P, hipMemcpyDeviceToHost, c->stream), "D2H feldman")))
    return rc;
  return c->sync();
}

int fsdkr_ring_pedersen_verify(fsdkr_ctx* ctx, uint32_t nl, uint32_t count, uint32_t m_security, uint32_t zl,
                               const uint32_t* S, const uint32_t* T, const uint32_t* N, const uint32_t* A,
                               const uint32_t* Z, uint8_t* verdict) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  const uint32_t M = m_security;
  if (!S || !T || !N || !A || !Z || !verdict || M == 0 || zl == 0) {
    c->fail("fsdkr_ring_pedersen_verify: bad argument");
    return FSDKR_E_ARG;
  }
  if (nl != 64 && nl != 96) {
    c->fail("fsdkr_ring_pedersen_verify: unsupported modulus width %u limbs", nl);
    return FSDKR_E_UNSUPPORTED;
  }
  for (uint32_t m = 0; m < count; ++m)
    if (!(N[(size_t)m * nl] & 1u)) {
      c->fail("fsdkr_ring_pedersen_verify: proof %u has an even modulus (unsupported)", m);
      return FSDKR_E_UNSUPPORTED;
    }
  const size_t MW = (M + 31) / 32;           // challenge-bit words per proof
  const size_t I = (size_t)count * M;        // T^Z instances
  const size_t bN = (size_t)count * nl * 4, bA = I * nl * 4, bZ = I * zl * 4;
  // device image: N | S | T | A | Z | one | bits | panic | TZ | eq | eq ops | eq mod idx
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = al256(off + (bytes ? bytes : 1)); return o; };
  const size_t oN = take(bN), oS = take(bN), oT = take(bN), oA = take(bA), oZ = take(bZ), oOne = take(nl * 4);
  const size_t oBits = take((size_t)count * MW * 4), oPanic = take((size_t)count * 4), oTZ = take(bA);
  const size_t oEq = take(I * 4), oOps = take(I * sizeof(EqOperand)), oMod = take(I * 4);
  uint8_t* d = (uint8_t*)c->buf("rp_io", off);
  if (!d) {
    c->fail("fsdkr_ring_pedersen_verify: device allocation failed");
    return FSDKR_E_OOM;
  }
  auto DA = [&](size_t o) { return (uint64_t)(uintptr_t)(d + o); };
  std::vector<uint32_t> one(nl, 0u);
  one[0] = 1;
  std::vector<EqOperand> ops(I);
  std::vector<uint32_t> mod_idx(I);
  // T^Z_k mod N (ring_pedersen_proof.rs:144): T is shared by the M checks of a proof -> fixed-base job
  FbJob job;
  job.k32 = nl;
  uint32_t zmax = 1;
  for (size_t k = 0; k < I; ++k) zmax = std::max(zmax, bit_len(Z + k * zl, zl));
  for (uint32_t m = 0; m < count; ++m) job.add_base(DA(oT + (size_t)m * nl * 4), nl, m);
  for (uint32_t m = 0; m < count; ++m)
    for (uint32_t k = 0; k < M; ++k) {
      const size_t q = (size_t)m * M + k;
      job.add(m, DA(oZ + q * zl * 4), zl, zmax, DA(oTZ + q * nl * 4));
      // T^Z_k == A_k * S^(e_k) mod N  (:144-148)
      EqOperand& e = ops[q];
      e.a = DA(oTZ + q * nl * 4);
      e.b = DA(oOne);
      e.c = DA(oA + q * nl * 4);
      e.d = DA(oS + (size_t)m * nl * 4);
      e.a_len = e.b_len = e.c_len = e.d_len = nl;
      e.sel = (uint32_t)((size_t)m * MW * 32 + k);
      e.flags = 0;
      mod_idx[q] = m;
    }
  hipStream_t st = c->stream;
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d + oN, N, bN, hipMemcpyHostToDevice, st), "H2D N")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oS, S, bN, hipMemcpyHostToDevice, st), "H2D S")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oT, T, bN, hipMemcpyHostToDevice, st), "H2D T")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oA, A, bA, hipMemcpyHostToDevice, st), "H2D A")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oZ, Z, bZ, hipMemcpyHostToDevice, st), "H2D Z")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oOne, one.data(), nl * 4, hipMemcpyHostToDevice, st), "H2D one")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oOps, ops.data(), I * sizeof(EqOperand), hipMemcpyHostToDevice, st),
                         "H2D eq ops")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oMod, mod_idx.data(), I * 4, hipMemcpyHostToDevice, st), "H2D idx")))
    return rc;
  uint32_t* cons = nullptr;
  if ((rc = setup_moduli(c, nl, (const uint32_t*)(d + oN), count, &cons, "rp"))) return rc;
  // challenge hash on a side stream, concurrent with the exponentiations
  hipEvent_t ready, hashed;
  if ((rc = c->hip_check(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "event"))) return rc;
  if ((rc = c->hip_check(hipEventCreateWithFlags(&hashed, hipEventDisableTiming), "event"))) return rc;
  (void)hipEventRecord(ready, st);
  hipStream_t hs = c->side_stream(0);
  (void)hipStreamWaitEvent(hs, ready, 0);
  PedHashArgs h{(const uint32_t*)(d + oA), M, nl, (uint32_t*)(d + oBits), (uint32_t*)(d + oPanic), count};
  c->mark("ped_hash", true, hs);
  rc = c->hip_check(launch_ped_hash(h, hs), "ped_hash");
  c->mark("ped_hash", false, hs);
  (void)hipEventRecord(hashed, hs);
  job.finalize();
  if (!rc) rc = fb_run(c, job, cons, "rp");
  (void)hipStreamWaitEvent(st, hashed, 0);
  (void)hipEventDestroy(ready);
  (void)hipEventDestroy(hashed);
  if (rc) return rc;
  EqCheckArgs ea{(const EqOperand*)(d + oOps), (const uint32_t*)(d + oMod), cons, (const uint32_t*)(d + oBits),
                 DA(oOne), (uint32_t*)(d + oEq), (uint32_t)I};
  c->mark("eq_check", true);
  rc = c->hip_check(launch_eq_check(nl, ea, st), "eq_check");
  c->mark("eq_check", false);
  if (rc) return rc;
  std::vector<uint32_t> eq(I), panic(count);
  if ((rc = c->hip_check(hipMemcpyAsync(eq.data(), d + oEq, I * 4, hipMemcpyDeviceToHost, st), "D2H eq")) ||
      (rc = c->hip_check(hipMemcpyAsync(panic.data(), d + oPanic, (size_t)count * 4, hipMemcpyDeviceToHost, st),
                         "D2H panic")))
    return rc;
  if ((rc = c->sync())) return rc;
  for (uint32_t m = 0; m < count; ++m) {
    verdict[m] = ped_verdict(&eq[(size_t)m * M], M, panic[m]);
  }
  return FSDKR_OK;
}

}  // extern "C"
