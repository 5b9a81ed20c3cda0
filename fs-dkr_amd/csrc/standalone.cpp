// Stand-alone verification entry points of the C ABI (include/fsdkr/fsdkr.h):
//   fsdkr_feldman_check          validate_collect's Feldman loop (refresh_message.rs:177-188)
//   fsdkr_ring_pedersen_verify   RingPedersenProof::verify (ring_pedersen_proof.rs:126-157)
//   fsdkr_pdl_u1_check           PDLwSlackProof::verify's u1 equation (zk_pdl_with_slack.rs:124-127,158)
// JoinMessage::collect (add_party_message.rs:136-175) needs exactly these two
// checks and none of the pair proofs, so it calls them instead of the whole
// fsdkr_verify_collect pipeline.  Both run on the context stream; the ring-
// Pedersen challenge hash overlaps the T^Z exponentiations (the challenge bits
// are only needed by the final equality check).
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "collect.hpp"
#include "ctx.hpp"
#include "fbjob.hpp"
#include "fsdkr/fsdkr.h"
#include "hostbn.hpp"
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
  const size_t vb = (size_t)n_msgs * (t + 1) * 16 * 4, cb = P * 16 * 4, ib = P * sizeof(FeldmanInfo);
  uint8_t* d = (uint8_t*)c->buf("fel_io", al256(vb) + al256(cb) + al256(ib) + P);
  if (!d) {
    c->fail("fsdkr_feldman_check: device allocation failed");
    return FSDKR_E_OOM;
  }
  uint32_t* d_vss = (uint32_t*)d;
  uint32_t* d_com = (uint32_t*)(d + al256(vb));
  FeldmanInfo* d_info = (FeldmanInfo*)(d + al256(vb) + al256(cb));
  uint8_t* d_out = d + al256(vb) + al256(cb) + al256(ib);
  std::vector<FeldmanInfo> info(P);
  for (size_t p = 0; p < P; ++p) info[p] = {(uint32_t)((p / n) * (t + 1)), t + 1, (uint32_t)(p % n) + 1, 0};
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_vss, vss, vb, hipMemcpyHostToDevice, c->stream), "H2D vss")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_com, commit, cb, hipMemcpyHostToDevice, c->stream), "H2D commit")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_info, info.data(), ib, hipMemcpyHostToDevice, c->stream), "H2D info")))
    return rc;
  FeldmanArgs f{d_vss, d_com, d_info, d_out, (uint32_t)P};
  c->mark("ec", true);
  rc = c->hip_check(launch_feldman(f, c->stream), "feldman");
  c->mark("ec", false);
  if (rc) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(verdict, d_out, P, hipMemcpyDeviceToHost, c->stream), "D2H feldman")))
    return rc;
  return c->sync();
}

int fsdkr_pdl_u1_check(fsdkr_ctx* ctx, uint32_t count, const uint32_t* s1, uint32_t s1_len, const uint32_t* e,
                       const uint32_t* Q, const uint32_t* u1, uint8_t* verdict) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!s1 || !e || !Q || !u1 || !verdict || s1_len == 0) {
    c->fail("fsdkr_pdl_u1_check: bad argument");
    return FSDKR_E_ARG;
  }
  const size_t sb = (size_t)count * s1_len * 4, eb = (size_t)count * 32, pb = (size_t)count * 64;
  uint8_t* d = (uint8_t*)c->buf("u1_io", al256(sb) + al256(eb) + 2 * al256(pb) + count);
  if (!d) {
    c->fail("fsdkr_pdl_u1_check: device allocation failed");
    return FSDKR_E_OOM;
  }
  uint32_t* d_s1 = (uint32_t*)d;
  uint32_t* d_e = (uint32_t*)(d + al256(sb));
  uint32_t* d_q = (uint32_t*)(d + al256(sb) + al256(eb));
  uint32_t* d_u = (uint32_t*)(d + al256(sb) + al256(eb) + al256(pb));
  uint8_t* d_out = d + al256(sb) + al256(eb) + 2 * al256(pb);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_s1, s1, sb, hipMemcpyHostToDevice, c->stream), "H2D s1")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_e, e, eb, hipMemcpyHostToDevice, c->stream), "H2D e")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_q, Q, pb, hipMemcpyHostToDevice, c->stream), "H2D Q")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_u, u1, pb, hipMemcpyHostToDevice, c->stream), "H2D u1")) ||
      (rc = c->hip_check(hipMemsetAsync(d_out, 0, count, c->stream), "memset u1")))
    return rc;
  PdlU1Args u{d_s1, d_e, d_q, d_u, s1_len, d_out, count};
  c->mark("ec", true);
  rc = c->hip_check(launch_pdl_u1(u, c->stream), "pdl_u1");
  c->mark("ec", false);
  if (rc) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(verdict, d_out, count, hipMemcpyDeviceToHost, c->stream), "D2H u1")))
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
  // N = 2^tz * odd: the Montgomery kernels run modulo the odd part, pow2.hip
  // checks the congruence modulo 2^tz (CRT).  N = 0: GMP aborts at the first
  // check (reported as the reference's panic); odd part 1: congruence mod 1 holds.
  std::vector<uint32_t> Nodd((size_t)count * nl), Sred((size_t)count * nl), tz(count, 0u);
  std::vector<uint8_t> mode(count, 0);   // 0 regular, 1 odd part 1, 2 modulus 0
  for (uint32_t m = 0; m < count; ++m) {
    uint32_t* on = Nodd.data() + (size_t)m * nl;
    memcpy(on, N + (size_t)m * nl, nl * 4);
    memcpy(Sred.data() + (size_t)m * nl, S + (size_t)m * nl, nl * 4);
    if (hbn::is_zero_raw(on, nl)) {
      mode[m] = 2;
      on[0] = 3;
      continue;
    }
    tz[m] = hbn::ctz_raw(on, nl);
    if (tz[m]) hbn::shr_raw(on, nl, tz[m]);
    if (on[0] == 1 && hbn::is_zero_raw(on + 1, nl - 1)) {
      mode[m] = 1;
      on[0] = 3;
      continue;
    }
    uint32_t* sd = Sred.data() + (size_t)m * nl;
    if (hbn::cmp_raw(sd, nl, on, nl) >= 0) hbn::store(hbn::mod(hbn::from(sd, nl), hbn::from(on, nl)), sd, nl);
  }
  const size_t MW = (M + 31) / 32;           // challenge-bit words per proof
  const size_t I = (size_t)count * M;        // T^Z instances
  const size_t bN = (size_t)count * nl * 4, bA = I * nl * 4, bZ = I * zl * 4;
  // device image: N | S | T | A | Z | one | bits | panic | TZ | eq | eq ops | eq mod idx
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off = al256(off + (bytes ? bytes : 1)); return o; };
  size_t n_p2 = 0;
  std::vector<uint32_t> p2_first(count, ~0u);
  for (uint32_t m = 0; m < count; ++m)
    if (tz[m] && mode[m] != 2) {
      p2_first[m] = (uint32_t)n_p2;
      n_p2 += M;
    }
  const size_t oN = take(bN), oS = take(bN), oT = take(bN), oA = take(bA), oZ = take(bZ), oOne = take(nl * 4);
  const size_t oBits = take((size_t)count * MW * 4), oPanic = take((size_t)count * 4), oTZ = take(bA);
  const size_t oEq = take(I * 4), oOps = take(I * sizeof(EqOperand)), oMod = take(I * 4);
  const size_t oSraw = take(bN), oP2 = take(n_p2 * sizeof(Pow2Op)), oP2o = take(n_p2 * 4);
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
  std::vector<Pow2Op> p2(n_p2);
  for (uint32_t m = 0; m < count; ++m) {
    if (p2_first[m] == ~0u) continue;
    for (uint32_t k = 0; k < M; ++k) {   // T^Z_k == A_k * S^e_k  (mod 2^tz)
      Pow2Op& o = p2[p2_first[m] + k];
      o = Pow2Op{};
      const size_t q = (size_t)m * M + k;
      o.a = DA(oT + (size_t)m * nl * 4);
      o.a_len = nl;
      o.ea = DA(oZ + q * zl * 4);
      o.ea_len = zl;
      o.c = DA(oA + q * nl * 4);
      o.c_len = nl;
      o.d = DA(oSraw + (size_t)m * nl * 4);
      o.d_len = nl;
      o.sel = (uint32_t)((size_t)m * MW * 32 + k);
      o.kbits = tz[m];
    }
  }
  hipStream_t st = c->stream;
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d + oN, Nodd.data(), bN, hipMemcpyHostToDevice, st), "H2D N")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oS, Sred.data(), bN, hipMemcpyHostToDevice, st), "H2D S")) ||
      (rc = c->hip_check(hipMemcpyAsync(d + oSraw, S, bN, hipMemcpyHostToDevice, st), "H2D S raw")) ||
      (n_p2 && (rc = c->hip_check(hipMemcpyAsync(d + oP2, p2.data(), n_p2 * sizeof(Pow2Op), hipMemcpyHostToDevice, st),
                                  "H2D pow2"))) ||
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
  if (!rc && n_p2) {
    Pow2Args pa{(const Pow2Op*)(d + oP2), (const uint32_t*)(d + oBits), (uint32_t*)(d + oP2o), (uint32_t)n_p2};
    rc = c->hip_check(launch_pow2_check(pa, hs), "pow2_check");
  }
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
  std::vector<uint32_t> eq(I), panic(count), p2o(n_p2);
  if ((rc = c->hip_check(hipMemcpyAsync(eq.data(), d + oEq, I * 4, hipMemcpyDeviceToHost, st), "D2H eq")) ||
      (rc = c->hip_check(hipMemcpyAsync(panic.data(), d + oPanic, (size_t)count * 4, hipMemcpyDeviceToHost, st),
                         "D2H panic")) ||
      (n_p2 && (rc = c->hip_check(hipMemcpyAsync(p2o.data(), d + oP2o, n_p2 * 4, hipMemcpyDeviceToHost, st),
                                  "D2H pow2"))))
    return rc;
  if ((rc = c->sync())) return rc;
  for (uint32_t m = 0; m < count; ++m) {
    uint32_t* e = &eq[(size_t)m * M];
    if (mode[m] == 1)
      for (uint32_t k = 0; k < M; ++k) e[k] = 1;
    if (p2_first[m] != ~0u)
      for (uint32_t k = 0; k < M; ++k) e[k] = e[k] && p2o[p2_first[m] + k];
    verdict[m] = mode[m] == 2 ? 2 : ped_verdict(e, M, panic[m]);
  }
  return FSDKR_OK;
}

// out[i] = base[i]^E[mod_idx[i]] * base2[i]^exp2[i] mod N[mod_idx[i]] through the
// split chains of collect()'s GA (head over E's bits >= 256, joint tail), for
// parity tests of that path (modexp.hip modexp_tail_kernel).
int fsdkr_modexp_joint_batch(fsdkr_ctx* ctx, uint32_t count, const uint32_t* base, const uint32_t* base2,
                             const uint32_t* exp2, const uint32_t* mod_idx, const uint32_t* mods,
                             const uint32_t* mod_exp, uint32_t exp_limbs, uint32_t n_mod, uint32_t* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  constexpr uint32_t K = 128, E2L = 8, LO = 256;
  if (!base || !base2 || !exp2 || !mod_idx || !mods || !mod_exp || !out || !n_mod || !exp_limbs) {
    c->fail("fsdkr_modexp_joint_batch: null pointer or empty table");
    return FSDKR_E_ARG;
  }
  uint32_t ebits = 1;
  for (uint32_t m = 0; m < n_mod; ++m) {
    if ((mods[(size_t)m * K] & 1u) == 0) {
      c->fail("fsdkr_modexp_joint_batch: modulus %u is even", m);
      return FSDKR_E_ARG;
    }
    ebits = std::max(ebits, bit_len(mod_exp + (size_t)m * exp_limbs, exp_limbs));
  }
  for (uint32_t i = 0; i < count; ++i)
    if (mod_idx[i] >= n_mod) {
      c->fail("fsdkr_modexp_joint_batch: mod_idx[%u] out of range", i);
      return FSDKR_E_ARG;
    }
  const uint32_t group = (c->modexp_group == 8 || c->modexp_group == 4 || c->modexp_group == kWideGroup)
                             ? c->modexp_group : 16u,
                 per_wave = 64 / group;
  const size_t o_b = 0, o_b2 = al256((size_t)count * K * 4), o_e2 = o_b2 + al256((size_t)count * K * 4),
               o_m = o_e2 + al256((size_t)count * E2L * 4), o_me = o_m + al256((size_t)n_mod * K * 4),
               o_out = o_me + al256((size_t)n_mod * exp_limbs * 4), o_desc = o_out + al256(((size_t)count + 1) * K * 4);
  const size_t cap = (size_t)count + (size_t)n_mod * per_wave;   // instances + pads
  const size_t o_desc2 = o_desc + al256(cap * 36), total = o_desc2 + al256(cap * 20);
  uint8_t* dev = (uint8_t*)c->buf("mxj", total);
  if (!dev) {
    c->fail("fsdkr_modexp_joint_batch: device allocation failed");
    return FSDKR_E_OOM;
  }
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };
  ModexpJob J;
  J.k32 = K;
  for (uint32_t i = 0; i < count; ++i)
    J.add(DI(o_b + (size_t)i * K * 4), K, DI(o_me + (size_t)mod_idx[i] * exp_limbs * 4), exp_limbs, ebits, mod_idx[i]);
  const bool aligned = group_by_exponent(J, per_wave, count);
  if (!aligned) {
    c->fail("fsdkr_modexp_joint_batch: instances not wave-uniform");
    return FSDKR_E_ARG;
  }
  std::vector<uint8_t> desc;
  J.pack(desc);
  const size_t n = J.size();
  std::vector<uint8_t> desc2(n * 20, 0);
  auto* b2p = reinterpret_cast<uint64_t*>(desc2.data());
  auto* e2p = reinterpret_cast<uint64_t*>(desc2.data() + n * 8);
  auto* e2l = reinterpret_cast<uint32_t*>(desc2.data() + n * 16);
  for (size_t k = 0; k < n; ++k) {
    const uint32_t r = J.out_idx[k];   // the pads write row `count`
    const uint32_t src = r < count ? r : 0u;
    b2p[k] = DI(o_b2 + (size_t)src * K * 4);
    e2p[k] = DI(o_e2 + (size_t)src * E2L * 4);
    e2l[k] = r < count ? E2L : 0u;
  }
  int rc;
  auto up = [&](size_t o, const void* src, size_t bytes) {
    return c->hip_check(hipMemcpyAsync(dev + o, src, bytes, hipMemcpyHostToDevice, c->stream), "H2D joint");
  };
  if ((rc = up(o_b, base, (size_t)count * K * 4)) || (rc = up(o_b2, base2, (size_t)count * K * 4)) ||
      (rc = up(o_e2, exp2, (size_t)count * E2L * 4)) || (rc = up(o_m, mods, (size_t)n_mod * K * 4)) ||
      (rc = up(o_me, mod_exp, (size_t)n_mod * exp_limbs * 4)) || (rc = up(o_desc, desc.data(), desc.size())) ||
      (rc = up(o_desc2, desc2.data(), desc2.size())))
    return rc;
  uint32_t* cons = nullptr;
  if ((rc = setup_moduli(c, K, reinterpret_cast<const uint32_t*>(dev + o_m), n_mod, &cons,
                         group == kWideGroup ? "joint_w" : "joint", group == kWideGroup ? kWideGroup : 0u)))
    return rc;
  const uint32_t flags = ga_desc_flags(true, group);
  SplitArgs head;
  head.lo_bit = LO;
  SplitArgs tail = head;
  tail.tail = true;
  tail.d_desc2 = dev + o_desc2;
  uint32_t* d_out = reinterpret_cast<uint32_t*>(dev + o_out);
  if ((rc = launch_modexp_desc(c, K, (uint32_t)n, ebits, dev + o_desc, cons, d_out, c->stream, "mxt_joint", 0, group,
                               flags, &head)) ||
      (rc = launch_modexp_desc(c, K, (uint32_t)n, ebits, dev + o_desc, cons, d_out, c->stream, "mxt_joint", 0, group,
                               flags, &tail)))
    return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(out, d_out, (size_t)count * K * 4, hipMemcpyDeviceToHost, c->stream), "D2H")))
    return rc;
  return c->sync();
}

}  // extern "C"
