// Host orchestration of the batched RefreshMessage::collect verification
// (fsdkr_verify_collect) and the first-error mapping (fsdkr_collect_first_error).
//
// Reference: /root/reference/src/refresh_message.rs:321-467 (collect),
// :147-191 (validate_collect); zk_pdl_with_slack.rs:113-188; range_proofs.rs:112-164;
// ring_pedersen_proof.rs:126-157; zk-paillier NiCorrectKeyProof / CompositeDLogProof.
//
// Pipeline (one HIP stream, one H2D copy of inputs + descriptors):
//   pdl_hash, ped_hash -> binom -> 9 modexp jobs -> inverses -> eq_check / prod3
//   -> alice_hash, pdl_u1, feldman -> one D2H copy of the verdict words.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.hpp"
#include "fbjob.hpp"
#include "fsdkr/fsdkr.h"
#include "hostbn.hpp"
#include "kernels.h"
#include "sha256.hpp"
#include "verify.h"

namespace fsdkr {
namespace {

constexpr uint32_t CK_M2 = 11;      // zk-paillier correct_key_ni M2
constexpr uint32_t CK_ALPHA = 6370; // zk-paillier primorial bound [dep, unverified]
const uint8_t SALT[4] = {75, 90, 101, 110};  // SALT_STRING "KZen" [dep, unverified]

const uint32_t Q_LIMBS_H[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                               0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

const std::vector<uint32_t>& small_primes() {
  static std::vector<uint32_t> ps = [] {
    std::vector<uint32_t> v;
    std::vector<bool> comp(CK_ALPHA, false);
    for (uint32_t i = 2; i < CK_ALPHA; ++i) {
      if (comp[i]) continue;
      v.push_back(i);
      for (uint32_t j = i * i; j < CK_ALPHA; j += i) comp[j] = true;
    }
    return v;
  }();
  return ps;
}

// Device layout builder: inputs (with host data) and outputs share one allocation.
struct Layout {
  std::vector<uint8_t> host;   // bytes to upload (inputs + descriptors)
  size_t out_bytes = 0;        // outputs placed after the inputs
  static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
  size_t in(const void* src, size_t bytes) {
    const size_t o = al(host.size());
    host.resize(o + al(bytes ? bytes : 1), 0);
    if (src && bytes) memcpy(host.data() + o, src, bytes);
    return o;
  }
  size_t in_vec(const std::vector<uint8_t>& v) { return in(v.data(), v.size()); }
  template <class T>
  size_t in_vecT(const std::vector<T>& v) { return in(v.data(), v.size() * sizeof(T)); }
  // returns an OUTPUT offset (relative to the output region)
  size_t out(size_t bytes) {
    const size_t o = al(out_bytes);
    out_bytes = o + al(bytes ? bytes : 1);
    return o;
  }
};

struct Sizes {
  uint32_t R, J, n, P, Mt, M, nl, nn;
};

inline bool is_odd(const uint32_t* p) { return (p[0] & 1u) != 0; }
inline bool all_zero(const uint32_t* p, size_t n) {
  for (size_t k = 0; k < n; ++k)
    if (p[k]) return false;
  return true;
}

// to_bytes(x) absorbed for a small non-negative integer
inline void absorb_u32(Sha256& h, uint32_t v) { h.bigint(&v, 1); }

}  // namespace

// ------------------------------------------------------------------------------
// Everything the run phase needs after the host pre-pass and the upload.
struct CollectPlan {
  Sizes s{};
  uint32_t el = 0, t = 0;
  size_t in_bytes = 0, out_off = 0, total = 0;
  uint8_t* dev = nullptr;
  // input offsets used by launches
  size_t o_Q, o_enc, o_pz, o_pu1, o_pu2, o_pu3, o_ps1, o_pA, o_az, o_ae, o_vss, o_NN, o_mods, o_one, o_rn;
  uint32_t s1l = 0, n_mods_nl = 0;
  // output offsets
  size_t x_epdl, x_pbits, x_ppanic, x_Bpdl, x_gs1, x_J[10], x_invc, x_invz, x_unn, x_uzA, x_uzp, x_eq2, x_eq3, x_u,
      x_w, x_fel, x_pdlv, x_rng;
  // descriptor offsets + counts
  size_t d_J[10], d_bs, d_bn, d_iynn, d_imnn, d_iynl, d_imnl, d_eqnn, d_eqnnm, d_eqnl, d_eqnlm, d_p3nn, d_p3nl, d_p3m,
      d_ahn, d_ahc, d_alpre;
  uint32_t jk32[10], jcount[10], jbits[10];
  uint32_t n_inv_nn = 0, n_eq_nn = 0, n_eq_nl = 0;
  std::vector<uint32_t> cpdl_extra, ae_bits;
  std::vector<uint8_t> ck_pre, dlog_pre;
  FbJob fb;                 // h1_i, h2_i, ring-Pedersen T: fixed-base job
  size_t d_FB = 0;          // its descriptor image (input region)
  uint32_t* fb_table = nullptr;   // its scratch (separate context buffer)
  uint16_t* fb_sched = nullptr;
  uint32_t* fb_nsteps = nullptr;
};

void free_collect_plan(Ctx* c) {
  delete reinterpret_cast<CollectPlan*>(c->plan);
  c->plan = nullptr;
}

int collect_prepare(Ctx* c, const fsdkr_collect_batch* b) {
  free_collect_plan(c);
  CollectPlan* plan = new CollectPlan();
  c->plan = plan;
  CollectPlan& pl = *plan;
  Sizes& s = pl.s;
  s.R = b->n_refresh;
  s.J = b->n_join;
  s.n = b->n_recv ? b->n_recv : s.R + s.J;
  s.P = s.R * s.n;
  s.Mt = s.R + s.J;
  s.M = b->m_security;
  s.nl = b->nl;
  s.nn = 2 * b->nl;
  if (s.n < s.R || s.M == 0 || !(s.nl == 64 || s.nl == 96) || b->s1l == 0 || b->s3l == 0 || b->el == 0 ||
      b->zl == 0 || (s.J && b->yl == 0)) {
    c->fail("fsdkr_verify_collect: unsupported shape (R=%u nl=%u)", s.R, s.nl);
    return FSDKR_E_UNSUPPORTED;
  }
  const uint32_t nl = s.nl, nn = s.nn, P = s.P, n = s.n, Mt = s.Mt, M = s.M, R = s.R, J = s.J;
  // odd moduli are required by the Montgomery kernels
  for (uint32_t i = 0; i < n; ++i)
    if (!is_odd(b->recv_n + (size_t)i * nl) || !is_odd(b->recv_ntilde + (size_t)i * nl)) {
      c->fail("receiver %u: even Paillier or DLog modulus (unsupported)", i);
      return FSDKR_E_UNSUPPORTED;
    }
  for (uint32_t m = 0; m < Mt; ++m)
    if (!is_odd(b->ped_N + (size_t)m * nl)) {
      c->fail("message %u: even ring-Pedersen modulus (unsupported)", m);
      return FSDKR_E_UNSUPPORTED;
    }
  for (uint32_t j = 0; j < J; ++j)
    if (!is_odd(b->dlog_N + (size_t)j * nl)) {
      c->fail("join %u: even DLog modulus (unsupported)", j);
      return FSDKR_E_UNSUPPORTED;
    }

  // ---------------- host pre-computation (O(n) + O(P) scans, no big exponentiations)
  // NN_i = N_i^2, N_i + 1
  std::vector<uint32_t> NN((size_t)n * nn), NP1((size_t)n * nn);
  for (uint32_t i = 0; i < n; ++i) {
    hbn::Limbs N = hbn::from(b->recv_n + (size_t)i * nl, nl);
    hbn::store(hbn::mul(N, N), NN.data() + (size_t)i * nn, nn);
    hbn::store(hbn::add_small(N, 1), NP1.data() + (size_t)i * nn, nn);
  }
  // q^3 for the Alice s1 bound (range_proofs.rs:125)
  const hbn::Limbs q = hbn::from(Q_LIMBS_H, 8);
  const hbn::Limbs q3 = hbn::mul(hbn::mul(q, q), q);
  std::vector<uint8_t> alice_pre(P), pdl_small(P);
  std::vector<uint32_t> s1_bits(P), s3_bits(P), a1_bits(P), a2_bits(P);
  std::vector<uint32_t>& ae_bits = pl.ae_bits;
  ae_bits.assign(P, 0);
  uint32_t pdl_s1_max = 1, pdl_s3_max = 1, a_s1_max = 1, a_s2_max = 1, a_e_max = 1;
  bool any_big_s1 = false;
  for (uint32_t p = 0; p < P; ++p) {
    const uint32_t i = p % n;
    const uint32_t Nbits = hbn::bitlen(b->recv_n + (size_t)i * nl, nl);
    const uint32_t* s1 = b->pdl_s1 + (size_t)p * b->s1l;
    s1_bits[p] = hbn::bitlen(s1, b->s1l);
    // s1 < N  -> (N+1)^s1 mod N^2 = 1 + s1*N  (binomial, bit-identical)
    bool small = s1_bits[p] < Nbits;
    if (!small && s1_bits[p] == Nbits) small = hbn::cmp(hbn::from(s1, b->s1l), hbn::from(b->recv_n + (size_t)i * nl, nl)) < 0;
    pdl_small[p] = small ? 1 : 0;
    any_big_s1 = any_big_s1 || !small;
    s3_bits[p] = hbn::bitlen(b->pdl_s3 + (size_t)p * b->s3l, b->s3l);
    const uint32_t* as1 = b->rp_s1 + (size_t)p * b->s1l;
    a1_bits[p] = hbn::bitlen(as1, b->s1l);
    a2_bits[p] = hbn::bitlen(b->rp_s2 + (size_t)p * b->s3l, b->s3l);
    ae_bits[p] = hbn::bitlen(b->rp_e + (size_t)p * b->el, b->el);
    const bool s1_ok = hbn::cmp(hbn::from(as1, b->s1l), q3) <= 0;
    alice_pre[p] = (s1_ok && ae_bits[p] <= 256) ? 1 : 0;
    pdl_s1_max = std::max(pdl_s1_max, s1_bits[p]);
    pdl_s3_max = std::max(pdl_s3_max, s3_bits[p]);
    if (alice_pre[p]) {  // exponents of rejected proofs are never used
      a_s1_max = std::max(a_s1_max, a1_bits[p]);
      a_s2_max = std::max(a_s2_max, a2_bits[p]);
      a_e_max = std::max(a_e_max, ae_bits[p]);
    }
  }
  // correct-key: rho_j = mask_generation(len(n), H(n, salt, j)) mod n; primorial gcd
  std::vector<uint32_t> RHO((size_t)Mt * CK_M2 * nl);
  std::vector<uint8_t>& ck_pre = pl.ck_pre;
  ck_pre.assign(Mt, 0);
  for (uint32_t m = 0; m < Mt; ++m) {
    const uint32_t* ckn = b->ck_n + (size_t)m * nl;
    const hbn::Limbs N = hbn::from(ckn, nl);
    bool ok = !N.empty();
    for (uint32_t pr : small_primes())
      if (ok && hbn::mod_small(N, pr) == 0) ok = false;
    ck_pre[m] = ok ? 1 : 0;
    const uint32_t key_len = hbn::bitlen(N);
    const uint32_t msklen = key_len / 256 + 1;
    const uint32_t salt_v = ((uint32_t)SALT[0] << 24) | ((uint32_t)SALT[1] << 16) | ((uint32_t)SALT[2] << 8) | SALT[3];
    for (uint32_t j = 0; j < CK_M2; ++j) {
      Sha256 h;
      h.init();
      h.bigint(ckn, nl);
      absorb_u32(h, salt_v);
      absorb_u32(h, j);
      uint32_t seed[8];
      h.finish_le(seed);
      std::vector<uint32_t> mask((size_t)msklen * 8, 0);
      for (uint32_t k = 0; k < msklen; ++k) {
        Sha256 hk;
        hk.init();
        hk.bigint(seed, 8);
        absorb_u32(hk, k);
        hk.finish_le(mask.data() + (size_t)k * 8);
      }
      if (N.empty()) continue;
      hbn::store(hbn::mod(hbn::from(mask.data(), mask.size()), N), RHO.data() + ((size_t)m * CK_M2 + j) * nl, nl);
    }
  }
  // DLog statements: N > 2^128, gcd(g, N) = gcd(ni, N) = 1; challenges e = H(x, g, N, ni)
  std::vector<uint8_t>& dlog_pre = pl.dlog_pre;
  dlog_pre.assign(J, 0);
  std::vector<uint32_t> DE((size_t)J * 2 * 8);
  uint32_t y_max = 1;
  for (uint32_t j = 0; j < J; ++j) {
    const uint32_t *N = b->dlog_N + (size_t)j * nl, *g = b->dlog_g + (size_t)j * nl, *ni = b->dlog_ni + (size_t)j * nl;
    const hbn::Limbs Nl = hbn::from(N, nl);
    bool ok = hbn::bitlen(Nl) > 129 || (hbn::bitlen(Nl) == 129 && !(Nl.size() == 5 && Nl[4] == 1 && all_zero(N, 4)));
    ok = ok && hbn::is_one(hbn::gcd(hbn::from(g, nl), Nl)) && hbn::is_one(hbn::gcd(hbn::from(ni, nl), Nl));
    dlog_pre[j] = ok ? 1 : 0;
    for (int which = 0; which < 2; ++which) {
      const uint32_t* x = (which == 0 ? b->dlog_x1 : b->dlog_x2) + (size_t)j * nl;
      const uint32_t* gg = which == 0 ? g : ni;
      const uint32_t* nn_ = which == 0 ? ni : g;
      Sha256 h;
      h.init();
      h.bigint(x, nl);
      h.bigint(gg, nl);
      h.bigint(N, nl);
      h.bigint(nn_, nl);
      h.finish_le(DE.data() + ((size_t)j * 2 + which) * 8);
    }
    y_max = std::max(y_max, hbn::bitlen(b->dlog_y1 + (size_t)j * b->yl, b->yl));
    y_max = std::max(y_max, hbn::bitlen(b->dlog_y2 + (size_t)j * b->yl, b->yl));
  }
  uint32_t z_max = 1;
  for (size_t k = 0; k < (size_t)Mt * M; ++k) z_max = std::max(z_max, hbn::bitlen(b->ped_Z + k * b->zl, b->zl));
  uint32_t ckn_max = 1;
  for (uint32_t m = 0; m < Mt; ++m) ckn_max = std::max(ckn_max, hbn::bitlen(b->ck_n + (size_t)m * nl, nl));
  uint32_t recvn_max = 1;
  for (uint32_t i = 0; i < n; ++i) recvn_max = std::max(recvn_max, hbn::bitlen(b->recv_n + (size_t)i * nl, nl));

  // ---------------- device layout: inputs
  Layout L;
  auto IN = [&](const uint32_t* p, size_t words) { return L.in(p, words * 4); };
  const size_t o_rn = IN(b->recv_n, (size_t)n * nl), o_rt = IN(b->recv_ntilde, (size_t)n * nl);
  const size_t o_h1 = IN(b->recv_h1, (size_t)n * nl), o_h2 = IN(b->recv_h2, (size_t)n * nl);
  const size_t o_NN = IN(NN.data(), NN.size()), o_NP1 = IN(NP1.data(), NP1.size());
  const size_t o_enc = IN(b->enc, (size_t)P * nn), o_Q = IN(b->commit, (size_t)P * 16);
  const size_t o_pz = IN(b->pdl_z, (size_t)P * nl), o_pu1 = IN(b->pdl_u1, (size_t)P * 16);
  const size_t o_pu2 = IN(b->pdl_u2, (size_t)P * nn), o_pu3 = IN(b->pdl_u3, (size_t)P * nl);
  const size_t o_ps1 = IN(b->pdl_s1, (size_t)P * b->s1l), o_ps2 = IN(b->pdl_s2, (size_t)P * nl);
  const size_t o_ps3 = IN(b->pdl_s3, (size_t)P * b->s3l);
  const size_t o_az = IN(b->rp_z, (size_t)P * nl), o_ae = IN(b->rp_e, (size_t)P * b->el);
  const size_t o_as = IN(b->rp_s, (size_t)P * nl), o_as1 = IN(b->rp_s1, (size_t)P * b->s1l);
  const size_t o_as2 = IN(b->rp_s2, (size_t)P * b->s3l);
  const size_t o_vss = IN(b->vss, (size_t)R * (b->t + 1) * 16);
  const size_t o_pS = IN(b->ped_S, (size_t)Mt * nl), o_pT = IN(b->ped_T, (size_t)Mt * nl);
  const size_t o_pN = IN(b->ped_N, (size_t)Mt * nl);
  const size_t o_pA = IN(b->ped_A, (size_t)Mt * M * nl), o_pZ = IN(b->ped_Z, (size_t)Mt * M * b->zl);
  const size_t o_ckn = IN(b->ck_n, (size_t)Mt * nl), o_cks = IN(b->ck_sigma, (size_t)Mt * CK_M2 * nl);
  const size_t o_rho = IN(RHO.data(), RHO.size());
  size_t o_dN = 0, o_dg = 0, o_dni = 0, o_dx1 = 0, o_dx2 = 0, o_dy1 = 0, o_dy2 = 0, o_de = 0;
  if (J) {
    o_dN = IN(b->dlog_N, (size_t)J * nl);
    o_dg = IN(b->dlog_g, (size_t)J * nl);
    o_dni = IN(b->dlog_ni, (size_t)J * nl);
    o_dx1 = IN(b->dlog_x1, (size_t)J * nl);
    o_dx2 = IN(b->dlog_x2, (size_t)J * nl);
    o_dy1 = IN(b->dlog_y1, (size_t)J * b->yl);
    o_dy2 = IN(b->dlog_y2, (size_t)J * b->yl);
    o_de = IN(DE.data(), DE.size());
  }
  std::vector<uint32_t> ONE(nn, 0);
  ONE[0] = 1;
  const size_t o_one = IN(ONE.data(), nn);
  // nl-width moduli table: Ntilde_i | ped_N | ck_n | dlog_N   (mod_setup reads [cnt][nl])
  std::vector<uint32_t> MODS((size_t)(n + 2 * Mt + J) * nl);
  memcpy(MODS.data(), b->recv_ntilde, (size_t)n * nl * 4);
  memcpy(MODS.data() + (size_t)n * nl, b->ped_N, (size_t)Mt * nl * 4);
  for (uint32_t m = 0; m < Mt; ++m) {  // even / zero correct-key moduli: placeholder 3 (verdict forced false)
    uint32_t* dst = MODS.data() + (size_t)(n + Mt + m) * nl;
    memcpy(dst, b->ck_n + (size_t)m * nl, nl * 4);
    if (!is_odd(dst)) {
      std::fill(dst, dst + nl, 0u);
      dst[0] = 3;
      ck_pre[m] = 0;
    }
  }
  if (J) memcpy(MODS.data() + (size_t)(n + 2 * Mt) * nl, b->dlog_N, (size_t)J * nl * 4);
  const uint32_t n_mods_nl = n + 2 * Mt + J;
  const size_t o_mods = IN(MODS.data(), MODS.size());

  // ---------------- device layout: outputs
  const size_t x_epdl = L.out((size_t)P * 8 * 4);
  const size_t x_pbits = L.out((size_t)Mt * ((M + 31) / 32) * 4), x_ppanic = L.out((size_t)Mt * 4);
  const size_t x_Bpdl = L.out((size_t)P * nn * 4), x_gs1 = L.out((size_t)P * nn * 4);
  // modexp outputs, laid out per merged launch (instance k of a launch writes slot k):
  //   GA (nn, long)  = J1 s2^N | s^N  [2P]  ++  J9 (N+1)^s1 for s1 >= N  [<= P]
  //   J2 (nn, short) = c^e_pdl | c^e_A  [2P]
  //   J5 (nl, short) = z^e_pdl | zA^e_A [2P]
  //   GD (nl, long)  = J7 g^y1 | ni^y2 [2J] ++ J6 sigma^n [Mt*11] ++ J8 ni^e1 | g^e2 [2J]
  //   FB (nl, fixed bases h1_i, h2_i, T_m; any slot) = J4 h2^s3 | h2^s2A [2P], J3 h1^s1 | h1^s1A [2P],
  //                    RP T^Z [Mt*M]
  const size_t x_GA = L.out((size_t)3 * P * nn * 4 + 4);
  const size_t x_J1 = x_GA, x_J9 = x_GA + (size_t)2 * P * nn * 4;
  const size_t x_J2 = L.out((size_t)2 * P * nn * 4);
  const size_t x_J5 = L.out((size_t)2 * P * nl * 4);
  const size_t x_GD = L.out(((size_t)4 * J + (size_t)Mt * CK_M2 + 1) * nl * 4);
  const size_t x_J7 = x_GD, x_J6 = x_J7 + (size_t)2 * J * nl * 4, x_J8 = x_J6 + (size_t)Mt * CK_M2 * nl * 4;
  const size_t x_FB = L.out(((size_t)4 * P + (size_t)Mt * M + 1) * nl * 4);
  const size_t x_J4 = x_FB, x_J3 = x_J4 + (size_t)2 * P * nl * 4, x_RP = x_J3 + (size_t)2 * P * nl * 4;
  const size_t x_invc = L.out((size_t)2 * P * nn * 4), x_invz = L.out((size_t)P * nl * 4);
  const size_t x_unn = L.out((size_t)2 * P * 4);    // unit flags of the nn inverses (c^eA, then extra c^e_pdl)
  const size_t x_uzA = L.out((size_t)P * 4), x_uzp = L.out((size_t)P * 4);
  const size_t x_eq2 = L.out((size_t)P * 4);
  const size_t n_eqnl = (size_t)P + (size_t)Mt * M + (size_t)Mt * CK_M2 + 2 * J;
  const size_t x_eq3 = L.out(n_eqnl * 4);           // [u3 P | RP Mt*M | CK Mt*11 | DLog 2J]
  const size_t x_u = L.out((size_t)P * nn * 4), x_w = L.out((size_t)P * nl * 4);
  const size_t x_fel = L.out(P), x_pdlv = L.out(P), x_rng = L.out(P);

  // single device allocation: [inputs | descriptors | outputs]; descriptors are
  // appended to the input image below once the device base address is known.
  const size_t in_bytes_pre = L.host.size();
  // upper bound of descriptor bytes
  const size_t n_inst_nn = 2 * P + 2 * P + (any_big_s1 ? P : 0);
  const size_t n_inst_nl = 2 * P * 3 + (size_t)Mt * (M + CK_M2) + 4 * J;
  const size_t desc_bound = (n_inst_nn + n_inst_nl) * 32 + 16 * 256 +
                            ((size_t)P + (size_t)Mt * M + (size_t)Mt * CK_M2 + 2 * J + P) * sizeof(EqOperand) +
                            2 * (size_t)P * sizeof(Prod3Operand) + (size_t)(2 * P + 2 * P) * 16 + (size_t)4 * P * 8 +
                            (size_t)(2 * P + 2 * P) * 4 + (size_t)(3 * n + Mt) * 32 + 64 * 1024;
  const size_t total = Layout::al(in_bytes_pre + desc_bound) + L.out_bytes;
  uint8_t* dev = (uint8_t*)c->buf("collect_arena", total);
  if (!dev) {
    c->fail("fsdkr_verify_collect: device allocation of %zu bytes failed", total);
    return FSDKR_E_OOM;
  }
  uint8_t* const out_base = dev + Layout::al(in_bytes_pre + desc_bound);
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };          // input address
  auto DX = [&](size_t o) { return (uint64_t)(uintptr_t)(out_base + o); };     // output address
  auto PX = [&](size_t o) { return (uint32_t*)(out_base + o); };
  auto PI = [&](size_t o) { return (const uint32_t*)(dev + o); };

  // ---------------- modexp jobs
  ModexpJob J1, J2, J5, J6, J7, J8, J9;
  J1.k32 = J2.k32 = J9.k32 = nn;
  J5.k32 = J6.k32 = J7.k32 = J8.k32 = nl;
  // receiver bases h1_i, h2_i (mod N~_i = nl-table row i) and ring-Pedersen T_m (row n + m):
  // shared by 2n resp. M exponents -> BGMW tables (fixedbase.hip)
  FbJob& FB = pl.fb;
  FB = FbJob();
  FB.k32 = nl;
  std::vector<uint32_t> fb_h1(n), fb_h2(n);
  for (uint32_t i = 0; i < n; ++i) {
    fb_h1[i] = FB.add_base(DI(o_h1 + (size_t)i * nl * 4), nl, i);
    fb_h2[i] = FB.add_base(DI(o_h2 + (size_t)i * nl * 4), nl, i);
  }
  for (uint32_t m = 0; m < Mt; ++m) FB.add_base(DI(o_pT + (size_t)m * nl * 4), nl, n + m);
  std::vector<uint32_t> j9_pairs;
  for (int which = 0; which < 2; ++which)
    for (uint32_t p = 0; p < P; ++p) {
      const uint32_t i = p % n;
      const uint64_t Ni = DI(o_rn + (size_t)i * nl * 4);
      // J1: s2^N (PDL, zk_pdl_with_slack.rs:129-135) | s^N (Alice, range_proofs.rs:148)
      J1.add(which == 0 ? DI(o_ps2 + (size_t)p * nl * 4) : DI(o_as + (size_t)p * nl * 4), nl, Ni, nl, recvn_max, i);
      // J2: c^e (PDL :136-142 via the cross-multiplied check) | c^e (Alice :142)
      const uint64_t cp = DI(o_enc + (size_t)p * nn * 4);
      if (which == 0) J2.add(cp, nn, DX(x_epdl + (size_t)p * 32), 8, 256, i);
      else J2.add(cp, nn, DI(o_ae + (size_t)p * b->el * 4), b->el, a_e_max, i);
      // fixed bases (FB): h1^s1 -> J3 slot | h2^s3 (s2 for Alice) -> J4 slot;  J5: z^e
      const size_t slot = (size_t)which * P + p;
      if (which == 0) {
        FB.add(fb_h1[i], DI(o_ps1 + (size_t)p * b->s1l * 4), b->s1l, pdl_s1_max, DX(x_J3 + slot * nl * 4));
        FB.add(fb_h2[i], DI(o_ps3 + (size_t)p * b->s3l * 4), b->s3l, pdl_s3_max, DX(x_J4 + slot * nl * 4));
        J5.add(DI(o_pz + (size_t)p * nl * 4), nl, DX(x_epdl + (size_t)p * 32), 8, 256, i);
      } else {
        const bool use = alice_pre[p];
        FB.add(fb_h1[i], DI(o_as1 + (size_t)p * b->s1l * 4), use ? b->s1l : 0, a_s1_max, DX(x_J3 + slot * nl * 4));
        FB.add(fb_h2[i], DI(o_as2 + (size_t)p * b->s3l * 4), use ? b->s3l : 0, a_s2_max, DX(x_J4 + slot * nl * 4));
        J5.add(DI(o_az + (size_t)p * nl * 4), nl, DI(o_ae + (size_t)p * b->el * 4), use ? b->el : 0, a_e_max, i);
      }
    }
  for (uint32_t p = 0; p < P; ++p)
    if (!pdl_small[p]) {
      const uint32_t i = p % n;
      J9.add(DI(o_NP1 + (size_t)i * nn * 4), nn, DI(o_ps1 + (size_t)p * b->s1l * 4), b->s1l, pdl_s1_max, i);
      j9_pairs.push_back(p);
    }
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < M; ++k)  // ring-Pedersen T^Z_k mod N (ring_pedersen_proof.rs:144)
      FB.add(2 * n + m, DI(o_pZ + ((size_t)m * M + k) * b->zl * 4), b->zl, z_max, DX(x_RP + ((size_t)m * M + k) * nl * 4));
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < CK_M2; ++k)  // correct-key sigma_k^n mod n
      J6.add(DI(o_cks + ((size_t)m * CK_M2 + k) * nl * 4), nl, DI(o_ckn + (size_t)m * nl * 4), nl,
             std::max(ckn_max, z_max), n + Mt + m);
  for (uint32_t j = 0; j < J; ++j) {
    const uint32_t mi = n + 2 * Mt + j;
    J7.add(DI(o_dg + (size_t)j * nl * 4), nl, DI(o_dy1 + (size_t)j * b->yl * 4), b->yl, y_max, mi);
    J7.add(DI(o_dni + (size_t)j * nl * 4), nl, DI(o_dy2 + (size_t)j * b->yl * 4), b->yl, y_max, mi);
    J8.add(DI(o_dni + (size_t)j * nl * 4), nl, DI(o_de + (size_t)(2 * j) * 32), 8, 256, mi);
    J8.add(DI(o_dg + (size_t)j * nl * 4), nl, DI(o_de + (size_t)(2 * j + 1) * 32), 8, 256, mi);
  }
  // descriptor images appended to the input image
  auto pack_job = [&](const ModexpJob& j) {
    const size_t o = Layout::al(L.host.size());
    L.host.resize(o);
    j.pack(L.host);
    return o;
  };
  ModexpJob GA = J1, GD = J7;
  GA.append(J9);
  GD.append(J6);
  GD.append(J8);
  const size_t d_GA = pack_job(GA), d_J2 = pack_job(J2), d_J5 = pack_job(J5), d_GD = pack_job(GD);
  FB.finalize();
  const size_t d_FB = Layout::al(L.host.size());
  {
    std::vector<uint8_t> img;
    FB.pack(img);
    L.host.resize(d_FB);
    L.host.insert(L.host.end(), img.begin(), img.end());
  }

  // binom descriptors: PDL B = 1 + s1*N (small s1) | Alice gs1 = 1 + s1A*N
  std::vector<uint64_t> bs_ptr(2 * (size_t)P), bn_ptr(2 * (size_t)P);
  for (uint32_t p = 0; p < P; ++p) {
    const uint32_t i = p % n;
    bs_ptr[p] = DI(o_ps1 + (size_t)p * b->s1l * 4);
    bs_ptr[P + p] = DI(o_as1 + (size_t)p * b->s1l * 4);
    bn_ptr[p] = bn_ptr[P + p] = DI(o_rn + (size_t)i * nl * 4);
  }
  const size_t d_bs = L.in_vecT(bs_ptr), d_bn = L.in_vecT(bn_ptr);
  // inverse descriptors: nn: c^eA (Alice; also the PDL unit test of c when eA != 0) + c^e_pdl (eA == 0)
  std::vector<uint64_t> inv_y_nn, inv_m_nn, inv_y_nl, inv_m_nl;
  std::vector<uint32_t>& cpdl_extra = pl.cpdl_extra;  // pairs whose PDL c unit test needs its own inverse
  cpdl_extra.clear();
  for (uint32_t p = 0; p < P; ++p) {
    inv_y_nn.push_back(DX(x_J2 + ((size_t)P + p) * nn * 4));
    inv_m_nn.push_back(DI(o_NN + (size_t)(p % n) * nn * 4));
  }
  for (uint32_t p = 0; p < P; ++p)
    if (ae_bits[p] == 0 || !alice_pre[p]) {  // c^eA does not witness c's unit-ness
      inv_y_nn.push_back(DX(x_J2 + (size_t)p * nn * 4));
      inv_m_nn.push_back(DI(o_NN + (size_t)(p % n) * nn * 4));
      cpdl_extra.push_back(p);
    }
  for (uint32_t p = 0; p < P; ++p) {  // zA^eA (value) then z^e_pdl (unit test)
    inv_y_nl.push_back(DX(x_J5 + ((size_t)P + p) * nl * 4));
    inv_m_nl.push_back(DI(o_rt + (size_t)(p % n) * nl * 4));
  }
  for (uint32_t p = 0; p < P; ++p) {
    inv_y_nl.push_back(DX(x_J5 + (size_t)p * nl * 4));
    inv_m_nl.push_back(DI(o_rt + (size_t)(p % n) * nl * 4));
  }
  const size_t d_iynn = L.in_vecT(inv_y_nn), d_imnn = L.in_vecT(inv_m_nn);
  const size_t d_iynl = L.in_vecT(inv_y_nl), d_imnl = L.in_vecT(inv_m_nl);
  // eq_check descriptors
  std::vector<EqOperand> eq_nn, eq_nl;
  std::vector<uint32_t> eq_nn_mod, eq_nl_mod;
  std::vector<uint32_t> j9_index(P, 0xFFFFFFFFu);
  for (size_t k = 0; k < j9_pairs.size(); ++k) j9_index[j9_pairs[k]] = (uint32_t)k;
  for (uint32_t p = 0; p < P; ++p) {  // PDL u2: (N+1)^s1 * s2^N == u2 * c^e  (mod N^2), u2 < N^2
    EqOperand e;
    e.a = pdl_small[p] ? DX(x_Bpdl + (size_t)p * nn * 4) : DX(x_J9 + (size_t)j9_index[p] * nn * 4);
    e.a_len = nn;
    e.b = DX(x_J1 + (size_t)p * nn * 4);
    e.b_len = nn;
    e.c = DI(o_pu2 + (size_t)p * nn * 4);
    e.c_len = nn;
    e.d = DX(x_J2 + (size_t)p * nn * 4);
    e.d_len = nn;
    e.sel = 0xFFFFFFFFu;
    e.flags = 1;
    eq_nn.push_back(e);
    eq_nn_mod.push_back(p % n);
  }
  for (uint32_t p = 0; p < P; ++p) {  // PDL u3: h1^s1 * h2^s3 == u3 * z^e  (mod N~), u3 < N~
    EqOperand e;
    e.a = DX(x_J3 + (size_t)p * nl * 4);
    e.b = DX(x_J4 + (size_t)p * nl * 4);
    e.c = DI(o_pu3 + (size_t)p * nl * 4);
    e.d = DX(x_J5 + (size_t)p * nl * 4);
    e.a_len = e.b_len = e.c_len = e.d_len = nl;
    e.sel = 0xFFFFFFFFu;
    e.flags = 1;
    eq_nl.push_back(e);
    eq_nl_mod.push_back(p % n);
  }
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < M; ++k) {  // RP: T^Z_k == A_k * S^(e_k)  (mod N)
      EqOperand e;
      e.a = DX(x_RP + ((size_t)m * M + k) * nl * 4);
      e.b = DI(o_one);
      e.c = DI(o_pA + ((size_t)m * M + k) * nl * 4);
      e.d = DI(o_pS + (size_t)m * nl * 4);
      e.a_len = e.b_len = e.c_len = e.d_len = nl;
      e.sel = m * M + k;
      e.flags = 0;
      eq_nl.push_back(e);
      eq_nl_mod.push_back(n + m);
    }
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < CK_M2; ++k) {  // correct key: sigma^n == rho (mod n)
      EqOperand e;
      e.a = DX(x_J6 + ((size_t)m * CK_M2 + k) * nl * 4);
      e.b = DI(o_one);
      e.c = DI(o_rho + ((size_t)m * CK_M2 + k) * nl * 4);
      e.d = DI(o_one);
      e.a_len = e.b_len = e.c_len = e.d_len = nl;
      e.sel = 0xFFFFFFFFu;
      e.flags = 0;
      eq_nl.push_back(e);
      eq_nl_mod.push_back(n + Mt + m);
    }
  for (uint32_t j = 0; j < J; ++j)
    for (int which = 0; which < 2; ++which) {  // DLog: g^y * ni^e == x (mod N), x < N
      EqOperand e;
      e.a = DX(x_J7 + ((size_t)2 * j + which) * nl * 4);
      e.b = DX(x_J8 + ((size_t)2 * j + which) * nl * 4);
      e.c = DI((which == 0 ? o_dx1 : o_dx2) + (size_t)j * nl * 4);
      e.d = DI(o_one);
      e.a_len = e.b_len = e.c_len = e.d_len = nl;
      e.sel = 0xFFFFFFFFu;
      e.flags = 1;
      eq_nl.push_back(e);
      eq_nl_mod.push_back(n + 2 * Mt + j);
    }
  const size_t d_eqnn = L.in_vecT(eq_nn), d_eqnnm = L.in_vecT(eq_nn_mod);
  const size_t d_eqnl = L.in_vecT(eq_nl), d_eqnlm = L.in_vecT(eq_nl_mod);
  // prod3 descriptors: u = gs1 * s^N * (c^e)^-1  (mod N^2) | w = h1^s1 * h2^s2 * (z^e)^-1 (mod N~)
  std::vector<Prod3Operand> p3_nn(P), p3_nl(P);
  std::vector<uint32_t> p3_mod(P);
  for (uint32_t p = 0; p < P; ++p) {
    p3_nn[p] = {DX(x_gs1 + (size_t)p * nn * 4), DX(x_J1 + ((size_t)P + p) * nn * 4), DX(x_invc + (size_t)p * nn * 4),
                nn, nn, nn, 0};
    p3_nl[p] = {DX(x_J3 + ((size_t)P + p) * nl * 4), DX(x_J4 + ((size_t)P + p) * nl * 4),
                DX(x_invz + (size_t)p * nl * 4), nl, nl, nl, 0};
    p3_mod[p] = p % n;
  }
  const size_t d_p3nn = L.in_vecT(p3_nn), d_p3nl = L.in_vecT(p3_nl), d_p3m = L.in_vecT(p3_mod);
  // alice hash descriptors + pre-verdicts
  std::vector<uint64_t> ah_n(P), ah_c(P);
  for (uint32_t p = 0; p < P; ++p) {
    ah_n[p] = DI(o_rn + (size_t)(p % n) * nl * 4);
    ah_c[p] = DI(o_enc + (size_t)p * nn * 4);
  }
  const size_t d_ahn = L.in_vecT(ah_n), d_ahc = L.in_vecT(ah_c);
  const size_t d_alpre = L.in_vecT(alice_pre);
  if (Layout::al(L.host.size()) > Layout::al(in_bytes_pre + desc_bound)) {
    c->fail("internal: descriptor bound exceeded");
    return FSDKR_E_ARG;
  }
  // fixed-base scratch (power tables, schedules, step counts): its own context buffer
  {
    const int KD = shape_digits(nl);
    const size_t tb = Layout::al(FB.table_bytes(KD)), sb = Layout::al(FB.sched_bytes());
    uint8_t* fbs = (uint8_t*)c->buf("collect_fb", tb + sb + FB.nsteps_bytes() + 256);
    if (!fbs) {
      c->fail("fsdkr_verify_collect: fixed-base scratch allocation failed");
      return FSDKR_E_OOM;
    }
    pl.fb_table = (uint32_t*)fbs;
    pl.fb_sched = (uint16_t*)(fbs + tb);
    pl.fb_nsteps = (uint32_t*)(fbs + tb + sb);
  }
  pl.d_FB = d_FB;

  // ---------------- record the plan and upload the image (the only host->device copy)
  pl.el = b->el;
  pl.t = b->t;
  pl.s1l = b->s1l;
  pl.n_mods_nl = n_mods_nl;
  pl.in_bytes = L.host.size();
  pl.out_off = Layout::al(in_bytes_pre + desc_bound);
  pl.total = total;
  pl.dev = dev;
  pl.o_Q = o_Q; pl.o_enc = o_enc; pl.o_pz = o_pz; pl.o_pu1 = o_pu1; pl.o_pu2 = o_pu2; pl.o_pu3 = o_pu3;
  pl.o_ps1 = o_ps1; pl.o_pA = o_pA; pl.o_az = o_az; pl.o_ae = o_ae; pl.o_vss = o_vss; pl.o_NN = o_NN;
  pl.o_mods = o_mods; pl.o_one = o_one; pl.o_rn = o_rn;
  pl.x_epdl = x_epdl; pl.x_pbits = x_pbits; pl.x_ppanic = x_ppanic; pl.x_Bpdl = x_Bpdl; pl.x_gs1 = x_gs1;
  // launch order = stream assignment in collect_run: GA, GD (long), J2, J5 (short, feed the inverses)
  const size_t xs[4] = {x_GA, x_GD, x_J2, x_J5};
  const size_t ds[4] = {d_GA, d_GD, d_J2, d_J5};
  const ModexpJob* js[4] = {&GA, &GD, &J2, &J5};
  for (int k = 0; k < 4; ++k) {
    pl.x_J[k] = xs[k];
    pl.d_J[k] = ds[k];
    pl.jk32[k] = js[k]->k32;
    pl.jcount[k] = (uint32_t)js[k]->size();
    pl.jbits[k] = js[k]->exp_bits;
  }
  pl.x_invc = x_invc; pl.x_invz = x_invz; pl.x_unn = x_unn; pl.x_uzA = x_uzA; pl.x_uzp = x_uzp;
  pl.x_eq2 = x_eq2; pl.x_eq3 = x_eq3; pl.x_u = x_u; pl.x_w = x_w; pl.x_fel = x_fel; pl.x_pdlv = x_pdlv;
  pl.x_rng = x_rng;
  pl.d_bs = d_bs; pl.d_bn = d_bn; pl.d_iynn = d_iynn; pl.d_imnn = d_imnn; pl.d_iynl = d_iynl; pl.d_imnl = d_imnl;
  pl.d_eqnn = d_eqnn; pl.d_eqnnm = d_eqnnm; pl.d_eqnl = d_eqnl; pl.d_eqnlm = d_eqnlm; pl.d_p3nn = d_p3nn;
  pl.d_p3nl = d_p3nl; pl.d_p3m = d_p3m; pl.d_ahn = d_ahn; pl.d_ahc = d_ahc; pl.d_alpre = d_alpre;
  pl.n_inv_nn = (uint32_t)inv_y_nn.size();
  pl.n_eq_nn = (uint32_t)eq_nn.size();
  pl.n_eq_nl = (uint32_t)eq_nl.size();
  int rc = c->hip_check(hipMemcpyAsync(dev, L.host.data(), L.host.size(), hipMemcpyHostToDevice, c->stream),
                        "H2D batch");
  if (rc) return rc;
  return c->hip_check(hipStreamSynchronize(c->stream), "sync H2D");
}

// Kernel pipeline on the prepared (device-resident) batch; writes verdicts.
int collect_run(Ctx* c, fsdkr_verdicts* v) {
  CollectPlan* plan = reinterpret_cast<CollectPlan*>(c->plan);
  if (!plan) {
    c->fail("fsdkr_collect_run: no prepared batch");
    return FSDKR_E_ARG;
  }
  CollectPlan& pl = *plan;
  const Sizes& s = pl.s;
  const uint32_t nl = s.nl, nn = s.nn, P = s.P, n = s.n, Mt = s.Mt, M = s.M, J = s.J;
  uint8_t* dev = pl.dev;
  uint8_t* const out_base = dev + pl.out_off;
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };
  auto PX = [&](size_t o) { return (uint32_t*)(out_base + o); };
  auto PI = [&](size_t o) { return (const uint32_t*)(dev + o); };
  const size_t o_Q = pl.o_Q, o_enc = pl.o_enc, o_pz = pl.o_pz, o_pu1 = pl.o_pu1, o_pu2 = pl.o_pu2, o_pu3 = pl.o_pu3;
  const size_t o_ps1 = pl.o_ps1, o_pA = pl.o_pA, o_az = pl.o_az, o_ae = pl.o_ae, o_vss = pl.o_vss, o_NN = pl.o_NN;
  const size_t o_mods = pl.o_mods, o_one = pl.o_one;
  const size_t x_epdl = pl.x_epdl, x_pbits = pl.x_pbits, x_ppanic = pl.x_ppanic, x_Bpdl = pl.x_Bpdl, x_gs1 = pl.x_gs1;
  const size_t x_invc = pl.x_invc, x_invz = pl.x_invz, x_unn = pl.x_unn, x_uzA = pl.x_uzA, x_uzp = pl.x_uzp;
  const size_t x_eq2 = pl.x_eq2, x_eq3 = pl.x_eq3, x_u = pl.x_u, x_w = pl.x_w, x_fel = pl.x_fel, x_pdlv = pl.x_pdlv;
  const size_t x_rng = pl.x_rng;
  const size_t d_bs = pl.d_bs, d_bn = pl.d_bn, d_iynn = pl.d_iynn, d_imnn = pl.d_imnn, d_iynl = pl.d_iynl;
  const size_t d_imnl = pl.d_imnl, d_eqnn = pl.d_eqnn, d_eqnnm = pl.d_eqnnm, d_eqnl = pl.d_eqnl, d_eqnlm = pl.d_eqnlm;
  const size_t d_p3nn = pl.d_p3nn, d_p3nl = pl.d_p3nl, d_p3m = pl.d_p3m, d_ahn = pl.d_ahn, d_ahc = pl.d_ahc;
  const size_t d_alpre = pl.d_alpre;
  const uint32_t n_mods_nl = pl.n_mods_nl;
  const std::vector<uint32_t>& ae_bits = pl.ae_bits;
  const std::vector<uint32_t>& cpdl_extra = pl.cpdl_extra;
  const std::vector<uint8_t>& ck_pre = pl.ck_pre;
  const std::vector<uint8_t>& dlog_pre = pl.dlog_pre;
  (void)ae_bits;
  // ---------------- launch
  int rc;
  hipStream_t st = c->stream;
  // the alice pre-verdicts become the initial range verdicts
  if ((rc = c->hip_check(hipMemcpyAsync(out_base + x_rng, dev + d_alpre, P, hipMemcpyDeviceToDevice, st), "D2D")))
    return rc;
  // moduli constants
  uint32_t *cons_nn = nullptr, *cons_nl = nullptr;
  if ((rc = setup_moduli(c, nn, PI(o_NN), n, &cons_nn, "collect_nn"))) return rc;
  if ((rc = setup_moduli(c, nl, PI(o_mods), n_mods_nl, &cons_nl, "collect_nl"))) return rc;
  // GA lanes per instance: GA shares the chip with the other streams, so it takes
  // the largest group that keeps it within about half the resident lanes
  // (measured at n = 64: 8 lanes 64 ms/step vs 16 lanes 70 ms); small batches
  // (multi-GPU shards) get 16 or 32 lanes (KD = 160 constants) for latency.
  // FSDKR_COLLECT_GA_G overrides.
  const uint32_t ga_forced = [] {
    const char* e = getenv("FSDKR_COLLECT_GA_G");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  uint32_t ga_group = 8;
  for (uint32_t g : {16u, kWideGroup})
    if ((uint64_t)pl.jcount[0] * g <= 65536u) ga_group = g;
  if (ga_forced) ga_group = ga_forced;
  uint32_t* cons_nn_w = nullptr;
  if (ga_group == kWideGroup && nn == 128 && pl.jcount[0] &&
      (rc = setup_moduli(c, nn, PI(o_NN), n, &cons_nn_w, "collect_nn_w", kWideGroup)))
    return rc;
  if (ga_group == kWideGroup && nn != 128) ga_group = 16;
  // ---- stream plan (up to eleven concurrent lanes of work: give HIP >= 12 hardware
  //      queues, GPU_MAX_HW_QUEUES, or streams share queues and serialise):
  //   side 0  : GA (nn, long exponents, priority)               | start after mod_setup
  //   side 8  : FB table chains (h1, h2, T: the longest dependent chain), top priority
  //   side 1  : FB schedules, then (after the tables) fixed-base exponents
  //   side 7  : J5 + nl inverses instead of st when CUs are reserved (FSDKR_RESERVE_CUS)
  //   side 3  : ped_hash (serial SHA-256 chains, priority)
  //   side 4  : GD (nl: correct-key, DLog; priority)
  //   side 6  : Feldman (secp256k1 Horner per pair)
  //   st      : pdl_hash, binom x2 | fork | J5, nl inverses | join | eq, prod3, alice
  //   side 2  :                    J2 (nn, 256-bit challenges) -> nn inverses
  //   side 5  :                    pdl_u1 (secp256k1)
  std::vector<hipEvent_t> done;
  // issue-priority levels of the serial chains (tuning knob FSDKR_PRIO="GA,FB,GD,J5";
  // measured defaults)
  // (knobs are read per call so one process can A/B them: tools/ab_collect.py)
  uint32_t prio[4] = {3, 3, 2, 1};
  if (const char* e = getenv("FSDKR_PRIO")) sscanf(e, "%u,%u,%u,%u", &prio[0], &prio[1], &prio[2], &prio[3]);
  pl.fb.table_prio = prio[1];
  auto fork = [&](hipStream_t from, hipEvent_t* ev) -> int {
    int r = c->hip_check(hipEventCreateWithFlags(ev, hipEventDisableTiming), "event");
    if (!r) (void)hipEventRecord(*ev, from);
    return r;
  };
  auto join_later = [&](hipStream_t ss) -> int {
    hipEvent_t ev;
    int r = c->hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
    if (r) return r;
    (void)hipEventRecord(ev, ss);
    done.push_back(ev);
    return FSDKR_OK;
  };
  static const char* tags[4] = {"mxt_GA", "mxt_GD", "mxt_J2", "mxt_J5"};
  // prio: s_setprio level of the launch's waves (latency-critical chains); group: lanes per instance
  auto launch_group = [&](int k, hipStream_t ss, uint32_t prio, uint32_t group) -> int {
    if (!pl.jcount[k]) return FSDKR_OK;
    const uint32_t* cons = (pl.jk32[k] == nn) ? (group == kWideGroup ? cons_nn_w : cons_nn) : cons_nl;
    return launch_modexp_desc(c, pl.jk32[k], pl.jcount[k], pl.jbits[k], dev + pl.d_J[k], cons, PX(pl.x_J[k]), ss,
                              tags[k], prio, group);
  };
  // GA-first ordering (tuning knob FSDKR_GA_FIRST, bit mask): the throughput jobs
  // fb_exp (1), J2 (2) and J5 (4) wait for GA, so GA's ~1 wave per SIMD runs beside
  // only the few-wave chains
  const uint32_t ga_first = [] {
    const char* e = getenv("FSDKR_GA_FIRST");
    return e ? (uint32_t)atoi(e) : 0u;
  }();
  hipEvent_t ga_done = nullptr;
  // (1) chains that need only the inputs and the moduli constants start at once
  hipEvent_t consts_ready;
  if ((rc = fork(st, &consts_ready))) return rc;
  {  // GA: s2^N, s^N mod N^2 (4096-bit, 2048-bit exponents): the longest chains
    hipStream_t ss = c->side_stream(0);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    // small batches (multi-GPU shards): the h2 fixed-base table chain (2816
    // dependent squarings) is the critical path, so GA steps down one issue
    // priority level below it (8-way shard: 33.4 -> 31.7 ms, tools/ab_hwq.sh)
    if (ga_group >= 16 && !getenv("FSDKR_PRIO")) prio[0] = 2;
    if ((rc = launch_group(0, ss, prio[0], ga_group)) || (rc = join_later(ss))) return rc;
    if (ga_first && (rc = fork(ss, &ga_done))) return rc;
  }
  {  // FB: h1, h2, T fixed-base tables -> schedules -> exponents
    hipStream_t ss = c->side_stream(1);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    FbDev fd{dev + pl.d_FB, pl.fb_table, pl.fb_sched, pl.fb_nsteps};
    // the table chains (thousands of dependent squarings, few waves) run on the
    // reserved CUs when FSDKR_RESERVE_CUS is set
    hipStream_t ts = c->crit_stream();
    if (!ts) ts = c->side_stream(8);   // own stream: the chain starts beside fb_sched
    (void)hipStreamWaitEvent(ts, consts_ready, 0);
    if ((rc = fb_launch(c, pl.fb, fd, cons_nl, ss, "fb collect", ts, (ga_first & 1) ? ga_done : nullptr)) ||
        (rc = join_later(ss)))
      return rc;
  }
  {  // ring-Pedersen challenges: one serial SHA-256 chain per message, needed only by the final checks
    hipStream_t ss = c->side_stream(3);
    PedHashArgs h{PI(o_pA), M, nl, PX(x_pbits), PX(x_ppanic), Mt};
    c->mark("ped_hash", true, ss);
    rc = c->hip_check(launch_ped_hash(h, ss), "ped_hash");
    c->mark("ped_hash", false, ss);
    if (rc || (rc = join_later(ss))) return rc;
  }
  {  // Feldman share checks (inputs only; one Horner chain per pair)
    hipStream_t ss = c->side_stream(6);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    FeldmanArgs f{PI(o_vss), PI(o_Q), n, pl.t, (uint8_t*)(out_base + x_fel), P};
    c->mark("ec", true, ss);
    rc = c->hip_check(launch_feldman(f, ss), "feldman");
    c->mark("ec", false, ss);
    if (rc || (rc = join_later(ss))) return rc;
  }
  {  // GD: correct-key sigma^n, DLog g^y / ni^e (2048-bit exponents, few instances)
    hipStream_t ss = c->side_stream(4);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    if ((rc = launch_group(1, ss, prio[2], 0)) || (rc = join_later(ss))) return rc;
  }
  // (2) PDL challenges, then the jobs that exponentiate by them
  {
    PdlHashArgs a{PI(o_Q), PI(o_enc), PI(o_pz), PI(o_pu1), PI(o_pu2), PI(o_pu3), nn, nl, PX(x_epdl), P};
    c->mark("pdl_hash", true);
    rc = c->hip_check(launch_pdl_hash(a, st), "pdl_hash");
    c->mark("pdl_hash", false);
    if (rc) return rc;
  }
  {
    BinomArgs a{(const uint64_t*)(dev + d_bs), (const uint64_t*)(dev + d_bn), pl.s1l, nl, nn, PX(x_Bpdl), P};
    if ((rc = c->hip_check(launch_binom(a, st), "binom"))) return rc;
    BinomArgs a2{(const uint64_t*)(dev + d_bs) + P, (const uint64_t*)(dev + d_bn) + P, pl.s1l, nl, nn, PX(x_gs1), P};
    if ((rc = c->hip_check(launch_binom(a2, st), "binom"))) return rc;
  }
  hipEvent_t ready;
  if ((rc = fork(st, &ready))) return rc;
  {  // J2: c^e (4096-bit, 256-bit challenges) -> nn inverses
    hipStream_t ss = c->side_stream(2);
    (void)hipStreamWaitEvent(ss, ready, 0);
    if (ga_first & 2) (void)hipStreamWaitEvent(ss, ga_done, 0);
    if ((rc = launch_group(2, ss, 0, 8))) return rc;
    InverseArgs a{(const uint64_t*)(dev + d_iynn), (const uint64_t*)(dev + d_imnn), PX(x_invc), PX(x_unn),
                  nullptr, pl.n_inv_nn};
    c->mark("inverse", true, ss);
    rc = c->hip_check(launch_inverse(nn, a, ss), "inverse nn");
    c->mark("inverse", false, ss);
    if (rc || (rc = join_later(ss))) return rc;
  }
  {  // PDL u1 on secp256k1 (one Shamir ladder per pair, latency-bound) off the main chain
    hipStream_t ss = c->side_stream(5);
    (void)hipStreamWaitEvent(ss, ready, 0);
    PdlU1Args u{PI(o_ps1), PX(x_epdl), PI(o_Q), PI(o_pu1), pl.s1l, (uint8_t*)(out_base + x_pdlv), P};
    c->mark("ec", true, ss);
    rc = c->hip_check(launch_pdl_u1(u, ss), "pdl_u1");
    c->mark("ec", false, ss);
    if (rc) return rc;
    if ((rc = join_later(ss))) return rc;
  }
  (void)hipEventDestroy(consts_ready);
  (void)hipEventDestroy(ready);
  {  // J5: z^e (2048-bit, 256-bit challenges) -> nl inverses; a side stream when CUs are
     // reserved (the main stream is unmasked), else the main stream
    hipStream_t js = st;
    if (c->reserve_cus) {
      js = c->side_stream(7);
      hipEvent_t r2;
      if ((rc = fork(st, &r2))) return rc;
      (void)hipStreamWaitEvent(js, r2, 0);
      (void)hipEventDestroy(r2);
    }
    if (ga_first & 4) (void)hipStreamWaitEvent(js, ga_done, 0);
    if ((rc = launch_group(3, js, prio[3], 8))) return rc;
    InverseArgs b1{(const uint64_t*)(dev + d_iynl), (const uint64_t*)(dev + d_imnl), PX(x_invz), PX(x_uzA),
                   nullptr, P};
    c->mark("inverse", true, js);
    rc = c->hip_check(launch_inverse(nl, b1, js), "inverse nl");
    c->mark("inverse", false, js);
    if (rc) return rc;
    InverseArgs b2{(const uint64_t*)(dev + d_iynl) + P, (const uint64_t*)(dev + d_imnl) + P, nullptr, PX(x_uzp),
                   nullptr, P};
    if ((rc = c->hip_check(launch_inverse(nl, b2, js), "inverse nl 2"))) return rc;
    if (js != st && (rc = join_later(js))) return rc;
  }
  if (ga_done) (void)hipEventDestroy(ga_done);
  for (hipEvent_t ev : done) {
    (void)hipStreamWaitEvent(st, ev, 0);
    (void)hipEventDestroy(ev);
  }
  // equality checks and exact products
  {
    EqCheckArgs a{(const EqOperand*)(dev + d_eqnn), PI(d_eqnnm), cons_nn, PX(x_pbits), DI(o_one), PX(x_eq2),
                  pl.n_eq_nn};
    c->mark("eq_check", true);
    rc = c->hip_check(launch_eq_check(nn, a, st), "eq_check nn");
    c->mark("eq_check", false);
    if (rc) return rc;
    // eq_nl outputs: [u3 P | RP Mt*M | CK Mt*11 | DLog 2J] contiguous from x_eq3
    EqCheckArgs b1{(const EqOperand*)(dev + d_eqnl), PI(d_eqnlm), cons_nl, PX(x_pbits), DI(o_one), PX(x_eq3),
                   pl.n_eq_nl};
    c->mark("eq_check", true);
    rc = c->hip_check(launch_eq_check(nl, b1, st), "eq_check nl");
    c->mark("eq_check", false);
    if (rc) return rc;
    Prod3Args pa{(const Prod3Operand*)(dev + d_p3nn), PI(d_p3m), cons_nn, PX(x_u), P};
    if ((rc = c->hip_check(launch_prod3(nn, pa, st), "prod3 nn"))) return rc;
    Prod3Args pb{(const Prod3Operand*)(dev + d_p3nl), PI(d_p3m), cons_nl, PX(x_w), P};
    if ((rc = c->hip_check(launch_prod3(nl, pb, st), "prod3 nl"))) return rc;
  }
  {
    AliceHashArgs a{(const uint64_t*)(dev + d_ahn), (const uint64_t*)(dev + d_ahc), PI(o_az), PX(x_u), PX(x_w),
                    PI(o_ae), nl, nn, nl, pl.el, (uint8_t*)(out_base + x_rng), P};
    c->mark("alice_hash", true);
    rc = c->hip_check(launch_alice_hash(a, st), "alice_hash");
    c->mark("alice_hash", false);
    if (rc) return rc;
  }
  // ---------------- results
  std::vector<uint32_t> e_pdl((size_t)P * 8), ppanic(Mt), unn(2 * (size_t)P), uzA(P), uzp(P), eq2(P),
      eq_nl_res(pl.n_eq_nl);
  std::vector<uint8_t> fel(P), pdlv(P), rng(P);
  auto D2H = [&](void* dst, size_t off, size_t bytes) {
    return c->hip_check(hipMemcpyAsync(dst, out_base + off, bytes, hipMemcpyDeviceToHost, st), "D2H verdicts");
  };
  if ((rc = D2H(e_pdl.data(), x_epdl, e_pdl.size() * 4)) || (rc = D2H(ppanic.data(), x_ppanic, Mt * 4)) ||
      (rc = D2H(unn.data(), x_unn, (size_t)pl.n_inv_nn * 4)) || (rc = D2H(uzA.data(), x_uzA, P * 4)) ||
      (rc = D2H(uzp.data(), x_uzp, P * 4)) || (rc = D2H(eq2.data(), x_eq2, P * 4)) ||
      (rc = D2H(eq_nl_res.data(), x_eq3, eq_nl_res.size() * 4)) || (rc = D2H(fel.data(), x_fel, P)) ||
      (rc = D2H(pdlv.data(), x_pdlv, P)) || (rc = D2H(rng.data(), x_rng, P)))
    return rc;
  if ((rc = c->sync())) return rc;
  // PDL unit test of c: c^eA witnesses it unless eA == 0 / the Alice proof was rejected early
  std::vector<uint32_t> unit_c_pdl(unn.begin(), unn.begin() + P);
  for (size_t k = 0; k < cpdl_extra.size(); ++k) unit_c_pdl[cpdl_extra[k]] = unn[P + k];
  const uint32_t* u_cA = unn.data();
  const uint32_t* u_zA = uzA.data();
  const uint32_t* u_zp = uzp.data();
  for (uint32_t p = 0; p < P; ++p) {
    bool ez = true;
    for (int k = 0; k < 8; ++k) ez = ez && e_pdl[(size_t)p * 8 + k] == 0;
    // reference panics (mod_inv(..).unwrap(), zk_pdl_with_slack.rs:180) when e != 0 and c or z is not a unit
    const bool cunit = unit_c_pdl[p] != 0;
    const bool panic = !ez && (!cunit || !u_zp[p]);
    uint8_t bits = (uint8_t)(pdlv[p] & 1u);
    if (eq2[p]) bits |= 2;
    if (eq_nl_res[p]) bits |= 4;
    if (panic) bits |= 8;
    v->pdl[p] = bits;
    v->feldman[p] = fel[p] ? 1 : 0;
    // Alice: pre-checks, invertibility of z^e and c^e, transcript hash (range_proofs.rs:125-163)
    v->range[p] = (rng[p] && u_cA[p] && u_zA[p]) ? 1 : 0;
  }
  for (uint32_t m = 0; m < Mt; ++m) {
    v->ped[m] = ped_verdict(&eq_nl_res[P + (size_t)m * M], M, ppanic[m]);
    bool ck = ck_pre[m];
    for (uint32_t k = 0; k < CK_M2; ++k) ck = ck && eq_nl_res[P + (size_t)Mt * M + (size_t)m * CK_M2 + k];
    v->ck[m] = ck ? 1 : 0;
  }
  for (uint32_t j = 0; j < J; ++j) {
    const size_t base = P + (size_t)Mt * M + (size_t)Mt * CK_M2 + 2 * j;
    uint8_t d = 0;
    if (dlog_pre[j] && eq_nl_res[base]) d |= 1;
    if (dlog_pre[j] && eq_nl_res[base + 1]) d |= 2;
    v->dlog[j] = d;
  }
  return FSDKR_OK;
}


int verify_collect_impl(Ctx* c, const fsdkr_collect_batch* b, fsdkr_verdicts* v) {
  int rc = collect_prepare(c, b);
  if (rc) return rc;
  return collect_run(c, v);
}

int first_error_impl(const fsdkr_collect_batch* b, const fsdkr_verdicts* v, fsdkr_error* e) {
  memset(e, 0, sizeof *e);
  const uint32_t R = b->n_refresh, J = b->n_join, n = R + J;
  // validate_collect (refresh_message.rs:147-191)
  if (R <= b->t) {
    e->variant = FSDKR_ERR_PARTIES_THRESHOLD_VIOLATION;
    e->f[0] = b->t;
    e->f[1] = R;
    return FSDKR_OK;
  }
  if (b->msg_lens) {
    const uint32_t ref = b->msg_lens[0];
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t* l = b->msg_lens + 3 * (size_t)k;
      if (!(l[0] == ref && l[1] == ref && l[2] == ref)) {
        e->variant = FSDKR_ERR_SIZE_MISMATCH;
        e->f[0] = k;
        e->f[1] = l[0];
        e->f[2] = l[1];
        e->f[3] = l[2];
        return FSDKR_OK;
      }
    }
    if (ref < n) {  // points_committed_vec[i] indexed past its end (:182)
      e->panic = 1;
      e->variant = FSDKR_ERR_PUBLIC_SHARE_VALIDATION;
      return FSDKR_OK;
    }
  }
  if (!v) return FSDKR_E_ARG;
  for (uint32_t k = 0; k < R; ++k)
    for (uint32_t i = 0; i < n; ++i)
      if (!v->feldman[(size_t)k * n + i]) {
        e->variant = FSDKR_ERR_PUBLIC_SHARE_VALIDATION;
        return FSDKR_OK;
      }
  // PDL then range, per (k, i)  (:330-350)
  for (uint32_t k = 0; k < R; ++k)
    for (uint32_t i = 0; i < n; ++i) {
      const uint8_t d = v->pdl[(size_t)k * n + i];
      if (d & 8) {
        e->panic = 1;
        e->variant = FSDKR_ERR_PDL_W_SLACK_PROOF;
        return FSDKR_OK;
      }
      if ((d & 7) != 7) {
        e->variant = FSDKR_ERR_PDL_W_SLACK_PROOF;
        e->f[0] = d & 1;
        e->f[1] = (d >> 1) & 1;
        e->f[2] = (d >> 2) & 1;
        return FSDKR_OK;
      }
      if (!v->range[(size_t)k * n + i]) {
        e->variant = FSDKR_ERR_RANGE_PROOF;
        e->f[0] = i;
        return FSDKR_OK;
      }
    }
  // ring-Pedersen: refresh then join (:353-365)
  for (uint32_t m = 0; m < R + J; ++m) {
    if (v->ped[m] & 2) {
      e->panic = 1;
      e->variant = FSDKR_ERR_RING_PEDERSEN_PROOF;
      return FSDKR_OK;
    }
    if (!(v->ped[m] & 1)) {
      e->variant = FSDKR_ERR_RING_PEDERSEN_PROOF;
      return FSDKR_OK;
    }
  }
  // correct key + modulus size per refresh message (:375-396)
  for (uint32_t m = 0; m < R; ++m) {
    const uint32_t pi = b->party_index[m];
    if (!v->ck[m]) {
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    const uint32_t bits = hbn::bitlen(b->ck_n + (size_t)m * b->nl, b->nl);
    if (bits > b->key_bits || bits < b->key_bits - 1) {
      e->variant = FSDKR_ERR_MODULI_TOO_SMALL;
      e->f[0] = pi;
      e->f[1] = bits;
      return FSDKR_OK;
    }
    e->keys_applied = m + 1;
  }
  // joins (:398-437)
  for (uint32_t j = 0; j < J; ++j) {
    const uint32_t pi = b->party_index[R + j];
    if (pi == 0) {
      e->variant = FSDKR_ERR_NEW_PARTY_UNASSIGNED_INDEX;
      return FSDKR_OK;
    }
    if (!v->ck[R + j]) {
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    if ((v->dlog[j] & 3) != 3) {
      e->variant = FSDKR_ERR_DLOG_PROOF_VALIDATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    const uint32_t bits = hbn::bitlen(b->ck_n + (size_t)(R + j) * b->nl, b->nl);
    if (bits > b->key_bits || bits < b->key_bits - 1) {
      e->variant = FSDKR_ERR_MODULI_TOO_SMALL;
      e->f[0] = pi;
      e->f[1] = bits;
      return FSDKR_OK;
    }
    e->keys_applied = R + j + 1;
  }
  e->variant = FSDKR_ERR_NONE;
  return FSDKR_OK;
}

}  // namespace fsdkr

extern "C" {

int fsdkr_verify_collect(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch, fsdkr_verdicts* out) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c || !batch || !out || !out->feldman || !out->pdl || !out->range || !out->ped || !out->ck ||
      (batch->n_join && !out->dlog))
    return FSDKR_E_ARG;
  return fsdkr::verify_collect_impl(c, batch, out);
}

int fsdkr_collect_prepare(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c || !batch) return FSDKR_E_ARG;
  return fsdkr::collect_prepare(c, batch);
}

int fsdkr_collect_run(fsdkr_ctx* ctx, fsdkr_verdicts* out) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c || !out || !out->feldman || !out->pdl || !out->range || !out->ped || !out->ck) return FSDKR_E_ARG;
  return fsdkr::collect_run(c, out);
}

int fsdkr_collect_first_error(const fsdkr_collect_batch* batch, const fsdkr_verdicts* verdicts, fsdkr_error* out) {
  if (!batch || !out) return FSDKR_E_ARG;
  return fsdkr::first_error_impl(batch, verdicts, out);
}

}  // extern "C"
