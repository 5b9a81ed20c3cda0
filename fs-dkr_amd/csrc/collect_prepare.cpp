// fsdkr_collect_prepare[_multi]: the host pre-pass of one or many collect()
// sessions (bounds, bit lengths, PDL challenges, correct-key rho_j, DLog
// challenges, even-modulus splits) and the ONE device image every kernel of the
// pipeline reads: the sessions' pairs, receivers, messages and joins
// concatenated at the widest limb widths, descriptors addressing its rows,
// uploaded with one H2D from a pinned arena.
#include "collect.hpp"

namespace fsdkr {


// ------------------------------------------------------------------------------
int collect_prepare_impl(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count) {
  free_collect_plan(c);   // a failed prepare leaves no plan behind
  c->reuse_mask = 0;
  if (!bs || count == 0) {
    c->fail("fsdkr_collect_prepare: no batch");
    return FSDKR_E_ARG;
  }
  std::unique_ptr<CollectPlan> plan(new CollectPlan());
  CollectPlan& pl = *plan;
  PhaseClock clk;
  // ---------------- shapes
  uint32_t nl = 0, s1l = 0, s3l = 0, el = 0, zl = 0, yl = 1, ckl = 0, M = 0;
  pl.ss.resize(count);
  uint32_t n = 0, P = 0, Mt = 0, J = 0, V = 0;
  for (uint32_t s = 0; s < count; ++s) {
    const fsdkr_collect_batch* b = bs + s;
    Sess& x = pl.ss[s];
    x.b = b;
    x.R = b->n_refresh;
    x.J = b->n_join;
    x.n = b->n_recv ? b->n_recv : x.R + x.J;
    x.Mt = x.R + x.J;
    x.P = x.R * x.n;
    x.ckl = b->ckl ? b->ckl : b->nl;
    if (x.n < x.R || x.n == 0 || b->m_security == 0 || !(b->nl == 64 || b->nl == 96) || b->s1l == 0 ||
        b->s3l == 0 || b->el == 0 || b->zl == 0 || (x.J && b->yl == 0) || !shape_digits(x.ckl) || x.ckl < b->nl ||
        (M && b->m_security != M) || !b->party_index) {
      c->fail("fsdkr_collect_prepare: session %u: unsupported shape (R=%u J=%u n=%u nl=%u ckl=%u M=%u)", s, x.R, x.J,
              x.n, b->nl, x.ckl, b->m_security);
      return FSDKR_E_UNSUPPORTED;
    }
    M = b->m_security;
    // the receivers' own keys (LocalKey state, not message data) must be odd for Montgomery
    for (uint32_t i = 0; i < x.n; ++i)
      if (!is_odd(b->recv_n + (size_t)i * b->nl) || !is_odd(b->recv_ntilde + (size_t)i * b->nl)) {
        c->fail("session %u receiver %u: even Paillier or DLog modulus in the LocalKey (unsupported)", s, i);
        return FSDKR_E_UNSUPPORTED;
      }
    x.V = 0;
    for (uint32_t k = 0; k < x.R; ++k) x.V += ncoef_of(b, k);
    x.rbase = n;
    x.mbase = Mt;
    x.jbase = J;
    x.pbase = P;
    x.vbase = V;
    n += x.n;
    Mt += x.Mt;
    J += x.J;
    P += x.P;
    V += x.V;
    nl = std::max(nl, b->nl);
    s1l = std::max(s1l, b->s1l);
    s3l = std::max(s3l, b->s3l);
    el = std::max(el, b->el);
    zl = std::max(zl, b->zl);
    if (x.J) yl = std::max(yl, b->yl);
    ckl = std::max(ckl, x.ckl);
  }
  const uint32_t nn = 2 * nl;
  pl.S = count;
  pl.n = n;
  pl.P = P;
  pl.Mt = Mt;
  pl.J = J;
  pl.M = M;
  pl.nl = nl;
  pl.nn = nn;
  pl.ckl = ckl;
  pl.s1l = s1l;
  pl.el = el;
  const uint32_t MW = (M + 31) / 32;
  // global index -> session
  std::vector<uint32_t> sess_of_pair(P), sess_of_recv(n), sess_of_msg(Mt), sess_of_join(J);
  for (uint32_t s = 0; s < count; ++s) {
    const Sess& x = pl.ss[s];
    std::fill(sess_of_pair.begin() + x.pbase, sess_of_pair.begin() + x.pbase + x.P, s);
    std::fill(sess_of_recv.begin() + x.rbase, sess_of_recv.begin() + x.rbase + x.n, s);
    std::fill(sess_of_msg.begin() + x.mbase, sess_of_msg.begin() + x.mbase + x.Mt, s);
    std::fill(sess_of_join.begin() + x.jbase, sess_of_join.begin() + x.jbase + x.J, s);
  }
  std::vector<uint32_t> recv_of_pair(P);   // global receiver row of each pair
  for (uint32_t p = 0; p < P; ++p) {
    const Sess& x = pl.ss[sess_of_pair[p]];
    recv_of_pair[p] = x.rbase + (p - x.pbase) % x.n;
  }
  // pairs whose PDL s3 is negative (pdl_s3 holds |s3|): u3 is checked as
  // h1^s1 == u3 * (z^e * h2^|s3|), the bracket an extra exact product row
  std::vector<uint32_t> neg3;
  for (const Sess& x : pl.ss)
    if (x.b->pdl_s3_neg)
      for (uint32_t lp = 0; lp < x.P; ++lp)
        if (x.b->pdl_s3_neg[lp]) neg3.push_back(x.pbase + lp);
  const size_t K3 = neg3.size();
  // a prestarted GA of this batch: J1 is not launched again
  pl.ga_hit = ga_pre_matches(c, bs, count);
  GaPre* gpre = reinterpret_cast<GaPre*>(c->ga_pre);
  if (pl.ga_hit) {
    pl.ga_done = gpre->done;
    pl.ga_setup = gpre->ga_setup;
    pl.pre_cons_nn = gpre->cons;
    pl.pre_cons_wide = gpre->wide;
    gpre->valid = false;   // consumed (the buffer lives until the next prestart)
  }
  // GA's joint tail: the prestart ran the split head (gpre->split), or prepare's own GA
  // (J1 alone, padded to whole waves) takes a sliding-window shape
  {
    const uint32_t g0 = ga_lanes(2 * P, nn);
    pl.joint = pl.ga_hit ? gpre->split : ga_split_ok(nn, g0, ga_desc_flags(true, g0));
  }
  if (pl.joint && pl.ga_hit)
    pl.ga_tail = CollectPlan::GaTail{gpre->ga_desc, gpre->cons, gpre->out, gpre->ga_count, gpre->ga_bits, gpre->ga_group,
                                     gpre->ga_flags};
  clk.lap("shapes");

  // ---------------- host pre-pass (O(n) + O(P) scans, no big exponentiations; threaded)
  std::vector<uint32_t> NN((size_t)n * nn), NP1((size_t)n * nn), recv_bits(n);
  parallel_for(n, 64, [&](size_t b0, size_t b1) {
    for (size_t r = b0; r < b1; ++r) {
      const Sess& x = pl.ss[sess_of_recv[r]];
      const uint32_t* Np = x.b->recv_n + (size_t)(r - x.rbase) * x.b->nl;
      hbn::Limbs N = hbn::from(Np, x.b->nl);
      hbn::store(hbn::mul(N, N), NN.data() + r * nn, nn);
      hbn::store(hbn::add_small(N, 1), NP1.data() + r * nn, nn);
      recv_bits[r] = hbn::bitlen(Np, x.b->nl);
    }
  });
  const hbn::Limbs& q3 = q_cubed();
  std::vector<uint8_t> alice_pre(P), pdl_small(P), big_c(P);
  std::vector<uint32_t> ae_bits(P);
  struct Maxes {
    uint32_t s1 = 1, s3 = 1, as1 = 1, as2 = 1, ae = 1;
    bool big_s1 = false;
  };
  std::vector<Maxes> tmax(host_threads() + 1);
  std::atomic<uint32_t> slot{0};
  // PDL challenges e = H(G, Q, c, z, u1, u2, u3) (zk_pdl_with_slack.rs:114-122) on the
  // host threads of this scan: J2 (c^e), J5 (z^e) and pdl_u1 can start with the pipeline
  std::vector<uint32_t>& EPDL = pl.e_pdl;
  EPDL.assign((size_t)P * 8, 0u);
  std::atomic<bool> sha_fail{false};
  parallel_for(P, 256, [&](size_t b0, size_t b1) {
    Maxes mx;
    HostSha sha;
    for (size_t p = b0; p < b1; ++p) {
      const Sess& x = pl.ss[sess_of_pair[p]];
      const fsdkr_collect_batch* b = x.b;
      const size_t lp = p - x.pbase;
      if (!pdl_challenge(sha, b, lp, EPDL.data() + p * 8)) sha_fail = true;
      // a ciphertext at or above N^2 (GMP reduces it; the joint tail's inverse needs it reduced)
      // (or a negative one, neg_bits bit 2: enc holds |c|, the arithmetic takes -|c| mod N^2)
      big_c[p] = hbn::cmp_raw(b->enc + lp * 2 * b->nl, 2 * b->nl, NN.data() + (size_t)recv_of_pair[p] * nn, nn) >= 0 ||
                 (b->neg_bits && (b->neg_bits[lp] & 4));
      const uint32_t* Np = b->recv_n + (size_t)(lp % x.n) * b->nl;
      const uint32_t* s1 = b->pdl_s1 + lp * b->s1l;
      // s1 < N -> (N+1)^s1 mod N^2 = 1 + s1*N  (binomial, bit-identical)
      const bool small = hbn::cmp_raw(s1, b->s1l, Np, b->nl) < 0;
      pdl_small[p] = small ? 1 : 0;
      mx.big_s1 = mx.big_s1 || !small;
      mx.s1 = std::max(mx.s1, hbn::bitlen(s1, b->s1l));
      mx.s3 = std::max(mx.s3, hbn::bitlen(b->pdl_s3 + lp * b->s3l, b->s3l));
      const uint32_t* as1 = b->rp_s1 + lp * b->s1l;
      ae_bits[p] = hbn::bitlen(b->rp_e + lp * b->el, b->el);
      const bool s1_ok = hbn::cmp_raw(as1, b->s1l, q3.data(), q3.size()) <= 0;
      alice_pre[p] = (s1_ok && ae_bits[p] <= 256) ? 1 : 0;
      if (alice_pre[p]) {  // exponents of rejected proofs are never used
        mx.as1 = std::max(mx.as1, hbn::bitlen(as1, b->s1l));
        mx.as2 = std::max(mx.as2, hbn::bitlen(b->rp_s2 + lp * b->s3l, b->s3l));
        mx.ae = std::max(mx.ae, ae_bits[p]);
      }
    }
    tmax[slot++ % tmax.size()] = mx;   // at most host_threads() chunks
  });
  Maxes mx;
  for (const Maxes& t : tmax) {
    mx.s1 = std::max(mx.s1, t.s1);
    mx.s3 = std::max(mx.s3, t.s3);
    mx.as1 = std::max(mx.as1, t.as1);
    mx.as2 = std::max(mx.as2, t.as2);
    mx.ae = std::max(mx.ae, t.ae);
    mx.big_s1 = mx.big_s1 || t.big_s1;
  }
  clk.lap("pair scan + PDL challenges");
  // c mod N^2 of the ciphertexts at or above N^2 (the joint tail's inverse needs it
  // reduced) and -|c| mod N^2 of the negative ones (every use but the hashes)
  std::vector<uint32_t> RC;
  if (std::find(big_c.begin(), big_c.end(), 1) != big_c.end()) {
    RC.assign((size_t)P * nn, 0u);
    parallel_for(P, 64, [&](size_t b0, size_t b1) {
      for (size_t p = b0; p < b1; ++p) {
        if (!big_c[p]) continue;
        const Sess& x = pl.ss[sess_of_pair[p]];
        const size_t lp = p - x.pbase;
        const hbn::Limbs cc = hbn::from(x.b->enc + lp * 2 * x.b->nl, 2 * x.b->nl);
        const hbn::Limbs NNr = hbn::from(NN.data() + (size_t)recv_of_pair[p] * nn, nn);
        hbn::Limbs v = hbn::mod(cc, NNr);
        if (x.b->neg_bits && (x.b->neg_bits[lp] & 4) && !v.empty()) v = hbn::sub(NNr, v);
        hbn::store(v, RC.data() + p * nn, nn);
      }
    });
  }
  pl.ae_zero.assign(P, 0);
  for (uint32_t p = 0; p < P; ++p) pl.ae_zero[p] = ae_bits[p] == 0;
  if (sha_fail) {
    c->fail("fsdkr_collect_prepare: SHA-256 (OpenSSL EVP) failed");
    return FSDKR_E_ARG;
  }
  // correct-key: rho_j = mask_generation(len(n), H(n, salt, j)) mod n; primorial gcd.
  // ring-Pedersen modulus split N = 2^k m (even N: 2-adic half in pow2.hip); S mod m.
  std::vector<uint32_t> RHO((size_t)Mt * CK_M2 * ckl, 0u), CKMODS((size_t)Mt * ckl, 0u), CKEXP((size_t)Mt * ckl, 0u),
      ck_bits(Mt);
  std::vector<uint32_t> PEDN((size_t)Mt * nl, 0u), PEDS((size_t)Mt * nl, 0u), ped_tz(Mt, 0u);
  pl.ck_pre.assign(Mt, 0);
  pl.ped_mode.assign(Mt, 0);
  pl.ped_zlen.assign(Mt, M);
  pl.ck_short.assign(Mt, 0);
  pl.ck_one.assign(Mt, 0);
  for (uint32_t m = 0; m < Mt; ++m) {
    const Sess& x = pl.ss[sess_of_msg[m]];
    const uint32_t lm = m - x.mbase;
    if (x.b->ped_lens) {
      if (x.b->ped_lens[2 * lm] < M) pl.ped_mode[m] = 2;   // A[i] indexed by the hash loop (:131-133)
      pl.ped_zlen[m] = std::min(M, x.b->ped_lens[2 * lm + 1]);
    }
    if (x.b->ck_lens && x.b->ck_lens[lm] < CK_M2) pl.ck_short[m] = 1;
  }
  parallel_for(Mt, 4, [&](size_t b0, size_t b1) {
    HostSha sha;
    for (size_t m = b0; m < b1; ++m) {
      const Sess& x = pl.ss[sess_of_msg[m]];
      const fsdkr_collect_batch* b = x.b;
      const size_t lm = m - x.mbase;
      const uint32_t* ckn = b->ck_n + lm * x.ckl;
      memcpy(CKEXP.data() + m * ckl, ckn, (size_t)x.ckl * 4);
      uint32_t* dst = CKMODS.data() + m * ckl;
      memcpy(dst, ckn, (size_t)x.ckl * 4);
      ck_bits[m] = hbn::bitlen(ckn, x.ckl);
      if (ck_bits[m] == 0) pl.ck_short[m] = 1;                  // rho = mask % 0: division by zero panics
      const bool one = ck_bits[m] == 1;                          // n = 1: every value is 0 mod 1 -> Ok
      const bool ok = !one && ck_bits[m] != 0 && is_odd(ckn) && !small_factor_sieve().divides(ckn, x.ckl);
      if (one) pl.ck_one[m] = 1;
      if (ok) {
        const uint32_t msklen = ck_bits[m] / 256 + 1;
        const uint32_t salt_v =
            ((uint32_t)SALT[0] << 24) | ((uint32_t)SALT[1] << 16) | ((uint32_t)SALT[2] << 8) | SALT[3];
        const hbn::Limbs Nl = hbn::from(ckn, x.ckl);
        std::vector<uint32_t> mask((size_t)msklen * 8, 0);
        for (uint32_t j = 0; j < CK_M2; ++j) {
          // seed = H(n, salt, j), mask block k = H(seed, k): each value as curv to_bytes
          sha.buf.clear();
          put_bigint(sha.buf, ckn, x.ckl);
          put_bigint(sha.buf, &salt_v, 1);
          put_bigint(sha.buf, &j, 1);
          uint32_t seed[8];
          if (!sha.digest(seed)) sha_fail = true;
          for (uint32_t k = 0; k < msklen; ++k) {
            sha.buf.clear();
            put_bigint(sha.buf, seed, 8);
            put_bigint(sha.buf, &k, 1);
            if (!sha.digest(mask.data() + (size_t)k * 8)) sha_fail = true;
          }
          hbn::store(hbn::mod(hbn::from(mask.data(), mask.size()), Nl), RHO.data() + (m * CK_M2 + j) * ckl, ckl);
        }
      } else {   // zero / even / smooth modulus: verdict false, placeholder modulus 3 for the kernels
        std::fill(dst, dst + ckl, 0u);
        dst[0] = 3;
      }
      pl.ck_pre[m] = ok ? 1 : 0;
      // ring-Pedersen statement modulus N = 2^tz * (odd part)
      const uint32_t* N = b->ped_N + lm * b->nl;
      uint32_t* on = PEDN.data() + m * nl;
      memcpy(on, N, (size_t)b->nl * 4);
      uint32_t* sd = PEDS.data() + m * nl;
      memcpy(sd, b->ped_S + lm * b->nl, (size_t)b->nl * 4);
      if (pl.ped_mode[m] == 2 || hbn::is_zero_raw(N, b->nl)) {   // A short / modulus 0: panic before any check
        pl.ped_mode[m] = 2;
        std::fill(on, on + nl, 0u);
        on[0] = 3;
        continue;
      }
      const uint32_t tz = hbn::ctz_raw(N, b->nl);
      ped_tz[m] = tz;
      if (tz) hbn::shr_raw(on, nl, tz);
      if (on[0] == 1 && hbn::is_zero_raw(on + 1, nl - 1)) {   // odd part 1: every congruence mod 1 holds
        pl.ped_mode[m] = 1;
        on[0] = 3;
        continue;
      }
      // S reduced mod the odd part (the eq kernel compares canonical residues of
      // A*S; the reference reduces S^e mod N itself, ring_pedersen_proof.rs:147)
      if (hbn::cmp_raw(sd, nl, on, nl) >= 0) hbn::store(hbn::mod(hbn::from(sd, nl), hbn::from(on, nl)), sd, nl);
    }
  });
  clk.lap("ck rho+primes");
  if (sha_fail) {
    c->fail("fsdkr_collect_prepare: SHA-256 (OpenSSL EVP) failed");
    return FSDKR_E_ARG;
  }
  // DLog statements: N > 2^128, gcd(g, N) = gcd(ni, N) = 1, x < N; challenges e = H(x, g, N, ni)
  pl.dlog_pre.assign(J, 0);
  pl.dlog_trivial.assign(J, 0);
  std::vector<uint32_t> DE((size_t)J * 2 * 8), DLOGN((size_t)J * nl, 0u), dlog_tz(J, 0u);
  parallel_for(J, 2, [&](size_t b0, size_t b1) {
    for (size_t j = b0; j < b1; ++j) {
      const Sess& x = pl.ss[sess_of_join[j]];
      const fsdkr_collect_batch* b = x.b;
      const size_t lj = j - x.jbase, w = b->nl;
      const uint32_t *N = b->dlog_N + lj * w, *g = b->dlog_g + lj * w, *ni = b->dlog_ni + lj * w;
      const uint32_t bl = hbn::bitlen(N, w);
      bool ok = bl > 129 || (bl == 129 && !(N[4] == 1 && hbn::is_zero_raw(N, 4)));
      ok = ok && hbn::gcd_is_one(g, w, N, w) && hbn::gcd_is_one(ni, w, N, w);
      uint8_t pre = 0;
      if (ok && hbn::cmp_raw(b->dlog_x1 + lj * w, w, N, w) < 0) pre |= 1;
      if (ok && hbn::cmp_raw(b->dlog_x2 + lj * w, w, N, w) < 0) pre |= 2;
      pl.dlog_pre[j] = pre;
      for (int which = 0; which < 2; ++which) {
        const uint32_t* xx = (which == 0 ? b->dlog_x1 : b->dlog_x2) + lj * w;
        const uint32_t* gg = which == 0 ? g : ni;
        const uint32_t* nn_ = which == 0 ? ni : g;
        Sha256 h;
        h.init();
        h.bigint(xx, w);
        h.bigint(gg, w);
        h.bigint(N, w);
        h.bigint(nn_, w);
        h.finish_le(DE.data() + (j * 2 + which) * 8);
      }
      uint32_t* on = DLOGN.data() + j * nl;
      memcpy(on, N, w * 4);
      if (!ok) {   // the checks fail before any exponentiation: placeholder modulus
        std::fill(on, on + nl, 0u);
        on[0] = 3;
        continue;
      }
      const uint32_t tz = hbn::ctz_raw(N, w);
      dlog_tz[j] = tz;
      if (tz) hbn::shr_raw(on, nl, tz);
      if (on[0] == 1 && hbn::is_zero_raw(on + 1, nl - 1)) {
        pl.dlog_trivial[j] = 1;
        on[0] = 3;
      }
    }
  });
  // exponent-length bounds
  uint32_t z_max = 1, y_max = 1, ckn_max = 1, recvn_max = 1;
  for (uint32_t s = 0; s < count; ++s) {
    const Sess& x = pl.ss[s];
    const fsdkr_collect_batch* b = x.b;
    for (size_t k = 0; k < (size_t)x.Mt * M; ++k) z_max = std::max(z_max, hbn::bitlen(b->ped_Z + k * b->zl, b->zl));
    for (uint32_t j = 0; j < x.J; ++j) {
      y_max = std::max(y_max, hbn::bitlen(b->dlog_y1 + (size_t)j * b->yl, b->yl));
      y_max = std::max(y_max, hbn::bitlen(b->dlog_y2 + (size_t)j * b->yl, b->yl));
    }
  }
  for (uint32_t m = 0; m < Mt; ++m)
    if (pl.ck_pre[m]) ckn_max = std::max(ckn_max, ck_bits[m]);
  // a prestarted correct-key job (fsdkr_collect_prestart_multi) of these messages:
  // same widths, same n and sigma rows (zero-extended), exponent bound covering
  {
    GaPre* gck = reinterpret_cast<GaPre*>(c->ga_pre);
    bool hit = gck && gck->ck_valid && gck->ck_l == ckl && gck->ck_Mt == Mt && gck->ck_bits >= ckn_max;
    auto same = [&](const uint32_t* pre, const uint32_t* src, uint32_t ws) {
      if (memcmp(pre, src, (size_t)ws * 4) != 0) return false;
      for (uint32_t k = ws; k < ckl; ++k)
        if (pre[k]) return false;
      return true;
    };
    for (uint32_t s = 0; s < count && hit; ++s) {
      const Sess& x = pl.ss[s];
      const fsdkr_collect_batch* b = x.b;
      if (b->ck_lens) hit = false;
      for (uint32_t lm = 0; lm < x.Mt && hit; ++lm) {
        const size_t m = x.mbase + lm;
        hit = same(gck->ck_n.data() + m * ckl, b->ck_n + (size_t)lm * x.ckl, x.ckl);
        for (uint32_t j = 0; j < CK_M2 && hit; ++j)
          hit = same(gck->ck_sigma.data() + (m * CK_M2 + j) * ckl, b->ck_sigma + ((size_t)lm * CK_M2 + j) * x.ckl, x.ckl);
      }
    }
    if (hit) {
      pl.ck_hit = true;
      pl.ck_done = gck->ck_done;
      gck->ck_valid = false;   // consumed (the buffer lives until the next prestart)
    }
  }
  for (uint32_t r = 0; r < n; ++r) recvn_max = std::max(recvn_max, recv_bits[r]);
  // Feldman share checks: per pair (commitment offset, count, index)
  std::vector<FeldmanInfo> finfo(P);
  for (uint32_t s = 0; s < count; ++s) {
    const Sess& x = pl.ss[s];
    uint32_t voff = x.vbase;
    for (uint32_t k = 0; k < x.R; ++k) {
      const uint32_t nc = ncoef_of(x.b, k);
      for (uint32_t i = 0; i < x.n; ++i) finfo[x.pbase + (size_t)k * x.n + i] = {voff, nc, i + 1, 0};
      voff += nc;
    }
  }
  // a prestarted ring-Pedersen T^Z job of these messages (fsdkr_collect_prestart_rp):
  // the same moduli, T rows and Z rows (digest), Z at the same width
  GaPre* gtz = reinterpret_cast<GaPre*>(c->ga_pre);
  bool tz_hit = gtz && gtz->tz_valid && gtz->nl == nl && gtz->tz_Mt == Mt && gtz->tz_M == M && gtz->tz_zl == zl &&
                gtz->pedmod.size() == (size_t)Mt * nl && gtz->T.size() == (size_t)Mt * nl &&
                memcmp(gtz->pedmod.data(), PEDN.data(), (size_t)Mt * nl * 4) == 0;
  for (uint32_t s = 0; s < count && tz_hit; ++s) {
    const Sess& x = pl.ss[s];
    for (uint32_t lm = 0; lm < x.Mt && tz_hit; ++lm) {
      const uint32_t* a = gtz->T.data() + (size_t)(x.mbase + lm) * nl;
      tz_hit = memcmp(a, x.b->ped_T + (size_t)lm * x.b->nl, (size_t)x.b->nl * 4) == 0;
      for (uint32_t k = x.b->nl; k < nl && tz_hit; ++k) tz_hit = a[k] == 0;
    }
  }
  if (tz_hit) {   // the Z rows themselves: SHA-256 per block of rows, as the prestart hashed them
    std::vector<size_t> zrow0(count + 1, 0);
    for (uint32_t s = 0; s < count; ++s) zrow0[s + 1] = zrow0[s] + (size_t)pl.ss[s].Mt * M;
    const std::vector<RowsSha> sha = rows_sha256(zrow0[count], [&](size_t r) {
      const size_t s = (size_t)(std::upper_bound(zrow0.begin(), zrow0.end(), r) - zrow0.begin()) - 1;
      const fsdkr_collect_batch* b = pl.ss[s].b;
      return std::make_pair(b->ped_Z + (r - zrow0[s]) * b->zl, b->zl);
    });
    tz_hit = !sha.empty() && sha == gtz->tz_sha;
  }
  if (tz_hit) {
    pl.tz_hit = true;
    pl.tz_done = gtz->tz_done;
    gtz->tz_valid = false;   // consumed (the buffers live until the next prestart)
  }
  // device address of Z row z: the prestart's copy on a hit (not uploaded again)
  const uint32_t* const tz_z = tz_hit ? gtz->tz_z : nullptr;
  const uint32_t* const tz_out = tz_hit ? gtz->tz_out : nullptr;
  clk.lap("dlog+maxes");

  // ---------------- device layout: inputs (planned; bytes written after the device allocation)
  Img I;
  using B = fsdkr_collect_batch;
  // merged field: the rows of every session at the merged width W
  auto field = [&](const uint32_t* B::*f, auto rows_of, auto width_of, uint32_t W) {
    size_t tot = 0;
    for (const Sess& x : pl.ss) tot += rows_of(x);
    const size_t o = I.reserve(tot * W * 4);
    size_t r = 0;
    for (const Sess& x : pl.ss) {
      const size_t rows = rows_of(x);
      I.rows_at(o + r * W * 4, x.b->*f, rows, width_of(x), W);
      r += rows;
    }
    return o;
  };
  auto R_recv = [](const Sess& x) { return (size_t)x.n; };
  auto R_pair = [](const Sess& x) { return (size_t)x.P; };
  auto R_join = [](const Sess& x) { return (size_t)x.J; };
  auto W_nl = [](const Sess& x) { return x.b->nl; };
  auto W_nn = [](const Sess& x) { return 2 * x.b->nl; };
  auto W_16 = [](const Sess&) { return 16u; };
  auto W_s1 = [](const Sess& x) { return x.b->s1l; };
  auto W_s3 = [](const Sess& x) { return x.b->s3l; };
  auto W_el = [](const Sess& x) { return x.b->el; };
  auto W_yl = [](const Sess& x) { return x.b->yl; };
  const size_t o_rn = field(&B::recv_n, R_recv, W_nl, nl), o_rt = field(&B::recv_ntilde, R_recv, W_nl, nl);
  const size_t o_h1 = field(&B::recv_h1, R_recv, W_nl, nl), o_h2 = field(&B::recv_h2, R_recv, W_nl, nl);
  const size_t o_NN = I.own(NN), o_NP1 = I.own(NP1);
  const size_t o_enc = field(&B::enc, R_pair, W_nn, nn), o_Q = field(&B::commit, R_pair, W_16, 16);
  const size_t o_pz = field(&B::pdl_z, R_pair, W_nl, nl), o_pu1 = field(&B::pdl_u1, R_pair, W_16, 16);
  const size_t o_pu2 = field(&B::pdl_u2, R_pair, W_nn, nn), o_pu3 = field(&B::pdl_u3, R_pair, W_nl, nl);
  const size_t o_ps1 = field(&B::pdl_s1, R_pair, W_s1, s1l), o_ps2 = field(&B::pdl_s2, R_pair, W_nl, nl);
  const size_t o_ps3 = field(&B::pdl_s3, R_pair, W_s3, s3l);
  const size_t o_az = field(&B::rp_z, R_pair, W_nl, nl), o_ae = field(&B::rp_e, R_pair, W_el, el);
  // negative z (fsdkr_collect_batch.neg_bits): the rows hold |z| (hashed); z^e takes -|z| mod N~
  std::vector<uint32_t> zneg_row(2 * (size_t)P, ~0u), ZR;
  for (const Sess& x : pl.ss)
    if (x.b->neg_bits)
      for (uint32_t lp = 0; lp < x.P; ++lp)
        for (int which = 0; which < 2; ++which)
          if (x.b->neg_bits[lp] & (1u << which)) {
            const uint32_t p = x.pbase + lp, r = recv_of_pair[p];
            const uint32_t* zr = (which ? x.b->rp_z : x.b->pdl_z) + (size_t)lp * x.b->nl;
            const hbn::Limbs Nt = hbn::from(x.b->recv_ntilde + (size_t)(r - x.rbase) * x.b->nl, x.b->nl);
            const hbn::Limbs zm = hbn::mod(hbn::from(zr, x.b->nl), Nt);
            const hbn::Limbs res = zm.empty() ? zm : hbn::sub(Nt, zm);
            zneg_row[(size_t)which * P + p] = (uint32_t)(ZR.size() / nl);
            ZR.resize(ZR.size() + nl);
            hbn::store(res, ZR.data() + ZR.size() - nl, nl);
          }
  const size_t o_zr = ZR.empty() ? 0 : I.own(ZR);
  auto z_off = [&](int which, uint32_t p, size_t o_raw) {   // image offset of z's row as J5's base
    const uint32_t k = zneg_row[(size_t)which * P + p];
    return k == ~0u ? o_raw + (size_t)p * nl * 4 : o_zr + (size_t)k * nl * 4;
  };
  const size_t o_as = field(&B::rp_s, R_pair, W_nl, nl), o_as1 = field(&B::rp_s1, R_pair, W_s1, s1l);
  const size_t o_as2 = field(&B::rp_s2, R_pair, W_s3, s3l);
  const size_t o_vss = I.reserve((size_t)V * 64);
  for (const Sess& x : pl.ss) I.rows_at(o_vss + (size_t)x.vbase * 64, x.b->vss, x.V, 16, 16);
  const size_t o_pSraw = I.reserve((size_t)Mt * nl * 4), o_pT = I.reserve((size_t)Mt * nl * 4);
  const size_t o_pA = I.reserve((size_t)Mt * M * nl * 4), o_pZ = tz_z ? 0 : I.reserve((size_t)Mt * M * zl * 4);
  for (const Sess& x : pl.ss) {
    I.rows_at(o_pSraw + (size_t)x.mbase * nl * 4, x.b->ped_S, x.Mt, x.b->nl, nl);
    I.rows_at(o_pT + (size_t)x.mbase * nl * 4, x.b->ped_T, x.Mt, x.b->nl, nl);
    I.rows_at(o_pA + (size_t)x.mbase * M * nl * 4, x.b->ped_A, (size_t)x.Mt * M, x.b->nl, nl);
    if (!tz_z) I.rows_at(o_pZ + (size_t)x.mbase * M * zl * 4, x.b->ped_Z, (size_t)x.Mt * M, x.b->zl, zl);
  }
  const size_t o_pS = I.own(PEDS);
  // negative ring-Pedersen A (ped_a_neg): the rows hold |A| (hashed); the check takes -|A| mod N
  std::vector<uint32_t> aneg_row((size_t)Mt * M, ~0u), AR;
  for (const Sess& x : pl.ss)
    if (x.b->ped_a_neg)
      for (size_t q = 0; q < (size_t)x.Mt * M; ++q)
        if (x.b->ped_a_neg[q]) {
          const size_t lm = q / M;
          const hbn::Limbs Nm = hbn::from(x.b->ped_N + lm * x.b->nl, x.b->nl);
          const hbn::Limbs am = hbn::mod(hbn::from(x.b->ped_A + q * x.b->nl, x.b->nl), Nm);
          aneg_row[(size_t)x.mbase * M + q] = (uint32_t)(AR.size() / nl);
          AR.resize(AR.size() + nl);
          hbn::store(am.empty() ? am : hbn::sub(Nm, am), AR.data() + AR.size() - nl, nl);
        }
  const size_t o_ar = AR.empty() ? 0 : I.own(AR);
  auto a_off = [&](size_t q) {   // image offset of A_q's row in the checks (q = m * M + k)
    return aneg_row[q] == ~0u ? o_pA + q * nl * 4 : o_ar + (size_t)aneg_row[q] * nl * 4;
  };
  const size_t o_cks = I.reserve((size_t)Mt * CK_M2 * ckl * 4);
  for (const Sess& x : pl.ss)
    I.rows_at(o_cks + (size_t)x.mbase * CK_M2 * ckl * 4, x.b->ck_sigma, (size_t)x.Mt * CK_M2, x.ckl, ckl);
  const size_t o_ckn = I.own(CKEXP);          // exponent: the caller's ek.n
  const size_t o_ckmods = I.own(CKMODS);      // modulus: ek.n, or placeholder 3 where the verdict is forced
  const size_t o_rho = I.own(RHO);
  size_t o_dg = 0, o_dni = 0, o_dx1 = 0, o_dx2 = 0, o_dy1 = 0, o_dy2 = 0, o_de = 0;
  if (J) {
    o_dg = field(&B::dlog_g, R_join, W_nl, nl);
    o_dni = field(&B::dlog_ni, R_join, W_nl, nl);
    o_dx1 = field(&B::dlog_x1, R_join, W_nl, nl);
    o_dx2 = field(&B::dlog_x2, R_join, W_nl, nl);
    o_dy1 = field(&B::dlog_y1, R_join, W_yl, yl);
    o_dy2 = field(&B::dlog_y2, R_join, W_yl, yl);
    o_de = I.own(DE);
  }
  std::vector<uint32_t> ONE(std::max(nn, ckl), 0);
  ONE[0] = 1;
  const size_t o_one = I.own(ONE);
  // nl-width moduli table: Ntilde_i | ring-Pedersen N (odd part) | DLog N (odd part)
  const uint32_t n_mods_nl = n + Mt + J;
  const size_t o_mods = I.reserve((size_t)n_mods_nl * nl * 4);
  for (const Sess& x : pl.ss) I.rows_at(o_mods + (size_t)x.rbase * nl * 4, x.b->recv_ntilde, x.n, x.b->nl, nl);
  {
    std::vector<uint8_t> tail(((size_t)Mt + J) * nl * 4);
    memcpy(tail.data(), PEDN.data(), (size_t)Mt * nl * 4);
    if (J) memcpy(tail.data() + (size_t)Mt * nl * 4, DLOGN.data(), (size_t)J * nl * 4);
    I.own_at(o_mods + (size_t)n * nl * 4, std::move(tail));
  }
  const size_t o_finfo = I.own(finfo);
  const size_t o_epdl = I.own(EPDL);
  const size_t o_rc = RC.empty() ? 0 : I.own(RC);
  clk.lap("layout plan");

  // ---------------- device layout: outputs (offsets relative to the output region)
  size_t out_bytes = 0;
  auto OUT = [&](size_t bytes) {
    const size_t o = Img::al(out_bytes);
    out_bytes = o + Img::al(bytes ? bytes : 1);
    return o;
  };
  const size_t x_pbits = OUT((size_t)Mt * MW * 4), x_ppanic = OUT((size_t)Mt * 4);
  const size_t x_Bpdl = OUT((size_t)P * nn * 4), x_gs1 = OUT((size_t)P * nn * 4);
  //   GA (nn, long)  = s2^N | s^N  [2P]  ++  (N+1)^s1 for s1 >= N  [<= P]
  //   J2 (nn, short) = c^e_pdl | c^e_A  [2P]
  //   J5 (nl, short) = z^e_pdl | zA^e_A [2P]
  //   GD (nl, long)  = g^y1 | ni^y2 [2J] ++ ni^e1 | g^e2 [2J]
  //   GC (ckl)       = sigma^n [Mt*11]
  //   FB (nl, fixed bases h1_i, h2_i, T_m) = h2^s3 | h2^s2A [2P], h1^s1 | h1^s1A [2P], T^Z [Mt*M]
  const size_t x_GA = OUT(((size_t)3 * P + 1) * nn * 4);   // + the joint GA's pad row 3P
  const size_t x_J1 = x_GA, x_J9 = x_GA + (size_t)2 * P * nn * 4;
  // J1 result row k (device address): the GA job's output, or the prestart buffer
  auto J1_at = [&](size_t k) -> uint64_t {
    return pl.ga_hit ? (uint64_t)(uintptr_t)(gpre->out + k * nn) : 0;
  };
  const size_t x_J2 = OUT((size_t)2 * P * nn * 4);
  const size_t x_J5 = OUT((size_t)2 * P * nl * 4);
  const size_t x_GD = OUT(((size_t)4 * J + 1) * nl * 4);
  const size_t x_J7 = x_GD, x_J8 = x_J7 + (size_t)2 * J * nl * 4;
  const size_t x_GC = OUT(((size_t)Mt * CK_M2 + 1) * ckl * 4);
  const size_t x_FB = OUT(((size_t)4 * P + (size_t)Mt * M + 1) * nl * 4);
  const size_t x_J4 = x_FB, x_J3 = x_J4 + (size_t)2 * P * nl * 4, x_RP = x_J3 + (size_t)2 * P * nl * 4;
  const size_t x_invc = OUT((size_t)2 * P * nn * 4), x_invz = OUT((size_t)P * nl * 4);
  const size_t x_unn = OUT((size_t)2 * P * 4);
  const size_t x_uzA = OUT((size_t)P * 4), x_uzp = OUT((size_t)P * 4);
  const size_t x_eq2 = OUT((size_t)P * 4);
  const size_t n_eqnl = (size_t)P + (size_t)Mt * M + 2 * (size_t)J;
  const size_t x_eq3 = OUT(n_eqnl * 4);               // [u3 P | RP Mt*M | DLog 2J]
  const size_t x_eqck = OUT((size_t)Mt * CK_M2 * 4);
  const size_t x_u = OUT((size_t)P * nn * 4), x_w = OUT(((size_t)P + K3) * nl * 4);   // + z^e h2^|s3| [K3]
  const size_t x_fel = OUT(P), x_pdlv = OUT(P), x_rng = OUT(P);
  // 2-adic checks of even moduli
  uint32_t n_p2 = 0;
  pl.ped_p2_first.assign(Mt, ~0u);
  pl.dlog_p2_first.assign(J, ~0u);
  for (uint32_t m = 0; m < Mt; ++m)
    if (ped_tz[m] && pl.ped_mode[m] != 2) {
      pl.ped_p2_first[m] = n_p2;
      n_p2 += M;
    }
  for (uint32_t j = 0; j < J; ++j)
    if (dlog_tz[j] && pl.dlog_pre[j]) {
      pl.dlog_p2_first[j] = n_p2;
      n_p2 += 2;
    }
  const size_t x_p2 = OUT((size_t)n_p2 * 4);

  // single device allocation: [inputs | descriptors | outputs]
  const size_t in_bytes_pre = Img::al(I.size);
  const size_t n_eqall = (size_t)P + n_eqnl + (size_t)Mt * CK_M2;
  const size_t desc_bound =
      ((size_t)7 * P + 4 * (size_t)J + (size_t)Mt * CK_M2) * 32 + (size_t)3 * P * 4 +    // modexp jobs (+ GA out_idx)
      (size_t)n * 63 * 36 +                                                                // GA pads
      (2 * (size_t)n + Mt) * 24 + (4 * (size_t)P + (size_t)Mt * M) * 32 + 24 * 512 +      // fixed-base job
      (2 * (size_t)n + Mt) * 8 + (4 * (size_t)P + (size_t)Mt * M) * 4 + 4 * (8192 + 2048) +   // its comb groups
      4 * (size_t)P * 8 + 4 * (size_t)P * 16 +                                            // binom, inverses
      n_eqall * (sizeof(EqOperand) + 4) + 2 * (size_t)P * sizeof(Prod3Operand) + 4 * (size_t)P +
      (K3 ? K3 * (sizeof(Prod3Operand) + 4) + 4 * (size_t)P + 1024 : 0) +               // negative s3 rows
      2 * (size_t)P * 8 + P + (size_t)n_p2 * sizeof(Pow2Op) + 32 * 256 + 64 * 1024 +
      ((size_t)2 * P + (size_t)n * 63) * kTailDescBytes;                                 // the joint tail's block
  const size_t out_off = Img::al(in_bytes_pre + desc_bound);
  const size_t total = out_off + out_bytes;
  uint8_t* dev = (uint8_t*)c->buf("collect_arena", total);
  if (!dev) {
    c->fail("fsdkr_verify_collect: device allocation of %zu bytes failed", total);
    return FSDKR_E_OOM;
  }
  uint8_t* const out_base = dev + out_off;
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };        // input address
  auto DX = [&](size_t o) { return (uint64_t)(uintptr_t)(out_base + o); };   // output address

  // the h1_i / h2_i tables of a prestart: sized for the prestart's exponent bounds
  // (taller tables only add unused entries), used if the layout then agrees
  const GaPre* gp = reinterpret_cast<const GaPre*>(c->ga_pre);
  // the prestart's rows are global (session s after s-1) at width nl, zero-extended
  auto same_rows = [&](const std::vector<uint32_t>& pre, size_t base, const uint32_t* src, size_t rows,
                       uint32_t ws) {
    if (pre.size() < (base + rows) * nl) return false;
    for (size_t r = 0; r < rows; ++r) {
      const uint32_t* a = pre.data() + (base + r) * nl;
      if (memcmp(a, src + r * ws, (size_t)ws * 4) != 0) return false;
      for (uint32_t k = ws; k < nl; ++k)
        if (a[k]) return false;
    }
    return true;
  };
  bool fb_cand = gp && gp->fb_valid && gp->nl == nl && gp->n == n && gp->Mt == Mt &&
                 memcmp(gp->pedmod.data(), PEDN.data(), (size_t)Mt * nl * 4) == 0 &&
                 std::max(mx.s1, mx.as1) <= gp->bits_h1 && std::max(mx.s3, mx.as2) <= gp->bits_h2 &&
                 z_max <= gp->bits_z;
  for (const Sess& x : pl.ss) {
    if (!fb_cand) break;
    fb_cand = same_rows(gp->ntilde, x.rbase, x.b->recv_ntilde, x.n, x.b->nl) &&
              same_rows(gp->h1, x.rbase, x.b->recv_h1, x.n, x.b->nl) &&
              same_rows(gp->h2, x.rbase, x.b->recv_h2, x.n, x.b->nl) &&
              same_rows(gp->T, x.mbase, x.b->ped_T, x.Mt, x.b->nl);
  }
  // ---------------- modexp jobs (descriptors addressed into the image)
  ModexpJob J1, J2, J5, J7, J8, J9, GC;
  J1.k32 = J2.k32 = J9.k32 = nn;
  J5.k32 = J7.k32 = J8.k32 = nl;
  GC.k32 = ckl;
  FbJob& FB = pl.fb;
  FB = FbJob();
  FB.k32 = nl;
  // base order [h1_i | T_m | h2_i] and instance order [h1 | T | h2]: group A (the
  // short h1 chains and the T chains) and group B (the long h2 chains) are
  // contiguous, so group A's exponents run as soon as its tables exist
  std::vector<uint32_t> fb_h1(n), fb_h2(n), fb_T(Mt);
  for (uint32_t r = 0; r < n; ++r) fb_h1[r] = FB.add_base(DI(o_h1 + (size_t)r * nl * 4), nl, r);
  for (uint32_t m = 0; m < Mt; ++m) fb_T[m] = FB.add_base(DI(o_pT + (size_t)m * nl * 4), nl, n + m);
  for (uint32_t r = 0; r < n; ++r) fb_h2[r] = FB.add_base(DI(o_h2 + (size_t)r * nl * 4), nl, r);
  struct FbAdd {
    uint32_t base;
    uint64_t exp;
    uint32_t elen, ebits;
    uint64_t out;
  };
  std::vector<FbAdd> fb_later;   // the h2 instances, added after the T instances
  fb_later.reserve(2 * (size_t)P);
  std::vector<uint32_t> j9_index(P, 0xFFFFFFFFu);
  for (int which = 0; which < 2; ++which)
    for (uint32_t p = 0; p < P; ++p) {
      const uint32_t r = recv_of_pair[p];
      const uint64_t Ni = DI(o_rn + (size_t)r * nl * 4);
      // J1: s2^N (PDL, zk_pdl_with_slack.rs:129-135) | s^N (Alice, range_proofs.rs:148)
      if (!pl.ga_hit)
        J1.add(which == 0 ? DI(o_ps2 + (size_t)p * nl * 4) : DI(o_as + (size_t)p * nl * 4), nl, Ni, nl, recvn_max, r);
      // J2: c^e (PDL :136-142 via the cross-multiplied check) | c^e (Alice :142)
      const uint64_t cp = big_c[p] ? DI(o_rc + (size_t)p * nn * 4) : DI(o_enc + (size_t)p * nn * 4);
      if (pl.joint) {   // (joined into GA's tail)
      } else if (which == 0) {
        J2.add(cp, nn, DI(o_epdl + (size_t)p * 32), 8, 256, r);
      } else {
        J2.add(cp, nn, DI(o_ae + (size_t)p * el * 4), el, mx.ae, r);
      }
      // fixed bases (FB): h1^s1 -> J3 slot | h2^s3 (s2 for Alice) -> J4 slot;  J5: z^e
      const size_t slot = (size_t)which * P + p;
      if (which == 0) {
        FB.add(fb_h1[r], DI(o_ps1 + (size_t)p * s1l * 4), s1l, mx.s1, DX(x_J3 + slot * nl * 4));
        fb_later.push_back({fb_h2[r], DI(o_ps3 + (size_t)p * s3l * 4), s3l, mx.s3, DX(x_J4 + slot * nl * 4)});
        J5.add(DI(z_off(0, p, o_pz)), nl, DI(o_epdl + (size_t)p * 32), 8, 256, r);
      } else {
        const bool use = alice_pre[p];
        FB.add(fb_h1[r], DI(o_as1 + (size_t)p * s1l * 4), use ? s1l : 0, mx.as1, DX(x_J3 + slot * nl * 4));
        fb_later.push_back({fb_h2[r], DI(o_as2 + (size_t)p * s3l * 4), use ? s3l : 0, mx.as2,
                            DX(x_J4 + slot * nl * 4)});
        J5.add(DI(z_off(1, p, o_az)), nl, DI(o_ae + (size_t)p * el * 4), use ? el : 0, mx.ae, r);
      }
    }
  for (uint32_t p = 0; p < P; ++p)
    if (!pdl_small[p]) {
      const uint32_t r = recv_of_pair[p];
      j9_index[p] = (uint32_t)J9.size();
      J9.add(DI(o_NP1 + (size_t)r * nn * 4), nn, DI(o_ps1 + (size_t)p * s1l * 4), s1l, mx.s1, r);
    }
  clk.lap("desc pairs");
  if (!tz_hit) {  // ring-Pedersen T^Z_k mod N (ring_pedersen_proof.rs:144): Mt*M instances, filled in parallel
    const size_t o = FB.grow((size_t)Mt * M);
    for (uint32_t m = 0; m < Mt; ++m) FB.b_bits[fb_T[m]] = std::max(FB.b_bits[fb_T[m]], std::max(z_max, 1u));
    parallel_for(Mt, 16, [&](size_t m0, size_t m1) {
      for (size_t m = m0; m < m1; ++m) {
        const uint32_t b = fb_T[m], md = FB.b_mod[b];
        for (uint32_t k = 0; k < M; ++k) {
          const size_t i = o + m * M + k, z = m * M + k;
          FB.e_ptr[i] = DI(o_pZ + z * zl * 4);   // (uploaded: no prestarted job)
          FB.e_len[i] = zl;
          FB.e_base[i] = b;
          FB.e_mod[i] = md;
          FB.o_ptr[i] = DX(x_RP + z * nl * 4);
        }
      }
    });
  }
  clk.lap("desc rp");
  for (const FbAdd& a : fb_later) FB.add(a.base, a.exp, a.elen, a.ebits, a.out);
  for (uint32_t m = 0; m < Mt && !pl.ck_hit; ++m)
    for (uint32_t k = 0; k < CK_M2; ++k)  // correct-key sigma_k^n mod n (unless prestarted)
      GC.add(DI(o_cks + ((size_t)m * CK_M2 + k) * ckl * 4), ckl, DI(o_ckn + (size_t)m * ckl * 4), ckl,
             pl.ck_pre[m] ? ckn_max : 0u, m);
  for (uint32_t j = 0; j < J; ++j) {
    const uint32_t mi = n + Mt + j;
    J7.add(DI(o_dg + (size_t)j * nl * 4), nl, DI(o_dy1 + (size_t)j * yl * 4), yl, y_max, mi);
    J7.add(DI(o_dni + (size_t)j * nl * 4), nl, DI(o_dy2 + (size_t)j * yl * 4), yl, y_max, mi);
    J8.add(DI(o_dni + (size_t)j * nl * 4), nl, DI(o_de + (size_t)(2 * j) * 32), 8, 256, mi);
    J8.add(DI(o_dg + (size_t)j * nl * 4), nl, DI(o_de + (size_t)(2 * j + 1) * 32), 8, 256, mi);
  }
  // descriptor image, placed right after the inputs (desc_base is 256-aligned, so
  // alignment inside `desc` carries over to device addresses)
  std::vector<uint8_t> desc;
  const size_t desc_base = in_bytes_pre;
  auto D_al = [&]() {
    desc.resize(Img::al(desc.size()), 0);
    return desc_base + desc.size();
  };
  auto pack_job = [&](const ModexpJob& j) {
    const size_t o = D_al();
    j.pack(desc);
    return o;
  };
  auto put = [&](const void* src, size_t bytes) {
    const size_t o = D_al();
    const size_t at = desc.size();
    desc.resize(at + bytes);
    if (bytes) memcpy(desc.data() + at, src, bytes);
    return o;
  };
  // GA: J1 receiver-major (every wave's chains share N_i: sliding windows when the
  // groups fill whole waves and no J9 instance joins the launch), then J9
  // joint: J1 alone (padded, pads write row 3P), J9 its own launch in job slot 2
  const uint32_t ga_group = ga_lanes((uint32_t)(J1.size() + (pl.joint ? 0 : J9.size())), nn);
  // (pads write the first J9 row, unused when J9 is empty)
  const uint32_t ga_pw = ga_per_wave(ga_group, nn);
  const uint32_t pad_row = pl.joint ? (uint32_t)(3 * P) : J9.size() ? kNoPad : (uint32_t)(2 * P);
  const bool ga_aligned = J1.size() && group_by_exponent(J1, ga_pw, pad_row) && (pl.joint || J9.size() == 0);
  ModexpJob GA = J1, GD = J7;
  if (!pl.joint) GA.append(J9);
  pl.jflags[0] = GA.out_idx.empty() ? 0u : ga_desc_flags(ga_aligned, ga_group);
  if (pl.joint && !pl.ga_hit && !ga_split_ok(nn, ga_group, pl.jflags[0])) {
    c->fail("internal: the joint GA lost its sliding-window shape");
    return FSDKR_E_ARG;
  }
  GD.append(J8);
  const size_t d_GA = pack_job(GA), d_J2 = pack_job(pl.joint ? J9 : J2), d_J5 = pack_job(J5), d_GD = pack_job(GD),
               d_GC = pack_job(GC);
  // the joint tail's per-instance block (base2 = c^-1 mod N^2 of the pair, exp2 = e_pdl |
  // e_A) in GA's instance order: the prestarted head's, or GA's own
  if (pl.joint) {
    const std::vector<uint32_t>& rows = pl.ga_hit ? gpre->ga_rows : GA.out_idx;
    const size_t ni = rows.size();
    std::vector<uint8_t> d2(ni * kTailDescBytes, 0);
    auto* b2p = reinterpret_cast<uint64_t*>(d2.data());
    auto* e2p = reinterpret_cast<uint64_t*>(d2.data() + ni * 8);
    auto* e2l = reinterpret_cast<uint32_t*>(d2.data() + ni * 16);
    for (size_t k = 0; k < ni; ++k) {
      const uint32_t r = rows[k];
      const uint32_t p = r < 2 * P ? r % P : 0u;
      b2p[k] = DX(x_invc + (size_t)p * nn * 4);
      if (r < P) {          // PDL: s2^N c^-e_pdl
        e2p[k] = DI(o_epdl + (size_t)p * 32);
        e2l[k] = 8;
      } else if (r < 2 * P) {   // Alice: s^N c^-e_A (a rejected proof's e unused: 0)
        e2p[k] = DI(o_ae + (size_t)p * el * 4);
        e2l[k] = alice_pre[p] ? std::min(el, 8u) : 0u;
      } else {              // pads
        e2p[k] = DI(o_epdl);
        e2l[k] = 0;
      }
    }
    pl.d_desc2 = put(d2.data(), d2.size());
  }
  if (fb_cand) {
    for (uint32_t r = 0; r < n; ++r) {
      FB.b_bits[fb_h1[r]] = gp->bits_h1;
      FB.b_bits[fb_h2[r]] = gp->bits_h2;
    }
    for (uint32_t m = 0; m < Mt; ++m) FB.b_bits[fb_T[m]] = gp->bits_z;
  }
  FB.finalize();
  if (fb_cand && FB.w == gp->fb_w && FB.bases() == 2 * (size_t)n + Mt) {
    const FbLayout L = fb_layout(n, Mt, FB.w, gp->bits_h1, gp->bits_h2, gp->bits_z);
    bool same = L.entries == gp->fb_entries;
    for (uint32_t k = 0; k < FB.bases() && same; ++k)
      same = FB.b_h[k] == L.h[k] && FB.b_toff[k] == L.toff[k] && FB.b_mod[k] == L.mod[k];
    if (same) {
      pl.fb_hit = true;
      pl.fb_pre.table = gp->fb_table;
      pl.fb_pre.entries = gp->fb_entries;
      pl.fb_pre.ready = gp->fb_done;
      reinterpret_cast<GaPre*>(c->ga_pre)->fb_valid = false;   // consumed
    }
  }
  // Lim-Lee combs per base class when they beat BGMW (comb.hip), over the
  // prestart's comb tables when it built them for the same classes
  FB.plan_comb(comb_mode(c), comb_mem_cap(c), pl.fb_hit && gp ? &gp->comb_pre : nullptr);
  if (pl.fb_hit && gp) pl.fb_pre.comb_ready = gp->comb_done;
  clk.lap("desc fb finalize");
  FB.pack(desc);   // FbJob offsets are positions in `desc`, i.e. relative to desc_base
  // binom descriptors: PDL B = 1 + s1*N (small s1) | Alice gs1 = 1 + s1A*N
  std::vector<uint64_t> bs_ptr(2 * (size_t)P), bn_ptr(2 * (size_t)P);
  for (uint32_t p = 0; p < P; ++p) {
    bs_ptr[p] = DI(o_ps1 + (size_t)p * s1l * 4);
    bs_ptr[P + p] = DI(o_as1 + (size_t)p * s1l * 4);
    bn_ptr[p] = bn_ptr[P + p] = DI(o_rn + (size_t)recv_of_pair[p] * nl * 4);
  }
  const size_t d_bs = put(bs_ptr.data(), bs_ptr.size() * 8), d_bn = put(bn_ptr.data(), bn_ptr.size() * 8);
  // inverse descriptors: nn: c^eA (Alice; also the PDL unit test of c when eA != 0) + c^e_pdl (eA == 0)
  std::vector<uint64_t> inv_y_nn, inv_m_nn, inv_y_nl(2 * (size_t)P), inv_m_nl(2 * (size_t)P);
  std::vector<uint32_t>& cpdl_extra = pl.cpdl_extra;
  cpdl_extra.clear();
  inv_y_nn.reserve(2 * (size_t)P);
  inv_m_nn.reserve(2 * (size_t)P);
  for (uint32_t p = 0; p < P && pl.joint; ++p) {   // joint: c^-1 mod N^2 (value for the tail, c's unit flag)
    inv_y_nn.push_back(big_c[p] ? DI(o_rc + (size_t)p * nn * 4) : DI(o_enc + (size_t)p * nn * 4));
    inv_m_nn.push_back(DI(o_NN + (size_t)recv_of_pair[p] * nn * 4));
  }
  for (uint32_t p = 0; p < P && !pl.joint; ++p) {
    inv_y_nn.push_back(DX(x_J2 + ((size_t)P + p) * nn * 4));
    inv_m_nn.push_back(DI(o_NN + (size_t)recv_of_pair[p] * nn * 4));
  }
  for (uint32_t p = 0; p < P && !pl.joint; ++p)
    if (ae_bits[p] == 0 || !alice_pre[p]) {  // c^eA does not witness c's unit-ness
      inv_y_nn.push_back(DX(x_J2 + (size_t)p * nn * 4));
      inv_m_nn.push_back(DI(o_NN + (size_t)recv_of_pair[p] * nn * 4));
      cpdl_extra.push_back(p);
    }
  for (uint32_t p = 0; p < P; ++p) {  // zA^eA (value) then z^e_pdl (unit test)
    const uint64_t mt = DI(o_rt + (size_t)recv_of_pair[p] * nl * 4);
    inv_y_nl[p] = DX(x_J5 + ((size_t)P + p) * nl * 4);
    inv_m_nl[p] = mt;
    inv_y_nl[P + p] = DX(x_J5 + (size_t)p * nl * 4);
    inv_m_nl[P + p] = mt;
  }
  const size_t d_iynn = put(inv_y_nn.data(), inv_y_nn.size() * 8), d_imnn = put(inv_m_nn.data(), inv_m_nn.size() * 8);
  const size_t d_iynl = put(inv_y_nl.data(), inv_y_nl.size() * 8), d_imnl = put(inv_m_nl.data(), inv_m_nl.size() * 8);
  // the pairs by receiver (counting sort): the groups of the simultaneous inversions
  {
    uint32_t nrecv = 0;
    for (uint32_t r : recv_of_pair) nrecv = std::max(nrecv, r + 1);
    std::vector<uint32_t> cnt((size_t)nrecv + 1, 0), order(P), gstart;
    for (uint32_t r : recv_of_pair) ++cnt[r + 1];
    for (size_t r = 1; r <= nrecv; ++r) cnt[r] += cnt[r - 1];
    gstart.reserve((size_t)nrecv + 1);
    for (size_t r = 0; r < nrecv; ++r)
      if (cnt[r + 1] > cnt[r]) gstart.push_back(cnt[r]);
    gstart.push_back(P);
    for (uint32_t p = 0; p < P; ++p) order[cnt[recv_of_pair[p]]++] = p;
    pl.binv_ngroups = (uint32_t)gstart.size() - 1;
    pl.d_binv_order = put(order.data(), order.size() * 4);
    pl.d_binv_gstart = put(gstart.data(), gstart.size() * 4);
  }
  // the rows of the fixed-base (J3, J4) and challenge (J2, J5) outputs
  auto J3_row = [&](size_t k) { return DX(x_J3 + k * nl * 4); };
  auto J4_row = [&](size_t k) { return DX(x_J4 + k * nl * 4); };
  auto J2_row = [&](size_t k) { return DX(x_J2 + k * nn * 4); };
  auto J5_row = [&](size_t k) { return DX(x_J5 + k * nl * 4); };
  // eq_check descriptors
  clk.lap("desc fb/binom/inv");
  std::vector<EqOperand> eq_nn(P), eq_nl, eq_ck;
  std::vector<uint32_t> eq_nn_mod(P), eq_nl_mod, eq_ck_mod;
  for (uint32_t p = 0; p < P; ++p) {  // PDL u2: (N+1)^s1 * s2^N == u2 * c^e  (mod N^2), u2 < N^2
    EqOperand& e = eq_nn[p];
    e.a = pdl_small[p] ? DX(x_Bpdl + (size_t)p * nn * 4) : DX(x_J9 + (size_t)j9_index[p] * nn * 4);
    e.b = pl.ga_hit ? J1_at(p) : DX(x_J1 + (size_t)p * nn * 4);
    e.c = DI(o_pu2 + (size_t)p * nn * 4);
    e.d = pl.joint ? DI(o_one) : J2_row(p);   // joint: b = s2^N c^-e_pdl already
    e.a_len = e.b_len = e.c_len = e.d_len = nn;
    e.sel = 0xFFFFFFFFu;
    e.flags = 1;
    eq_nn_mod[p] = recv_of_pair[p];
  }
  eq_nl.reserve(n_eqnl);
  eq_nl_mod.reserve(n_eqnl);
  for (uint32_t p = 0; p < P; ++p) {  // PDL u3: h1^s1 * h2^s3 == u3 * z^e  (mod N~), u3 < N~
    EqOperand e;
    e.a = J3_row(p);
    e.b = J4_row(p);
    e.c = DI(o_pu3 + (size_t)p * nl * 4);
    e.d = J5_row(p);
    e.a_len = e.b_len = e.c_len = e.d_len = nl;
    e.sel = 0xFFFFFFFFu;
    e.flags = 1;
    eq_nl.push_back(e);
    eq_nl_mod.push_back(recv_of_pair[p]);
  }
  for (size_t k = 0; k < K3; ++k) {   // s3 < 0: h1^s1 * 1 == u3 * (z^e * h2^|s3|), prod3 row P + k
    EqOperand& e = eq_nl[neg3[k]];
    e.b = DI(o_one);
    e.d = DX(x_w + ((size_t)P + k) * nl * 4);
  }
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < M; ++k) {  // RP: T^Z_k == A_k * S^(e_k)  (mod N; the odd part here)
      EqOperand e;
      e.a = tz_out ? (uint64_t)(uintptr_t)(tz_out + ((size_t)m * M + k) * nl)
                   : DX(x_RP + ((size_t)m * M + k) * nl * 4);
      e.b = DI(o_one);
      e.c = DI(a_off((size_t)m * M + k));
      e.d = DI(o_pS + (size_t)m * nl * 4);
      e.a_len = e.b_len = e.c_len = e.d_len = nl;
      e.sel = m * MW * 32 + k;
      e.flags = 0;
      eq_nl.push_back(e);
      eq_nl_mod.push_back(n + m);
    }
  for (uint32_t j = 0; j < J; ++j)
    for (int which = 0; which < 2; ++which) {  // DLog: g^y * ni^e == x (mod N; x < N checked on the host)
      EqOperand e;
      e.a = DX(x_J7 + ((size_t)2 * j + which) * nl * 4);
      e.b = DX(x_J8 + ((size_t)2 * j + which) * nl * 4);
      e.c = DI((which == 0 ? o_dx1 : o_dx2) + (size_t)j * nl * 4);
      e.d = DI(o_one);
      e.a_len = e.b_len = e.c_len = e.d_len = nl;
      e.sel = 0xFFFFFFFFu;
      e.flags = 0;
      eq_nl.push_back(e);
      eq_nl_mod.push_back(n + Mt + j);
    }
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < CK_M2; ++k) {  // correct key: sigma^n == rho (mod n)
      EqOperand e;
      e.a = pl.ck_hit ? (uint64_t)(uintptr_t)(reinterpret_cast<const GaPre*>(c->ga_pre)->ck_out +
                                               ((size_t)m * CK_M2 + k) * ckl)
                      : DX(x_GC + ((size_t)m * CK_M2 + k) * ckl * 4);
      e.b = DI(o_one);
      e.c = DI(o_rho + ((size_t)m * CK_M2 + k) * ckl * 4);
      e.d = DI(o_one);
      e.a_len = e.b_len = e.c_len = e.d_len = ckl;
      e.sel = 0xFFFFFFFFu;
      e.flags = 0;
      eq_ck.push_back(e);
      eq_ck_mod.push_back(m);
    }
  clk.lap("desc eq build");
  const size_t d_eqnn = put(eq_nn.data(), eq_nn.size() * sizeof(EqOperand)),
               d_eqnnm = put(eq_nn_mod.data(), eq_nn_mod.size() * 4);
  const size_t d_eqnl = put(eq_nl.data(), eq_nl.size() * sizeof(EqOperand)),
               d_eqnlm = put(eq_nl_mod.data(), eq_nl_mod.size() * 4);
  const size_t d_eqck = put(eq_ck.data(), eq_ck.size() * sizeof(EqOperand)),
               d_eqckm = put(eq_ck_mod.data(), eq_ck_mod.size() * 4);
  // prod3 descriptors: u = gs1 * s^N * (c^e)^-1  (mod N^2) | w = h1^s1 * h2^s2 * (z^e)^-1 (mod N~)
  std::vector<Prod3Operand> p3_nn(P), p3_nl(P);
  for (uint32_t p = 0; p < P; ++p) {
    p3_nn[p] = {DX(x_gs1 + (size_t)p * nn * 4), pl.ga_hit ? J1_at((size_t)P + p) : DX(x_J1 + ((size_t)P + p) * nn * 4),
                pl.joint ? DI(o_one)   // joint: b = s^N c^-e_A already
                         : DX(x_invc + (size_t)p * nn * 4),
                nn, nn, nn, 0};
    p3_nl[p] = {J3_row((size_t)P + p), J4_row((size_t)P + p),
                DX(x_invz + (size_t)p * nl * 4),
                nl, nl, nl, 0};
  }
  std::vector<uint32_t> p3_nl_mod;
  if (K3) {   // the negative-s3 rows: z^e * h2^|s3| * 1  (mod N~)
    p3_nl_mod = recv_of_pair;
    for (size_t k = 0; k < K3; ++k) {
      p3_nl.push_back({J5_row(neg3[k]), J4_row(neg3[k]), DI(o_one), nl, nl, nl, 0});
      p3_nl_mod.push_back(recv_of_pair[neg3[k]]);
    }
  }
  const size_t d_p3nn = put(p3_nn.data(), p3_nn.size() * sizeof(Prod3Operand)),
               d_p3nl = put(p3_nl.data(), p3_nl.size() * sizeof(Prod3Operand)),
               d_p3m = put(recv_of_pair.data(), recv_of_pair.size() * 4),
               d_p3mnl = K3 ? put(p3_nl_mod.data(), p3_nl_mod.size() * 4) : d_p3m;
  // alice hash descriptors + pre-verdicts
  std::vector<uint64_t> ah_n(P), ah_c(P);
  for (uint32_t p = 0; p < P; ++p) {
    ah_n[p] = DI(o_rn + (size_t)recv_of_pair[p] * nl * 4);
    ah_c[p] = DI(o_enc + (size_t)p * nn * 4);
  }
  const size_t d_ahn = put(ah_n.data(), ah_n.size() * 8), d_ahc = put(ah_c.data(), ah_c.size() * 8);
  const size_t d_alpre = put(alice_pre.data(), alice_pre.size());
  // 2-adic halves (even ring-Pedersen / DLog moduli): a^ea * b^eb == c * d^[bit] (mod 2^k)
  std::vector<Pow2Op> p2(n_p2);
  for (uint32_t m = 0; m < Mt; ++m) {
    if (pl.ped_p2_first[m] == ~0u) continue;
    for (uint32_t k = 0; k < M; ++k) {   // T^Z_k == A_k * S^e_k  (S unreduced: pow2 reduces mod 2^k)
      Pow2Op& o = p2[pl.ped_p2_first[m] + k];
      o = Pow2Op{};
      o.a = DI(o_pT + (size_t)m * nl * 4);
      o.a_len = nl;
      o.ea = tz_z ? (uint64_t)(uintptr_t)(tz_z + ((size_t)m * M + k) * zl) : DI(o_pZ + ((size_t)m * M + k) * zl * 4);
      o.ea_len = zl;
      o.c = DI(a_off((size_t)m * M + k));
      o.c_len = nl;
      o.d = DI(o_pSraw + (size_t)m * nl * 4);
      o.d_len = nl;
      o.sel = m * MW * 32 + k;
      o.kbits = ped_tz[m];
    }
  }
  for (uint32_t j = 0; j < J; ++j) {
    if (pl.dlog_p2_first[j] == ~0u) continue;
    for (int which = 0; which < 2; ++which) {   // g^y * ni^e == x
      Pow2Op& o = p2[pl.dlog_p2_first[j] + which];
      o = Pow2Op{};
      o.a = DI((which == 0 ? o_dg : o_dni) + (size_t)j * nl * 4);
      o.a_len = nl;
      o.ea = DI((which == 0 ? o_dy1 : o_dy2) + (size_t)j * yl * 4);
      o.ea_len = yl;
      o.b = DI((which == 0 ? o_dni : o_dg) + (size_t)j * nl * 4);
      o.b_len = nl;
      o.eb = DI(o_de + (size_t)(2 * j + which) * 32);
      o.eb_len = 8;
      o.c = DI((which == 0 ? o_dx1 : o_dx2) + (size_t)j * nl * 4);
      o.c_len = nl;
      o.sel = 0xFFFFFFFFu;
      o.kbits = dlog_tz[j];
    }
  }
  const size_t d_p2 = put(p2.data(), p2.size() * sizeof(Pow2Op));
  if (desc_base + desc.size() > out_off) {
    c->fail("internal: descriptor bound exceeded (%zu > %zu)", desc.size(), desc_bound);
    return FSDKR_E_ARG;
  }
  // fixed-base scratch (power tables, schedules, step counts): its own context buffer
  {
    const int KD = shape_digits(nl);
    const size_t tb = Img::al(FB.table_bytes(KD)), sb = Img::al(FB.sched_bytes()), nb = Img::al(FB.nsteps_bytes());
    uint8_t* fbs = (uint8_t*)c->buf("collect_fb", tb + sb + nb + FB.comb_scratch + 256);
    if (!fbs) {
      c->fail("fsdkr_verify_collect: fixed-base scratch allocation failed");
      return FSDKR_E_OOM;
    }
    pl.fb_table = (uint32_t*)fbs;
    pl.fb_sched = (uint16_t*)(fbs + tb);
    pl.fb_nsteps = (uint32_t*)(fbs + tb + sb);
    pl.fb_comb = FB.cgroups.empty() ? nullptr : fbs + tb + sb + nb;
  }
  pl.d_FB = desc_base;
  clk.lap("descriptors");

  // ---------------- materialise the image in the pinned arena; ONE host->device copy
  const size_t up_bytes = desc_base + desc.size();
  uint8_t* host = c->host_arena(up_bytes);
  if (!host) {
    c->fail("fsdkr_verify_collect: pinned host allocation of %zu bytes failed", up_bytes);
    return FSDKR_E_OOM;
  }
  I.materialize(host);
  memcpy(host + desc_base, desc.data(), desc.size());
  clk.lap("materialize");
  int rc = c->hip_check(hipMemcpyAsync(dev, host, up_bytes, hipMemcpyHostToDevice, c->stream), "H2D batch");
  if (!rc) rc = c->hip_check(hipStreamSynchronize(c->stream), "sync H2D");
  clk.lap("H2D");
  if (rc) return rc;

  // ---------------- record the plan
  pl.out_off = out_off;
  pl.total = total;
  pl.dev = dev;
  pl.o_Q = o_Q; pl.o_enc = o_enc; pl.o_pz = o_pz; pl.o_pu1 = o_pu1; pl.o_pu2 = o_pu2; pl.o_pu3 = o_pu3;
  pl.o_ps1 = o_ps1; pl.o_pA = o_pA; pl.o_az = o_az; pl.o_ae = o_ae; pl.o_vss = o_vss; pl.o_NN = o_NN;
  pl.o_mods = o_mods; pl.o_ckmods = o_ckmods; pl.o_one = o_one;
  pl.d_finfo = o_finfo;
  pl.d_p2 = d_p2;
  pl.n_p2 = n_p2;
  pl.n_mods_nl = n_mods_nl;
  pl.o_epdl = o_epdl; pl.x_pbits = x_pbits; pl.x_ppanic = x_ppanic; pl.x_Bpdl = x_Bpdl; pl.x_gs1 = x_gs1;
  // with a prestarted J1 the GA job is J9 alone, written where J9's rows live
  // (joint: GA = J1 alone, or nothing after a split prestart; slot 2 = J9 at its rows)
  const size_t xs[CollectPlan::NJOB] = {pl.ga_hit ? x_J9 : x_GA, x_GD, pl.joint ? x_J9 : x_J2, x_J5, x_GC};
  const size_t ds[CollectPlan::NJOB] = {d_GA, d_GD, d_J2, d_J5, d_GC};
  const ModexpJob* js[CollectPlan::NJOB] = {pl.joint && pl.ga_hit ? &J2 : &GA, &GD, pl.joint ? &J9 : &J2, &J5, &GC};
  for (int k = 0; k < CollectPlan::NJOB; ++k) {
    pl.x_J[k] = xs[k];
    pl.d_J[k] = ds[k];
    pl.jk32[k] = js[k]->k32;
    pl.jcount[k] = (uint32_t)js[k]->size();
    pl.jbits[k] = js[k]->exp_bits;
  }
  pl.x_invc = x_invc; pl.x_invz = x_invz; pl.x_unn = x_unn; pl.x_uzA = x_uzA; pl.x_uzp = x_uzp;
  pl.x_eq2 = x_eq2; pl.x_eq3 = x_eq3; pl.x_eqck = x_eqck; pl.x_u = x_u; pl.x_w = x_w; pl.x_fel = x_fel;
  pl.x_pdlv = x_pdlv; pl.x_rng = x_rng; pl.x_p2 = x_p2;
  pl.d_bs = d_bs; pl.d_bn = d_bn; pl.d_iynn = d_iynn; pl.d_imnn = d_imnn; pl.d_iynl = d_iynl; pl.d_imnl = d_imnl;
  pl.d_eqnn = d_eqnn; pl.d_eqnnm = d_eqnnm; pl.d_eqnl = d_eqnl; pl.d_eqnlm = d_eqnlm; pl.d_eqck = d_eqck;
  pl.d_eqckm = d_eqckm; pl.d_p3nn = d_p3nn; pl.d_p3nl = d_p3nl; pl.d_p3m = d_p3m; pl.d_ahn = d_ahn; pl.d_ahc = d_ahc;
  pl.d_p3mnl = d_p3mnl;
  pl.n_p3nl = (uint32_t)(P + K3);
  pl.d_alpre = d_alpre;
  pl.n_inv_nn = (uint32_t)inv_y_nn.size();
  pl.r_unn = out_base + x_unn;
  pl.r_uzA = out_base + x_uzA;
  pl.r_uzp = out_base + x_uzp;
  pl.r_pdlv = out_base + x_pdlv;
  pl.r_fel = out_base + x_fel;
  pl.n_eq_nn = (uint32_t)eq_nn.size();
  pl.n_eq_nl = (uint32_t)eq_nl.size();
  pl.n_eq_ck = (uint32_t)eq_ck.size();
  for (Sess& x : pl.ss) x.b = nullptr;   // the caller's buffers are not used after prepare
  c->reuse_mask = (pl.ga_hit ? 1u : 0u) | (pl.fb_hit ? 2u : 0u) | (pl.ck_hit ? 4u : 0u) | (pl.tz_hit ? 8u : 0u);
  c->plan = plan.release();
  return FSDKR_OK;
}

}  // namespace fsdkr
