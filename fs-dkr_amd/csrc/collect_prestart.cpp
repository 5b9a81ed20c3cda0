// fsdkr_collect_prestart[_multi]: the longest device chains of a collect()
// batch -- GA (s2^N, s^N mod N^2 per pair, zk_pdl_with_slack.rs:129-135,
// range_proofs.rs:148) and the fixed-base tables of h1_i, h2_i and every
// ring-Pedersen T -- started from the few fields stage 1 packs, while the caller
// packs the rest.  prepare consumes them when the batch matches.
#include "collect.hpp"

namespace fsdkr {


// The fixed-base table chains of collect()'s FbJob, in its base order: h1_i, h2_i
// of every receiver's DLogStatement (h2: one squaring per exponent bit of s3,
// ~2816 at 2048-bit keys), then every message's ring-Pedersen T, sized by the
// bit lengths of the exponents they serve (PDL / Alice s1, s3|s2; RP Z), on the
// table chain's stream.  `count` sessions in prepare's global order (session
// s's receivers and messages after session s-1's, rows at the widest nl); the
// sessions' row bases come from the GA prestart (g.sess).  A stage 1 without
// the exponents sizes the tables by the slots' widths (s1l, s3l, zl): honest
// exponents fit (s1 < 2^770, s3 < 2^770 N~, Z < phi(N)), and prepare rebuilds
// the tables if one does not.
static int prestart_fb_tables(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count, GaPre& g, uint32_t n, uint32_t P) {
  if (g.sess.size() != count) return FSDKR_OK;
  const uint32_t M = bs[0].m_security;
  bool exact_s = true, exact_z = true;
  uint32_t nl = 0, Mt = 0, s1l = 0, s3l = 0, zl = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    if (!b->recv_ntilde || !b->recv_h1 || !b->recv_h2 || !b->s1l || !b->s3l || !b->ped_T || !b->ped_N || !b->zl ||
        !b->m_security || b->m_security != M)
      return FSDKR_OK;   // stage 1 did not pack them: prepare builds every table
    exact_s = exact_s && b->pdl_s1 && b->pdl_s3 && b->rp_s1 && b->rp_s2;
    exact_z = exact_z && b->ped_Z;
    nl = std::max(nl, b->nl);
    Mt += b->n_refresh + b->n_join;
    s1l = std::max(s1l, b->s1l);
    s3l = std::max(s3l, b->s3l);
    zl = std::max(zl, b->zl);
    for (uint32_t i = 0; i < g.sess[k].n; ++i)
      if (!is_odd(b->recv_ntilde + (size_t)i * b->nl)) return FSDKR_OK;
  }
  // exponent bit bounds: exact from the packed exponents, else their slot widths
  uint32_t bh1 = 1, bh2 = 1, bz = 1;
  if (exact_s) {
    for (uint32_t k = 0; k < count; ++k) {
      const fsdkr_collect_batch* b = bs + k;
      for (size_t p = 0; p < (size_t)g.sess[k].R * g.sess[k].n; ++p) {
        bh1 = std::max(bh1, std::max(hbn::bitlen(b->pdl_s1 + p * b->s1l, b->s1l), hbn::bitlen(b->rp_s1 + p * b->s1l, b->s1l)));
        bh2 = std::max(bh2, std::max(hbn::bitlen(b->pdl_s3 + p * b->s3l, b->s3l), hbn::bitlen(b->rp_s2 + p * b->s3l, b->s3l)));
      }
    }
  } else {
    bh1 = 32 * s1l;
    bh2 = 32 * s3l;
  }
  if (exact_z) {
    for (uint32_t k = 0; k < count; ++k) {
      const fsdkr_collect_batch* b = bs + k;
      const size_t rows = (size_t)(b->n_refresh + b->n_join) * M;
      for (size_t q = 0; q < rows; ++q) bz = std::max(bz, hbn::bitlen(b->ped_Z + q * b->zl, b->zl));
    }
  } else {
    bz = 32 * zl;
  }
  const uint32_t w = fb_window(std::max(std::max(bh1, bh2), bz));
  const FbLayout L = fb_layout(n, Mt, w, bh1, bh2, bz);
  const uint32_t nb = 2 * n + Mt, entries = L.entries, nmod = n + Mt;
  const int KD = shape_digits(nl);
  // the Lim-Lee comb tables of every base class, as prepare's FbJob::plan_comb
  // will choose them (runs of bases with one bound; instances per base: 2 R_s for
  // h1_i / h2_i, M for T_m), built behind the chains on their stream
  std::vector<uint32_t> bbits(nb), bcnt(nb, M);
  for (uint32_t r = 0; r < n; ++r) {
    bbits[r] = bh1;
    bbits[n + Mt + r] = bh2;
  }
  for (uint32_t m = 0; m < Mt; ++m) bbits[n + m] = bz;
  for (const GaPre::Sess& x : g.sess)
    for (uint32_t i = 0; i < x.n; ++i) bcnt[x.rbase + i] = bcnt[n + Mt + x.rbase + i] = 2 * x.R;
  struct PreRun {
    uint32_t b0, b1;
    CombJob cj;
    size_t o_pt = 0, o_bm = 0, o_ul = 0, s_tab = 0;
  };
  std::vector<PreRun> runs;
  size_t comb_bytes = 0, comb_desc = 0;
  if (comb_mode(c) != 0 && (nl == 64 || nl == 96)) {
    for (const auto& r : base_runs(bbits.data(), L.h.data(), nb)) {
      double tot = 0;
      for (uint32_t b = r.first; b < r.second; ++b) tot += bcnt[b];
      const uint32_t nbr = r.second - r.first;
      const CombParams p = comb_choose(bbits[r.first], w, L.h[r.first], comb_mode(c) == 2 ? 1e9 : tot / nbr, nbr,
                                       (size_t)KD * 4, comb_mem_cap(c));
      if (!p.h) continue;
      runs.push_back(PreRun{r.first, r.second, CombJob()});
      runs.back().cj.init(p, nl, nbr, 0);
      runs.back().s_tab = comb_bytes;
      comb_bytes += Img::al(runs.back().cj.table_bytes());
      comb_desc += Img::al((size_t)nbr * 4) * 2 + Img::al(runs.back().cj.ulist.size() * 2);
    }
    if (comb_bytes > comb_mem_cap(c)) {
      runs.clear();
      comb_bytes = comb_desc = 0;
    }
  }
  auto al = Img::al;
  const size_t o_mod = 0, o_h1 = al((size_t)nmod * nl * 4), o_h2 = o_h1 + al((size_t)n * nl * 4),
               o_T = o_h2 + al((size_t)n * nl * 4), o_bp = o_T + al((size_t)Mt * nl * 4),
               o_bl = o_bp + al((size_t)nb * 8), o_bm = o_bl + al((size_t)nb * 4), o_bt = o_bm + al((size_t)nb * 4),
               o_bh = o_bt + al((size_t)nb * 4), o_cd = o_bh + al((size_t)nb * 4), o_tab = o_cd + comb_desc;
  const size_t total = o_tab + (size_t)entries * KD * 4;
  uint8_t* dev = (uint8_t*)c->buf("collect_fb_pre", total);
  uint8_t* cdev = comb_bytes ? (uint8_t*)c->buf("collect_comb_pre", comb_bytes) : nullptr;
  if (!dev || (comb_bytes && !cdev)) {
    c->fail("fsdkr_collect_prestart: device allocation of %zu bytes failed", total + comb_bytes);
    return FSDKR_E_OOM;
  }
  std::vector<uint8_t> img(o_tab, 0);
  {
    size_t o = o_cd;
    for (PreRun& r : runs) {
      const size_t nbr = r.b1 - r.b0;
      r.o_pt = o;
      memcpy(img.data() + o, L.toff.data() + r.b0, nbr * 4);
      o += al(nbr * 4);
      r.o_bm = o;
      memcpy(img.data() + o, L.mod.data() + r.b0, nbr * 4);
      o += al(nbr * 4);
      r.o_ul = o;
      memcpy(img.data() + o, r.cj.ulist.data(), r.cj.ulist.size() * 2);
      o += al(r.cj.ulist.size() * 2);
    }
  }
  uint32_t* mods = reinterpret_cast<uint32_t*>(img.data() + o_mod);   // [Ntilde_i | RP modulus_m]
  uint32_t* H1 = reinterpret_cast<uint32_t*>(img.data() + o_h1);
  uint32_t* H2 = reinterpret_cast<uint32_t*>(img.data() + o_h2);
  uint32_t* TT = reinterpret_cast<uint32_t*>(img.data() + o_T);
  auto rows_to = [&](uint32_t* dst, const uint32_t* src, size_t rows, uint32_t ws) {   // zero-extended to nl
    for (size_t r = 0; r < rows; ++r) memcpy(dst + r * nl, src + r * ws, (size_t)ws * 4);
  };
  for (uint32_t k = 0, mb = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    const size_t rb = g.sess[k].rbase, ns = g.sess[k].n;
    const uint32_t mt = b->n_refresh + b->n_join;
    rows_to(mods + rb * nl, b->recv_ntilde, ns, b->nl);
    rows_to(H1 + rb * nl, b->recv_h1, ns, b->nl);
    rows_to(H2 + rb * nl, b->recv_h2, ns, b->nl);
    rows_to(TT + (size_t)mb * nl, b->ped_T, mt, b->nl);
    for (uint32_t m = 0; m < mt; ++m) ped_modulus(b, m, M, nl, mods + (size_t)(n + mb + m) * nl);
    mb += mt;
  }
  auto* bp = reinterpret_cast<uint64_t*>(img.data() + o_bp);
  for (uint32_t r = 0; r < n; ++r) {   // prepare's base order [h1_i | T_m | h2_i]
    bp[r] = (uint64_t)(uintptr_t)(dev + o_h1 + (size_t)r * nl * 4);
    bp[n + Mt + r] = (uint64_t)(uintptr_t)(dev + o_h2 + (size_t)r * nl * 4);
  }
  for (uint32_t m = 0; m < Mt; ++m) bp[n + m] = (uint64_t)(uintptr_t)(dev + o_T + (size_t)m * nl * 4);
  g.fb_bptr.assign(bp, bp + nb);
  std::vector<uint32_t> blen(nb, nl);
  memcpy(img.data() + o_bl, blen.data(), (size_t)nb * 4);
  memcpy(img.data() + o_bm, L.mod.data(), (size_t)nb * 4);
  memcpy(img.data() + o_bt, L.toff.data(), (size_t)nb * 4);
  memcpy(img.data() + o_bh, L.h.data(), (size_t)nb * 4);
  // every table chain in one launch on launch()'s table-chain stream; launch()'s
  // fixed-base exponent stream waits for it through fb_done
  hipStream_t ts = c->side_stream(8);
  StreamScope scope(c, ts);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(dev, img.data(), img.size(), hipMemcpyHostToDevice, ts), "prestart fb H2D")) ||
      (rc = c->hip_check(hipStreamSynchronize(ts), "prestart fb H2D sync")))
    return rc;
  uint32_t* cons = nullptr;
  // the table chains are the head of the fixed-base chain (tables -> comb levels -> comb
  // exponents): their setup runs one wave per modulus so it starts beside GA's waves
  if ((rc = setup_moduli(c, nl, reinterpret_cast<const uint32_t*>(dev + o_mod), nmod, &cons, "collect_fbpre_nl", 0,
                         true)))
    return rc;
  if (!g.fb_setup && (rc = c->hip_check(hipEventCreateWithFlags(&g.fb_setup, hipEventDisableTiming), "event")))
    return rc;
  if ((rc = c->hip_check(hipEventRecord(g.fb_setup, ts), "event record"))) return rc;   // N~_i constants ready
  if (!g.fb_done && (rc = c->hip_check(hipEventCreateWithFlags(&g.fb_done, hipEventDisableTiming), "event")))
    return rc;
  g.fb_table = reinterpret_cast<uint32_t*>(dev + o_tab);
  g.fb_cons = cons;
  auto U64 = [&](size_t o) { return reinterpret_cast<const uint64_t*>(dev + o); };
  auto U32 = [&](size_t o) { return reinterpret_cast<const uint32_t*>(dev + o); };
  FbTableArgs tall{U64(o_bp), U32(o_bl), U32(o_bm), U32(o_bt), U32(o_bh), cons, g.fb_table, w, nb, 3};
  if ((rc = c->hip_check(launch_fb_table(nl, tall, ts), "prestart fb_table"))) return rc;
  if ((rc = c->hip_check(hipEventRecord(g.fb_done, ts), "event record"))) return rc;
  g.comb_pre.clear();
  for (const PreRun& r : runs) {
    CombDev d{U32(r.o_pt), U32(r.o_bm), nullptr, nullptr, nullptr, nullptr, nullptr,
              reinterpret_cast<const uint16_t*>(dev + r.o_ul), reinterpret_cast<uint32_t*>(cdev + r.s_tab), nullptr};
    if ((rc = comb_build_launch(c, r.cj, d, g.fb_table, cons, ts))) return rc;
    g.comb_pre.push_back(CombPre{r.b0, r.b1, r.cj.p, d.comb});
  }
  if (!runs.empty()) {
    if (!g.comb_done && (rc = c->hip_check(hipEventCreateWithFlags(&g.comb_done, hipEventDisableTiming), "event")))
      return rc;
    if ((rc = c->hip_check(hipEventRecord(g.comb_done, ts), "event record"))) return rc;
  }
  g.ntilde.assign(mods, mods + (size_t)n * nl);
  g.h1.assign(H1, H1 + (size_t)n * nl);
  g.h2.assign(H2, H2 + (size_t)n * nl);
  g.T.assign(TT, TT + (size_t)Mt * nl);
  g.pedmod.assign(mods + (size_t)n * nl, mods + (size_t)nmod * nl);
  g.Mt = Mt;
  g.fb_w = w;
  g.bits_h1 = bh1;
  g.bits_h2 = bh2;
  g.bits_z = bz;
  g.fb_entries = entries;
  g.fb_valid = true;
  (void)P;
  return FSDKR_OK;
}


// The correct-key job GC of a multi-session batch (zk-paillier NiCorrectKeyProof:
// sigma_k^n mod n, k < 11, per message), when stage 1 packed ck_n and ck_sigma:
// it needs nothing else, so it fills the chip beside GA's last chains while the
// caller packs and prepares the rest.  Moduli that are not odd and > 1 get the
// placeholder 3 and no exponent (prepare's verdict for them never reads GC);
// smooth ones run with their own modulus (their verdict is false either way).
static int prestart_ck(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count, GaPre& g) {
  if (g.sess.size() != count) return FSDKR_OK;
  uint32_t ckl = 0, Mt = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    if (!b->ck_n || !b->ck_sigma || !b->ckl || !shape_digits(b->ckl) || b->ck_lens) return FSDKR_OK;
    ckl = std::max(ckl, b->ckl);
    Mt += b->n_refresh + b->n_join;
  }
  if (Mt == 0) return FSDKR_OK;
  g.ck_n.assign((size_t)Mt * ckl, 0u);
  g.ck_sigma.assign((size_t)Mt * CK_M2 * ckl, 0u);
  for (uint32_t k = 0, mb = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    const uint32_t mt = b->n_refresh + b->n_join;
    for (uint32_t m = 0; m < mt; ++m) {
      memcpy(g.ck_n.data() + (size_t)(mb + m) * ckl, b->ck_n + (size_t)m * b->ckl, (size_t)b->ckl * 4);
      for (uint32_t j = 0; j < CK_M2; ++j)
        memcpy(g.ck_sigma.data() + ((size_t)(mb + m) * CK_M2 + j) * ckl, b->ck_sigma + ((size_t)m * CK_M2 + j) * b->ckl,
               (size_t)b->ckl * 4);
    }
    mb += mt;
  }
  auto al = Img::al;
  const size_t o_mod = 0, o_sig = al((size_t)Mt * ckl * 4), o_desc = o_sig + al((size_t)Mt * CK_M2 * ckl * 4);
  const size_t count_i = (size_t)Mt * CK_M2, o_out = o_desc + al(count_i * 32);
  const size_t total = o_out + count_i * ckl * 4;
  uint8_t* dev = (uint8_t*)c->buf("collect_ck_pre", total);
  if (!dev) {
    c->fail("fsdkr_collect_prestart: device allocation of %zu bytes failed", total);
    return FSDKR_E_OOM;
  }
  std::vector<uint8_t> img(o_out, 0);
  uint32_t* mods = reinterpret_cast<uint32_t*>(img.data() + o_mod);
  memcpy(img.data() + o_sig, g.ck_sigma.data(), g.ck_sigma.size() * 4);
  std::vector<uint32_t> ebits(Mt, 0u);
  uint32_t bits = 1;
  for (uint32_t m = 0; m < Mt; ++m) {
    const uint32_t* n = g.ck_n.data() + (size_t)m * ckl;
    uint32_t* dst = mods + (size_t)m * ckl;
    const uint32_t nb = hbn::bitlen(n, ckl);
    if (nb > 1 && is_odd(n)) {
      memcpy(dst, n, (size_t)ckl * 4);
      ebits[m] = nb;
      bits = std::max(bits, nb);
    } else {
      dst[0] = 3;
    }
  }
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };
  ModexpJob GC;
  GC.k32 = ckl;
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t j = 0; j < CK_M2; ++j)   // prepare's GC order: base sigma, exponent n, modulus m
      GC.add(DI(o_sig + ((size_t)m * CK_M2 + j) * ckl * 4), ckl, DI(o_mod + (size_t)m * ckl * 4), ckl, ebits[m], m);
  GC.exp_bits = bits;
  std::vector<uint8_t> desc;
  GC.pack(desc);
  memcpy(img.data() + o_desc, desc.data(), desc.size());
  hipStream_t cs = c->side_stream(9);   // launch()'s correct-key stream
  StreamScope scope(c, cs);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(dev, img.data(), img.size(), hipMemcpyHostToDevice, cs), "prestart ck H2D")) ||
      (rc = c->hip_check(hipStreamSynchronize(cs), "prestart ck H2D sync")))   // img is pageable and local
    return rc;
  uint32_t* cons = nullptr;
  if ((rc = setup_moduli(c, ckl, reinterpret_cast<const uint32_t*>(dev + o_mod), Mt, &cons, "collect_ckpre")))
    return rc;
  g.ck_out = reinterpret_cast<uint32_t*>(dev + o_out);
  if ((rc = launch_modexp_desc(c, ckl, (uint32_t)count_i, bits, dev + o_desc, cons, g.ck_out, cs, "mxt_GCpre", 2, 0)))
    return rc;
  if (!g.ck_done && (rc = c->hip_check(hipEventCreateWithFlags(&g.ck_done, hipEventDisableTiming), "event")))
    return rc;
  if ((rc = c->hip_check(hipEventRecord(g.ck_done, cs), "event record"))) return rc;
  g.ck_l = ckl;
  g.ck_bits = bits;
  g.ck_Mt = Mt;
  g.ck_valid = true;
  return FSDKR_OK;
}


// GA prestart of `count` sessions (one: fsdkr_collect_prestart; many:
// fsdkr_collect_prestart_multi), in prepare's global order: session s's
// receivers and pairs after session s-1's, every row at the widest nl.
int prestart_ga(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count, uint32_t* n_out, uint32_t* P_out) {
  if (!c->ga_pre) c->ga_pre = new GaPre();
  GaPre& g = *reinterpret_cast<GaPre*>(c->ga_pre);
  // an earlier prestart's work that no prepare consumed (a changed batch) may still
  // run and read the buffers this one overwrites: wait for it (a consumed prestart
  // finished before the pipeline that waited on it)
  for (hipEvent_t e : {g.done, g.fb_done, g.comb_done, g.ck_done, g.tz_done})
    if (e) (void)hipEventSynchronize(e);
  g.valid = false;
  g.fb_valid = false;
  g.comb_pre.clear();
  g.ck_valid = false;
  g.tz_valid = false;
  *n_out = *P_out = 0;
  const CollectPlan* running = reinterpret_cast<const CollectPlan*>(c->plan);
  if (running && running->launched) {
    c->fail("fsdkr_collect_prestart: a batch is in flight (call finish first)");
    return FSDKR_E_ARG;
  }
  // a prepared plan that consumed the previous prestart reads its s^N rows and
  // fixed-base tables in place: this prestart overwrites (or reallocates) those
  // buffers, so the plan is dropped (a later launch reports "no prepared batch")
  if (running && (running->ga_hit || running->fb_hit || running->ck_hit || running->tz_hit))
    free_collect_plan(c);
  if (!bs || count == 0) {
    c->fail("fsdkr_collect_prestart: no batch");
    return FSDKR_E_ARG;
  }
  uint32_t nl = 0, n = 0, P = 0;
  std::vector<GaPre::Sess> ss(count);
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    if (!(b->nl == 64 || b->nl == 96) || !b->recv_n || !b->pdl_s2 || !b->rp_s) {
      c->fail("fsdkr_collect_prestart: session %u needs nl, recv_n, pdl_s2 and rp_s", k);
      return FSDKR_E_ARG;
    }
    const uint32_t R = b->n_refresh, ns = b->n_recv ? b->n_recv : R + b->n_join;
    if (R == 0 || ns < R) return FSDKR_OK;   // nothing to start (prepare reports bad shapes)
    for (uint32_t i = 0; i < ns; ++i)
      if (!is_odd(b->recv_n + (size_t)i * b->nl)) return FSDKR_OK;   // prepare reports it
    ss[k] = GaPre::Sess{b->nl, ns, R, (size_t)n, (size_t)P};
    nl = std::max(nl, b->nl);
    n += ns;
    P += R * ns;
  }
  const uint32_t nn = 2 * nl;
  // image: [N^2 | N | s2 | s | descriptors], outputs after it
  auto al = Img::al;
  const size_t o_NN = 0, o_rn = al((size_t)n * nn * 4), o_s2 = o_rn + al((size_t)n * nl * 4),
               o_s = o_s2 + al((size_t)P * nl * 4), o_desc = o_s + al((size_t)P * nl * 4);
  // the lanes launch() would give GA: 32 lanes (KD = 160 constants) for the small
  // batches of a multi-GPU shard, where GA's chain latency is the critical path
  const uint32_t group = ga_lanes(2 * P, nn), per_wave = ga_per_wave(group, nn);
  // descriptors with out_idx, for 2P chains + at most per_wave - 1 pads per receiver
  const size_t desc_bytes = ((size_t)2 * P + (size_t)n * (per_wave ? per_wave - 1 : 0)) * 36,
               o_out = o_desc + al(desc_bytes);
  const size_t total = o_out + ((size_t)2 * P + 1) * nn * 4;   // + the pads' scratch row
  uint8_t* dev = (uint8_t*)c->buf("collect_ga", total);
  if (!dev) {
    c->fail("fsdkr_collect_prestart: device allocation of %zu bytes failed", total);
    return FSDKR_E_OOM;
  }
  // the image in the pinned arena (prepare reuses it later: this H2D completes
  // before the call returns), one fast H2D
  uint8_t* img = c->host_arena(o_out);
  if (!img) {
    c->fail("fsdkr_collect_prestart: pinned host allocation of %zu bytes failed", o_out);
    return FSDKR_E_OOM;
  }
  bool narrow = false;   // a session narrower than nl: its rows are zero-extended
  for (const GaPre::Sess& x : ss) narrow = narrow || x.nl != nl;
  parallel_for(narrow ? o_desc / 4096 + 1 : o_rn / 4096 + 1, 16, [&](size_t c0, size_t c1) {
    const size_t lo = c0 * 4096, hi = std::min(c1 * 4096, narrow ? o_desc : o_rn);
    if (lo < hi) memset(img + lo, 0, hi - lo);
  });
  uint32_t* NN = reinterpret_cast<uint32_t*>(img + o_NN);
  uint32_t* RN = reinterpret_cast<uint32_t*>(img + o_rn);
  uint32_t* S2 = reinterpret_cast<uint32_t*>(img + o_s2);
  uint32_t* S1 = reinterpret_cast<uint32_t*>(img + o_s);
  std::vector<uint32_t> rbits(n);
  std::vector<uint32_t> sess_of_recv(n);
  for (uint32_t k = 0; k < count; ++k) std::fill(sess_of_recv.begin() + ss[k].rbase, sess_of_recv.begin() + ss[k].rbase + ss[k].n, k);
  parallel_for(n, 4, [&](size_t r0, size_t r1) {   // N^2 per receiver: 64 products of 2048-bit N at n = 64, ~5 us each
    for (size_t r = r0; r < r1; ++r) {
      const GaPre::Sess& x = ss[sess_of_recv[r]];
      const uint32_t* Np = bs[sess_of_recv[r]].recv_n + (r - x.rbase) * x.nl;
      const hbn::Limbs N = hbn::from(Np, x.nl);
      hbn::store(hbn::mul(N, N), NN + r * nn, nn);
      memcpy(RN + r * nl, Np, (size_t)x.nl * 4);
      rbits[r] = hbn::bitlen(Np, x.nl);
    }
  });
  uint32_t recvn_max = 1;
  for (uint32_t r = 0; r < n; ++r) recvn_max = std::max(recvn_max, rbits[r]);
  // the moduli go up first and their setup starts at once; the pair rows and the
  // descriptors are laid out and copied on another stream meanwhile, so the setup
  // kernel is off the path to GA's first chain (round 5: one H2D, a host sync, then
  // the setup)
  // the smallest batches (an 8-way n = 64 rank's 960 chains) keep round 5's order:
  // one H2D of the whole image, then the setup; the emulated 8-way n = 64 rank
  // 25.8 -> 21.7 ms with it, while the 4- and 2-way ranks (1 920 / 3 840 chains)
  // ran 2-4 % faster with the split copies (profiles/r06/r06zl_*, r06zm_*)
  const bool overlap = 2 * (size_t)P > 1024;
  hipStream_t gs = c->side_stream(0);                          // GA's stream in launch()
  hipStream_t us = overlap ? c->side_stream(10) : nullptr;   // the bulk copy (the ring-Pedersen prestart's copy stream)
  StreamScope scope(c, gs);
  int rc;
  auto fail_sync = [&](int r) {   // the arena is reused by prepare: no copy may still read it
    (void)hipStreamSynchronize(gs);
    if (us) (void)hipStreamSynchronize(us);
    return r;
  };
  uint32_t* cons = nullptr;
  auto setup = [&]() -> int {
    int r = c->span_begin(gs);   // the call's first device work
    if (!r)
      r = setup_moduli(c, nn, reinterpret_cast<const uint32_t*>(dev + o_NN), n, &cons,
                       group == kWideGroup ? "collect_ga_nn_w" : "collect_ga_nn", group == kWideGroup ? kWideGroup : 0u);
    return r;
  };
  if (overlap) {
    if ((rc = c->hip_check(hipMemcpyAsync(dev, img, o_s2, hipMemcpyHostToDevice, gs), "prestart H2D moduli")) ||
        (rc = setup()))
      return fail_sync(rc);
  }
  for (uint32_t k = 0; k < count; ++k) {   // pair rows, zero-extended to nl
    const GaPre::Sess& x = ss[k];
    const size_t cnt = (size_t)x.R * x.n;
    parallel_for(cnt, 2048, [&](size_t q0, size_t q1) {
      if (x.nl == nl) {
        memcpy(S2 + (x.pbase + q0) * nl, bs[k].pdl_s2 + q0 * nl, (q1 - q0) * nl * 4);
        memcpy(S1 + (x.pbase + q0) * nl, bs[k].rp_s + q0 * nl, (q1 - q0) * nl * 4);
      } else {
        for (size_t q = q0; q < q1; ++q) {
          memcpy(S2 + (x.pbase + q) * nl, bs[k].pdl_s2 + q * x.nl, (size_t)x.nl * 4);
          memcpy(S1 + (x.pbase + q) * nl, bs[k].rp_s + q * x.nl, (size_t)x.nl * 4);
        }
      }
    });
  }
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };
  ModexpJob J1;
  J1.k32 = nn;
  for (int which = 0; which < 2; ++which)   // the order prepare's J1 uses
    for (uint32_t k = 0; k < count; ++k) {
      const GaPre::Sess& x = ss[k];
      for (uint32_t q = 0; q < x.R * x.n; ++q) {
        const size_t p = x.pbase + q, r = x.rbase + q % x.n;
        J1.add(DI((which == 0 ? o_s2 : o_s) + p * nl * 4), nl, DI(o_rn + r * nl * 4), nl, recvn_max, (uint32_t)r);
      }
    }
  // receiver-major, padded to whole waves: the chains of a wave share N_i -> sliding windows
  const uint32_t flags = ga_desc_flags(group_by_exponent(J1, per_wave, (uint32_t)(2 * P)), group);
  std::vector<uint8_t> desc;
  J1.pack(desc);
  if (desc.size() > desc_bytes) {
    c->fail("fsdkr_collect_prestart: GA descriptors %zu > %zu bytes", desc.size(), desc_bytes);
    return fail_sync(FSDKR_E_ARG);
  }
  memcpy(img + o_desc, desc.data(), desc.size());
  memset(img + o_desc + desc.size(), 0, o_out - o_desc - desc.size());
  if (!overlap) {
    if ((rc = c->hip_check(hipMemcpyAsync(dev, img, o_out, hipMemcpyHostToDevice, gs), "prestart H2D")) ||
        (rc = c->hip_check(hipStreamSynchronize(gs), "prestart H2D sync")) || (rc = setup()))
      return fail_sync(rc);
  } else {
    if (!g.ga_rows_up && (rc = c->hip_check(hipEventCreateWithFlags(&g.ga_rows_up, hipEventDisableTiming), "event")))
      return fail_sync(rc);
    if ((rc = c->hip_check(hipMemcpyAsync(dev + o_s2, img + o_s2, o_out - o_s2, hipMemcpyHostToDevice, us),
                           "prestart H2D rows")) ||
        (rc = c->hip_check(hipEventRecord(g.ga_rows_up, us), "event record")) ||
        (rc = c->hip_check(hipStreamWaitEvent(gs, g.ga_rows_up, 0), "stream wait")))
      return fail_sync(rc);
  }
  g.out = reinterpret_cast<uint32_t*>(dev + o_out);
  g.cons = cons;
  g.wide = group == kWideGroup;
  if (!g.ga_setup && (rc = c->hip_check(hipEventCreateWithFlags(&g.ga_setup, hipEventDisableTiming), "event")))
    return rc;
  (void)hipEventRecord(g.ga_setup, gs);   // GA's constants are ready
  // issue priority 2: GA ends ~13 ms before the pipeline's last jobs, which need
  // the issue slots more (n = 64 median of 7 interleaved calls 56.4 -> 55.3 ms vs
  // priority 3, profiles/r03s_ga_prio_ab.jsonl; again 0.5 ms in round 4 with
  // 16-lane GA, profiles/r04/r04g_*)
  const uint32_t gprio = ga_prio();
  // the head of the split chains when the tail can join c^-e in (prepare launches it)
  g.split = ga_split_ok(nn, group, flags);
  SplitArgs head;
  head.lo_bit = kGaSplit;
  if ((rc = launch_modexp_desc(c, nn, (uint32_t)J1.size(), recvn_max, dev + o_desc, cons, g.out, gs, "mxt_GApre", gprio, group,
                               flags, g.split ? &head : nullptr)))
    return fail_sync(rc);
  // the arena is reused by prepare: the copies complete before the call returns
  if (overlap && (rc = c->hip_check(hipStreamSynchronize(us), "prestart H2D sync"))) return fail_sync(rc);
  // the inputs, at each session's own width, for the match in prepare (copied in
  // parallel chunks: 67 MB at n = 256; after GA's launch, off its path)
  size_t words_n = 0, words_p = 0;
  for (const GaPre::Sess& x : ss) {
    words_n += (size_t)x.n * x.nl;
    words_p += (size_t)x.R * x.n * x.nl;
  }
  g.recv_n.resize(words_n);
  g.s2.resize(words_p);
  g.s.resize(words_p);
  {
    struct Cp { uint32_t* dst; const uint32_t* src; size_t words; };
    std::vector<Cp> cps;
    size_t on = 0, op = 0;
    constexpr size_t kChunk = 1u << 18;   // 1 MB pieces
    auto add = [&](uint32_t* dst, const uint32_t* src, size_t words) {
      for (size_t o = 0; o < words; o += kChunk) cps.push_back(Cp{dst + o, src + o, std::min(kChunk, words - o)});
    };
    for (uint32_t k = 0; k < count; ++k) {
      const fsdkr_collect_batch* b = bs + k;
      const GaPre::Sess& x = ss[k];
      const size_t wn = (size_t)x.n * x.nl, wp = (size_t)x.R * x.n * x.nl;
      add(g.recv_n.data() + on, b->recv_n, wn);
      add(g.s2.data() + op, b->pdl_s2, wp);
      add(g.s.data() + op, b->rp_s, wp);
      on += wn;
      op += wp;
    }
    parallel_for(cps.size(), 1, [&](size_t c0, size_t c1) {
      for (size_t q = c0; q < c1; ++q) memcpy(cps[q].dst, cps[q].src, cps[q].words * 4);
    });
  }
  g.ga_group = group;
  g.ga_flags = flags;
  g.ga_count = (uint32_t)J1.size();
  g.ga_bits = recvn_max;
  g.ga_desc = dev + o_desc;
  g.ga_rows = J1.out_idx;
  if (!g.done && (rc = c->hip_check(hipEventCreateWithFlags(&g.done, hipEventDisableTiming), "event"))) return rc;
  if ((rc = c->hip_check(hipEventRecord(g.done, gs), "event record"))) return rc;
  g.nl = nl;
  g.n = n;
  g.R = count == 1 ? bs->n_refresh : 0;
  g.sess = std::move(ss);
  g.valid = true;
  *n_out = n;
  *P_out = P;
  return FSDKR_OK;
}

int collect_prestart_impl(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count) {
  (void)hipGetLastError();   // launch checks read it: start from a clean slate
  uint32_t n = 0, P = 0;
  int rc;
  GaPre* gp = reinterpret_cast<GaPre*>(c->ga_pre);
  const CollectPlan* running = reinterpret_cast<const CollectPlan*>(c->plan);
  if (gp && gp->valid && !(running && running->launched) && ga_pre_matches(c, bs, count)) {
    // a second call for the same batches (a caller that packed GA's fields first and
    // started it at once, then the rest of stage 1): GA keeps running, the missing
    // parts start now
    n = gp->n;
    for (const GaPre::Sess& x : gp->sess) P += x.R * x.n;
  } else {
    if ((rc = prestart_ga(c, bs, count, &n, &P)) || P == 0) return rc;
    gp = reinterpret_cast<GaPre*>(c->ga_pre);
  }
  GaPre& g = *gp;
  if (!g.fb_valid && (rc = prestart_fb_tables(c, bs, count, g, n, P))) return rc;
  return g.ck_valid ? FSDKR_OK : prestart_ck(c, bs, count, g);
}

std::vector<RowsSha> rows_sha256(size_t rows, const std::function<std::pair<const uint32_t*, uint32_t>(size_t)>& row) {
  const size_t blocks = (rows + kShaRows - 1) / kShaRows;
  std::vector<RowsSha> out(blocks);
  std::atomic<bool> ok{true};
  parallel_for(blocks, 1, [&](size_t b0, size_t b1) {
    EVP_MD_CTX* ctx = EVP_MD_CTX_new();
    for (size_t bl = b0; bl < b1 && ctx; ++bl) {
      bool good = EVP_DigestInit_ex(ctx, sha256_md(), nullptr) == 1;
      for (size_t r = bl * kShaRows; r < std::min(rows, (bl + 1) * kShaRows) && good; ++r) {
        const std::pair<const uint32_t*, uint32_t> x = row(r);
        uint32_t top = x.second;
        while (top && x.first[top - 1] == 0) --top;
        good = EVP_DigestUpdate(ctx, &top, 4) == 1 && (!top || EVP_DigestUpdate(ctx, x.first, (size_t)top * 4) == 1);
      }
      unsigned int len = 0;
      if (!good || EVP_DigestFinal_ex(ctx, out[bl].data(), &len) != 1 || len != 32) ok = false;
    }
    if (!ctx) ok = false;
    EVP_MD_CTX_free(ctx);
  });
  if (!ok) out.clear();   // no digest: never equal to a prestart's (callers recompute)
  return out;
}

// fsdkr_collect_prestart_rp: every message's ring-Pedersen T^Z_k (ring_pedersen_proof.rs:144)
// as fixed-base exponents behind the prestarted T tables, once stage 1b packed Z.
// For many small sessions (BASELINE configs[4]) the prestarted GA fills the chip
// for one dispatch round and leaves it mostly idle until the pipeline launches;
// these waves take that window.  (In one n = 64 collect the same early exponents
// slowed the GA chains of the critical path, profiles/r03zc_fb_sched_variants/.)
int collect_prestart_rp_impl(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count) {
  GaPre* gp = reinterpret_cast<GaPre*>(c->ga_pre);
  if (!bs || count == 0) {
    c->fail("fsdkr_collect_prestart_rp: no batch");
    return FSDKR_E_ARG;
  }
  if (!gp || !gp->fb_valid || gp->sess.size() != count || !gp->fb_cons) return FSDKR_OK;   // nothing to start behind
  GaPre& g = *gp;
  g.tz_valid = false;
  const uint32_t M = bs[0].m_security, nl = g.nl, n = g.n, Mt = g.Mt;
  uint32_t zl = 0, mt_sum = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    if (!b->ped_Z || !b->zl || b->m_security != M || b->ped_lens) return FSDKR_OK;
    zl = std::max(zl, b->zl);
    mt_sum += b->n_refresh + b->n_join;
  }
  if (mt_sum != Mt || !M) return FSDKR_OK;
  // the Z rows, zero-extended to zl, in the prestart's message order; their bound
  // must fit the T tables (sized for g.bits_z exponent bits)
  const size_t rows = (size_t)Mt * M;
  auto al = Img::al;
  const size_t o_z = 0, o_out = al(rows * zl * 4), o_sched0 = o_out + al(rows * nl * 4);
  FbJob TZ;
  TZ.k32 = nl;
  for (uint32_t r = 0; r < n; ++r) TZ.add_base(0, nl, r);
  for (uint32_t m = 0; m < Mt; ++m) TZ.add_base(0, nl, n + m);
  for (uint32_t r = 0; r < n; ++r) TZ.add_base(0, nl, r);
  for (uint32_t r = 0; r < n; ++r) {
    TZ.b_bits[r] = g.bits_h1;
    TZ.b_bits[n + Mt + r] = g.bits_h2;
  }
  for (uint32_t m = 0; m < Mt; ++m) TZ.b_bits[n + m] = g.bits_z;
  const size_t o0 = TZ.grow(rows);
  // device buffer first (the descriptors hold device addresses)
  TZ.finalize();   // b_h / b_toff / w / stride only depend on the bases
  if (TZ.w != g.fb_w || TZ.entries != g.fb_entries) return FSDKR_OK;
  // M = 256 exponents per T: a Lim-Lee comb over the same T chains (entries every
  // w squarings: P_m = entry m pstep) takes ~30 % fewer products than BGMW
  // (3072-bit: ~400 instead of ~575 per exponent, comb.hip)
  CombParams cp;
  if (comb_mode(c) != 0)
    cp = comb_choose(g.bits_z, g.fb_w, TZ.b_h[n], comb_mode(c) == 2 ? 1e9 : (double)M, Mt,
                     (size_t)shape_digits(nl) * 4, comb_mem_cap(c));
  CombJob CJ;
  if (cp.h) CJ.init(cp, nl, Mt, (uint32_t)rows);
  const size_t sched_b = cp.h ? CJ.sched_bytes() : rows * (size_t)TZ.stride * 2;
  const size_t o_nsteps = o_sched0 + al(sched_b), o_desc = o_nsteps + al(rows * 4);
  const size_t desc_est = rows * 40 + (size_t)(2 * n + Mt) * 32 + 16 * 256 + CJ.ulist.size() * 2;
  const size_t o_comb = o_desc + al(desc_est);
  const size_t total = o_comb + (cp.h ? al(CJ.table_bytes()) : 0);
  uint8_t* dev = (uint8_t*)c->buf("collect_tz_pre", total);
  if (!dev) {
    c->fail("fsdkr_collect_prestart_rp: device allocation of %zu bytes failed", total);
    return FSDKR_E_OOM;
  }
  std::atomic<bool> fits{true};
  parallel_for(Mt, 64, [&](size_t m0, size_t m1) {
    for (size_t m = m0; m < m1; ++m)
      for (uint32_t k = 0; k < M; ++k) {
        const size_t i = o0 + m * M + k;
        TZ.e_ptr[i] = (uint64_t)(uintptr_t)(dev + o_z + (m * M + k) * zl * 4);
        TZ.e_len[i] = zl;
        TZ.e_base[i] = n + (uint32_t)m;
        TZ.e_mod[i] = n + (uint32_t)m;
        TZ.o_ptr[i] = (uint64_t)(uintptr_t)(dev + o_out + (m * M + k) * nl * 4);
      }
  });
  TZ.finalize();
  std::vector<uint8_t> desc;
  size_t c_ptoff = 0, c_bmod = 0, c_ibase = 0, c_ul = 0;
  if (cp.h) {   // the comb job's descriptors: TZ's instance arrays, T bases only
    auto put = [&](const void* src, size_t bytes) {
      const size_t o = (desc.size() + 255) & ~(size_t)255;
      desc.resize(o + ((bytes + 255) & ~(size_t)255) + 256, 0);
      if (bytes) memcpy(desc.data() + o, src, bytes);
      return o;
    };
    std::vector<uint32_t> ptoff(Mt), bmod(Mt), ibase(rows);
    for (uint32_t m = 0; m < Mt; ++m) {
      ptoff[m] = TZ.b_toff[n + m];
      bmod[m] = n + m;
    }
    for (size_t i = 0; i < rows; ++i) ibase[i] = TZ.e_base[o0 + i] - n;
    c_ptoff = put(ptoff.data(), (size_t)Mt * 4);
    c_bmod = put(bmod.data(), (size_t)Mt * 4);
    c_ibase = put(ibase.data(), rows * 4);
    c_ul = put(CJ.ulist.data(), CJ.ulist.size() * 2);
    TZ.off.e_ptr = put(TZ.e_ptr.data() + o0, rows * 8);
    TZ.off.e_len = put(TZ.e_len.data() + o0, rows * 4);
    TZ.off.e_mod = put(TZ.e_mod.data() + o0, rows * 4);
    TZ.off.o_ptr = put(TZ.o_ptr.data() + o0, rows * 8);
  } else {
    TZ.pack(desc);
  }
  if (desc.size() > o_comb - o_desc) {
    c->fail("fsdkr_collect_prestart_rp: descriptor image larger than planned");
    return FSDKR_E_ARG;
  }
  hipStream_t zs = c->side_stream(10);
  StreamScope scope(c, zs);
  int rc;
  // Z rows: H2D per session (contiguous when the sessions' rows are); prepare reuses
  // the results only for rows equal to these (SHA-256 per block of rows, below)
  std::vector<std::pair<const uint32_t*, uint32_t>> zsess(count);
  std::vector<size_t> zrow0(count + 1, 0);
  size_t row = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    const size_t r = (size_t)(b->n_refresh + b->n_join) * M;
    for (size_t q = 0; q < r; ++q) {
      const uint32_t* z = b->ped_Z + q * b->zl;
      if (hbn::bitlen(z, b->zl) > g.bits_z) fits = false;
    }
    if (b->zl == zl) {
      if ((rc = c->hip_check(hipMemcpyAsync(dev + o_z + row * zl * 4, b->ped_Z, r * zl * 4, hipMemcpyHostToDevice, zs),
                             "prestart rp Z H2D")))
        return rc;
    } else {   // zero-extend row by row
      std::vector<uint32_t> tmp(r * zl, 0u);
      for (size_t q = 0; q < r; ++q) memcpy(tmp.data() + q * zl, b->ped_Z + q * b->zl, (size_t)b->zl * 4);
      if ((rc = c->hip_check(hipMemcpyAsync(dev + o_z + row * zl * 4, tmp.data(), tmp.size() * 4,
                                            hipMemcpyHostToDevice, zs), "prestart rp Z H2D")) ||
          (rc = c->hip_check(hipStreamSynchronize(zs), "prestart rp Z sync")))
        return rc;
    }
    zsess[k] = {b->ped_Z, b->zl};
    row += r;
    zrow0[k + 1] = row;
  }
  if (!fits) return c->hip_check(hipStreamSynchronize(zs), "prestart rp sync");   // prepare sizes its own tables
  if ((rc = c->hip_check(hipMemcpyAsync(dev + o_desc, desc.data(), desc.size(), hipMemcpyHostToDevice, zs),
                         "prestart rp desc H2D")) ||
      (rc = c->hip_check(hipStreamSynchronize(zs), "prestart rp H2D sync")))   // pageable sources
    return rc;
  if (cp.h) {
    const uint8_t* D = dev + o_desc;
    auto U32 = [&](size_t o) { return reinterpret_cast<const uint32_t*>(D + o); };
    auto U64 = [&](size_t o) { return reinterpret_cast<const uint64_t*>(D + o); };
    CombDev cd{U32(c_ptoff), U32(c_bmod), U64(TZ.off.e_ptr), U32(TZ.off.e_len), U32(c_ibase), U32(TZ.off.e_mod),
               U64(TZ.off.o_ptr), reinterpret_cast<const uint16_t*>(D + c_ul),
               reinterpret_cast<uint32_t*>(dev + o_comb), reinterpret_cast<uint16_t*>(dev + o_sched0)};
    const uint32_t* pre_tab = nullptr;   // the T class's tables from the prestart, when they match
    for (const CombPre& q : g.comb_pre)
      if (q.b0 == n && q.b1 == n + Mt && same_params(q.p, cp)) pre_tab = q.tables;
    if ((rc = comb_launch(c, CJ, cd, g.fb_table, g.fb_cons, zs, pre_tab ? g.comb_done : g.fb_done, "comb rp prestart",
                          pre_tab)))
      return rc;
  } else {
    FbDev fd{dev + o_desc, nullptr, reinterpret_cast<uint16_t*>(dev + o_sched0),
             reinterpret_cast<uint32_t*>(dev + o_nsteps)};
    FbPre pre{g.fb_table, g.fb_entries, g.fb_done};
    if ((rc = fb_launch(c, TZ, fd, g.fb_cons, zs, "fb rp prestart", nullptr, &pre))) return rc;
  }
  if (!g.tz_done && (rc = c->hip_check(hipEventCreateWithFlags(&g.tz_done, hipEventDisableTiming), "event")))
    return rc;
  if ((rc = c->hip_check(hipEventRecord(g.tz_done, zs), "event record"))) return rc;
  g.tz_out = reinterpret_cast<uint32_t*>(dev + o_out);
  g.tz_z = reinterpret_cast<const uint32_t*>(dev + o_z);
  g.tz_zl = zl;
  g.tz_Mt = Mt;
  g.tz_M = M;
  g.tz_sha = rows_sha256(row, [&](size_t r) {
    const size_t k = (size_t)(std::upper_bound(zrow0.begin(), zrow0.end(), r) - zrow0.begin()) - 1;
    return std::make_pair(zsess[k].first + (r - zrow0[k]) * zsess[k].second, zsess[k].second);
  });
  g.tz_valid = !g.tz_sha.empty();
  return FSDKR_OK;
}

// does the prestarted GA belong to these sessions (same shapes, same inputs)?
bool ga_pre_matches(const Ctx* c, const fsdkr_collect_batch* bs, uint32_t count) {
  const GaPre* g = reinterpret_cast<const GaPre*>(c->ga_pre);
  if (!g || !g->valid || g->sess.size() != count) return false;
  uint32_t nl = 0;
  for (uint32_t k = 0; k < count; ++k) nl = std::max(nl, bs[k].nl);
  if (g->nl != nl) return false;
  size_t on = 0, op = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    const GaPre::Sess& x = g->sess[k];
    const uint32_t ns = b->n_recv ? b->n_recv : b->n_refresh + b->n_join;
    if (x.nl != b->nl || x.n != ns || x.R != b->n_refresh) return false;
    const size_t rows = (size_t)x.R * x.n * x.nl;
    if (memcmp(g->recv_n.data() + on, b->recv_n, (size_t)x.n * x.nl * 4) != 0 ||
        memcmp(g->s2.data() + op, b->pdl_s2, rows * 4) != 0 || memcmp(g->s.data() + op, b->rp_s, rows * 4) != 0)
      return false;
    on += (size_t)x.n * x.nl;
    op += rows;
  }
  return true;
}

}  // namespace fsdkr
