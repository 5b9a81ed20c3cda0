// fsdkr_collect_launch / _finish: the kernel pipeline of a prepared batch on
// the context's streams (ped_hash -> binom -> modexp jobs GA, GD, GC, J2, J5, FB
// -> inverses -> eq_check / prod3 -> alice_hash; pdl_u1, Feldman and the 2-adic
// checks of even moduli beside them) and the one D2H of the verdict words.
#include "collect.hpp"

namespace fsdkr {


// Enqueue the kernel pipeline on the prepared (device-resident) batch.
int collect_launch_impl(Ctx* c) {
  CollectPlan* plan = reinterpret_cast<CollectPlan*>(c->plan);
  if (!plan) {
    c->fail("fsdkr_collect_launch: no prepared batch");
    return FSDKR_E_ARG;
  }
  CollectPlan& pl = *plan;
  if (pl.launched) {
    c->fail("fsdkr_collect_launch: the batch is already in flight (call finish first)");
    return FSDKR_E_ARG;
  }
  const uint32_t nl = pl.nl, nn = pl.nn, P = pl.P, n = pl.n, Mt = pl.Mt, M = pl.M;
  uint8_t* dev = pl.dev;
  uint8_t* const out_base = dev + pl.out_off;
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };
  auto PX = [&](size_t o) { return (uint32_t*)(out_base + o); };
  auto PI = [&](size_t o) { return (const uint32_t*)(dev + o); };
  int rc;
  hipStream_t st = c->stream;
  if (!c->span_armed && (rc = c->span_begin(st))) return rc;   // no prestart: the span starts here
  // the alice pre-verdicts become the initial range verdicts
  if ((rc = c->hip_check(hipMemcpyAsync(out_base + pl.x_rng, dev + pl.d_alpre, P, hipMemcpyDeviceToDevice, st), "D2D")))
    return rc;
  // moduli constants
  uint32_t *cons_nn = nullptr, *cons_nl = nullptr, *cons_ck = nullptr;
  const bool reuse_nn = pl.ga_hit && pl.pre_cons_nn && !pl.pre_cons_wide;
  if (reuse_nn) {   // the prestart's constants of the same N_i^2 rows
    (void)hipStreamWaitEvent(st, pl.ga_setup, 0);
    cons_nn = const_cast<uint32_t*>(pl.pre_cons_nn);
  } else if ((rc = setup_moduli(c, nn, PI(pl.o_NN), n, &cons_nn, "collect_nn"))) {
    return rc;
  }
  if ((rc = setup_moduli(c, nl, PI(pl.o_mods), pl.n_mods_nl, &cons_nl, "collect_nl"))) return rc;
  if ((rc = setup_moduli(c, pl.ckl, PI(pl.o_ckmods), Mt, &cons_ck, "collect_ck"))) return rc;
  // J2 / J5 (256-bit challenge exponents): the 4096-bit J2 at 16 lanes (the
  // quotient-scaled 16-lane shape, with GA at 16 lanes: n = 64 51.0 ms per call,
  // profiles/r04/r04d_ab_lanes_v3), a small J2 (a multi-GPU rank's slice) one
  // instance per wave: its chain is on the critical path of the rank (J2 ->
  // inverses -> equalities); J5 (2048-bit) at 8 lanes (4 lanes measured no
  // better, profiles/r04/r04a_ab_ck_j2j5_v*)
  const uint32_t j2_group = j2_lanes(pl.jcount[2], nn);
  const uint32_t j5_group = 8;
  const uint32_t ga_group = ga_lanes(pl.jcount[0], nn);
  uint32_t* cons_nn_w = nullptr;
  if (ga_group == kWideGroup && pl.jcount[0]) {
    if (pl.ga_hit && pl.pre_cons_nn && pl.pre_cons_wide) {
      (void)hipStreamWaitEvent(st, pl.ga_setup, 0);
      cons_nn_w = const_cast<uint32_t*>(pl.pre_cons_nn);
    } else if ((rc = setup_moduli(c, nn, PI(pl.o_NN), n, &cons_nn_w, "collect_nn_w", kWideGroup))) {
      return rc;
    }
  }
  // ---- stream plan (up to thirteen concurrent lanes of work: give HIP >= 12 hardware
  //      queues, GPU_MAX_HW_QUEUES, or streams share queues and serialise):
  //   side 0  : GA (nn, long exponents, priority)               | start after mod_setup
  //   side 8  : FB table chains (h1, h2, T: the longest dependent chain), top priority
  //   side 1  : FB schedules, then (after the tables) fixed-base exponents
  //   side 3  : ped_hash (serial SHA-256 chains, priority) -> 2-adic checks of even moduli
  //   side 4  : GD (DLog), GC (correct key) -> correct-key equalities
  //   side 6  : Feldman (secp256k1 Horner per pair)
  //   st      : binom x2 | fork | J5, nl inverses | join | eq, prod3, alice  (the PDL
  //             challenges come from prepare's host pass)
  //   side 2  :                    J2 (nn, 256-bit challenges) -> nn inverses
  //   side 5  :                    pdl_u1 (secp256k1)
  //   side 7  :                    Alice's hash prefix (alice_prefix)
  std::vector<hipEvent_t> done;
  // issue-priority levels of the serial chains: GA, FB tables, GD/GC, J5 (measured)
  uint32_t prio[4] = {3, 3, 2, 1};
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
  static const char* tags[CollectPlan::NJOB] = {"mxt_GA", "mxt_GD", "mxt_J2", "mxt_J5", "mxt_GC"};
  auto launch_group = [&](int k, hipStream_t ss, uint32_t pr, uint32_t group, const uint32_t* cons) -> int {
    if (!pl.jcount[k]) return FSDKR_OK;
    return launch_modexp_desc(c, pl.jk32[k], pl.jcount[k], pl.jbits[k], dev + pl.d_J[k], cons, PX(pl.x_J[k]), ss,
                              tags[k], pr, group, pl.jflags[k]);
  };
  // (1) chains that need only the inputs and the moduli constants start at once
  hipEvent_t consts_ready;
  if ((rc = fork(st, &consts_ready))) return rc;
  // per-pair inverses (one per pair, in pair order): Montgomery's simultaneous
  // inversion per receiver where the width has the shape, else one inverse each
  auto pair_inverse = [&](uint32_t k32, const uint64_t* y, const uint64_t* m, uint32_t* out, uint32_t* unit,
                          uint32_t count, hipStream_t s, const char* scratch_tag, const char* what) -> int {
    const size_t kd = inverse_batch_scratch_words(k32);
    if (batch_inv_on(c) && kd && count == P && pl.binv_ngroups) {
      uint32_t* scr = (uint32_t*)c->buf(scratch_tag, (size_t)count * kd * 4);
      if (!scr) {
        c->fail("device allocation failed (inverse scratch)");
        return FSDKR_E_OOM;
      }
      BatchInverseArgs b{y, m, (const uint32_t*)(dev + pl.d_binv_order), (const uint32_t*)(dev + pl.d_binv_gstart),
                         out, unit, scr, pl.binv_ngroups};
      return c->hip_check(launch_inverse_batch(k32, b, s), what);
    }
    InverseArgs a{y, m, out, unit, nullptr, count};
    return c->hip_check(launch_inverse(k32, a, s), what);
  };
  hipEvent_t inv_done = nullptr;
  if (pl.joint) {   // c^-1 mod N^2 of every pair: c's unit flag, and the joint tail's base2
    hipStream_t s2 = c->side_stream(2);
    c->mark("inverse", true, s2);
    rc = pair_inverse(nn, (const uint64_t*)(dev + pl.d_iynn), (const uint64_t*)(dev + pl.d_imnn), PX(pl.x_invc),
                      PX(pl.x_unn), pl.n_inv_nn, s2, "binv_nn", "inverse c");
    c->mark("inverse", false, s2);
    if (rc || (rc = fork(s2, &inv_done))) return rc;
  }
  {  // GA: s2^N, s^N mod N^2 (4096-bit, 2048-bit exponents): the longest chains
    hipStream_t ss = c->side_stream(0);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    // small batches (multi-GPU shards): the h2 fixed-base table chain (2816
    // dependent squarings) is the critical path, so GA steps down one issue
    // priority level below it (8-way shard: 33.4 -> 31.7 ms, tools/ab_hwq.sh)
    if (ga_group >= 16) prio[0] = 2;
    const uint32_t* cga = (ga_group == kWideGroup) ? cons_nn_w : cons_nn;
    if (pl.joint) {
      SplitArgs head, tail;
      head.lo_bit = tail.lo_bit = kGaSplit;
      tail.tail = true;
      tail.d_desc2 = dev + pl.d_desc2;
      if (pl.ga_hit) {   // the prestarted head runs on this stream: its tail follows c^-1
        const CollectPlan::GaTail& t = pl.ga_tail;
        (void)hipStreamWaitEvent(ss, inv_done, 0);
        if ((rc = launch_modexp_desc(c, nn, t.count, t.bits, t.desc, t.cons, t.out, ss, "mxt_GApre", ga_prio(), t.group,
                                     t.flags, &tail)) ||
            (rc = c->hip_check(hipEventRecord(pl.ga_done, ss), "event record")))   // the s^N rows: after the tail
          return rc;
      } else if (pl.jcount[0]) {
        if ((rc = launch_modexp_desc(c, nn, pl.jcount[0], pl.jbits[0], dev + pl.d_J[0], cga, PX(pl.x_J[0]), ss, "mxt_GA",
                                     prio[0], ga_group, pl.jflags[0], &head)))
          return rc;
        (void)hipStreamWaitEvent(ss, inv_done, 0);
        if ((rc = launch_modexp_desc(c, nn, pl.jcount[0], pl.jbits[0], dev + pl.d_J[0], cga, PX(pl.x_J[0]), ss, "mxt_GA",
                                     prio[0], ga_group, pl.jflags[0], &tail)))
          return rc;
      }
      if ((rc = join_later(ss))) return rc;
    } else if ((rc = launch_group(0, ss, prio[0], ga_group, cga)) || (rc = join_later(ss))) {
      return rc;
    }
  }
  {  // FB: h1, h2, T fixed-base tables -> schedules -> exponents
    hipStream_t ss = c->side_stream(1);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    FbDev fd{dev + pl.d_FB, pl.fb_table, pl.fb_sched, pl.fb_nsteps, pl.fb_comb};
    hipStream_t ts = c->side_stream(8);   // own stream: the chain starts beside fb_sched
    (void)hipStreamWaitEvent(ts, consts_ready, 0);
    if ((rc = fb_launch(c, pl.fb, fd, cons_nl, ss, "fb collect", ts, pl.fb_hit ? &pl.fb_pre : nullptr)) ||
        (rc = join_later(ss)))
      return rc;
  }
  {  // ring-Pedersen challenges (one serial SHA-256 chain per message), then the
     // 2-adic halves of even-modulus checks (they read the challenge bits)
    hipStream_t ss = c->side_stream(3);
    PedHashArgs h{PI(pl.o_pA), M, nl, PX(pl.x_pbits), PX(pl.x_ppanic), Mt};
    c->mark("ped_hash", true, ss);
    rc = c->hip_check(launch_ped_hash(h, ss), "ped_hash");
    c->mark("ped_hash", false, ss);
    if (rc) return rc;
    if (pl.n_p2) {
      Pow2Args a{(const Pow2Op*)(dev + pl.d_p2), PX(pl.x_pbits), PX(pl.x_p2), pl.n_p2};
      if ((rc = c->hip_check(launch_pow2_check(a, ss), "pow2_check"))) return rc;
    }
    if ((rc = join_later(ss))) return rc;
  }
  {  // Feldman share checks (inputs only; one Horner chain per pair)
    hipStream_t ss = c->side_stream(6);
    // one Horner chain of t+1 small-scalar steps per pair on one thread: ~2 % of
    // GA's work at n = 256, but a long serial chain; at the default priority it
    // was the last job of an 8-way n = 256 shard rank (64.5 of 85 ms,
    // profiles/r04/r04w_*), so its waves take issue priority
    FeldmanArgs f{PI(pl.o_vss), PI(pl.o_Q), (const FeldmanInfo*)(dev + pl.d_finfo), (uint8_t*)(out_base + pl.x_fel),
                  P, 3};
    c->mark("ec", true, ss);
    rc = c->hip_check(launch_feldman(f, ss), "feldman");
    c->mark("ec", false, ss);
    if (rc || (rc = join_later(ss))) return rc;
  }
  {  // GD: DLog g^y / ni^e (few long chains); GC: correct-key sigma^n (2048-bit
     // exponents, Mt*11 instances) on a stream of its own, so the two latency-bound
     // jobs run side by side
    hipStream_t ss = c->side_stream(4);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    if ((rc = launch_group(1, ss, prio[2], 0, cons_nl)) || (rc = join_later(ss))) return rc;
    ss = c->side_stream(9);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    if (pl.ck_hit) (void)hipStreamWaitEvent(ss, pl.ck_done, 0);   // the prestarted sigma^n rows
    if ((rc = launch_group(4, ss, prio[2], 0, cons_ck))) return rc;
    EqCheckArgs a{(const EqOperand*)(dev + pl.d_eqck), PI(pl.d_eqckm), cons_ck, PX(pl.x_pbits), DI(pl.o_one),
                  PX(pl.x_eqck), pl.n_eq_ck};
    c->mark("eq_check", true, ss);
    rc = c->hip_check(launch_eq_check(pl.ckl, a, ss), "eq_check ck");
    c->mark("eq_check", false, ss);
    if (rc || (rc = join_later(ss))) return rc;
  }
  // (2) the jobs that exponentiate by the PDL challenges (hashed on the host by prepare)
  {
    BinomArgs a{(const uint64_t*)(dev + pl.d_bs), (const uint64_t*)(dev + pl.d_bn), pl.s1l, nl, nn, PX(pl.x_Bpdl), P};
    if ((rc = c->hip_check(launch_binom(a, st), "binom"))) return rc;
    BinomArgs a2{(const uint64_t*)(dev + pl.d_bs) + P, (const uint64_t*)(dev + pl.d_bn) + P, pl.s1l, nl, nn,
                 PX(pl.x_gs1), P};
    if ((rc = c->hip_check(launch_binom(a2, st), "binom"))) return rc;
  }
  hipEvent_t ready;
  if ((rc = fork(st, &ready))) return rc;
  {  // J2: c^e (4096-bit, 256-bit challenges) -> nn inverses
    hipStream_t ss = c->side_stream(2);
    (void)hipStreamWaitEvent(ss, ready, 0);
    // (joint: slot 2 holds J9, (N+1)^s1 for s1 >= N, at the generic lane count)
    if ((rc = launch_group(2, ss, 0, pl.joint ? 0u : j2_group, cons_nn))) return rc;
    if (!pl.joint) {
      InverseArgs a{(const uint64_t*)(dev + pl.d_iynn), (const uint64_t*)(dev + pl.d_imnn), PX(pl.x_invc),
                    PX(pl.x_unn), nullptr, pl.n_inv_nn};
      c->mark("inverse", true, ss);
      rc = c->hip_check(launch_inverse(nn, a, ss), "inverse nn");
      c->mark("inverse", false, ss);
    }
    if (rc || (rc = join_later(ss))) return rc;
  }
  // Alice's hash prefix H(N, N+1, c, z) (inputs only) beside the exponentiations:
  // the pipeline's last kernel, alice_hash, then absorbs only u and w (device span
  // -0.5 ms at n = 64 against the whole hash at the end, profiles/r05/r05ahp_ab/)
  const bool ahp = P != 0;
  uint32_t* ah_state = ahp ? (uint32_t*)c->buf("alice_state", (size_t)P * 32 * 4) : nullptr;
  if (ahp && !ah_state) {
    c->fail("fsdkr_collect_launch: device allocation failed (alice hash state)");
    return FSDKR_E_OOM;
  }
  if (ahp) {
    hipStream_t ss = c->side_stream(7);
    (void)hipStreamWaitEvent(ss, ready, 0);
    AliceHashArgs a{(const uint64_t*)(dev + pl.d_ahn), (const uint64_t*)(dev + pl.d_ahc), PI(pl.o_az), PX(pl.x_u),
                    PX(pl.x_w), PI(pl.o_ae), nl, nn, nl, pl.el, (uint8_t*)(out_base + pl.x_rng), P, ah_state};
    if ((rc = c->hip_check(launch_alice_prefix(a, ss), "alice_prefix")) || (rc = join_later(ss))) return rc;
  }
  {  // PDL u1 on secp256k1 (one Shamir ladder per pair, latency-bound) off the main chain
    hipStream_t ss = c->side_stream(5);
    (void)hipStreamWaitEvent(ss, ready, 0);
    PdlU1Args u{PI(pl.o_ps1), PI(pl.o_epdl), PI(pl.o_Q), PI(pl.o_pu1), pl.s1l, (uint8_t*)(out_base + pl.x_pdlv), P};
    c->mark("ec", true, ss);
    rc = c->hip_check(launch_pdl_u1(u, ss), "pdl_u1");
    c->mark("ec", false, ss);
    if (rc) return rc;
    if ((rc = join_later(ss))) return rc;
  }
  (void)hipEventDestroy(consts_ready);
  (void)hipEventDestroy(ready);
  if (inv_done) (void)hipEventDestroy(inv_done);
  {  // J5: z^e (2048-bit, 256-bit challenges) -> nl inverses
    hipStream_t js = st;
    if ((rc = launch_group(3, js, prio[3], j5_group, cons_nl))) return rc;
    c->mark("inverse", true, js);
    rc = pair_inverse(nl, (const uint64_t*)(dev + pl.d_iynl), (const uint64_t*)(dev + pl.d_imnl), PX(pl.x_invz),
                      PX(pl.x_uzA), P, js, "binv_nl", "inverse nl");
    c->mark("inverse", false, js);
    if (rc) return rc;
    if ((rc = pair_inverse(nl, (const uint64_t*)(dev + pl.d_iynl) + P, (const uint64_t*)(dev + pl.d_imnl) + P,
                           nullptr, PX(pl.x_uzp), P, js, "binv_nl", "inverse nl 2")))
      return rc;
  }
  for (hipEvent_t ev : done) {
    (void)hipStreamWaitEvent(st, ev, 0);
    (void)hipEventDestroy(ev);
  }
  if (pl.ga_hit) (void)hipStreamWaitEvent(st, pl.ga_done, 0);   // the prestarted s^N rows
  if (pl.tz_hit) (void)hipStreamWaitEvent(st, pl.tz_done, 0);   // the prestarted ring-Pedersen T^Z rows
  // exact products (first: the negative-s3 pairs' u3 check reads rows of x_w), equality checks
  {
    Prod3Args pa{(const Prod3Operand*)(dev + pl.d_p3nn), PI(pl.d_p3m), cons_nn, PX(pl.x_u), P};
    if ((rc = c->hip_check(launch_prod3(nn, pa, st), "prod3 nn"))) return rc;
    Prod3Args pb{(const Prod3Operand*)(dev + pl.d_p3nl), PI(pl.d_p3mnl), cons_nl, PX(pl.x_w), pl.n_p3nl};
    if ((rc = c->hip_check(launch_prod3(nl, pb, st), "prod3 nl"))) return rc;
    EqCheckArgs a{(const EqOperand*)(dev + pl.d_eqnn), PI(pl.d_eqnnm), cons_nn, PX(pl.x_pbits), DI(pl.o_one),
                  PX(pl.x_eq2), pl.n_eq_nn};
    c->mark("eq_check", true);
    rc = c->hip_check(launch_eq_check(nn, a, st), "eq_check nn");
    c->mark("eq_check", false);
    if (rc) return rc;
    // eq_nl outputs: [u3 P | RP Mt*M | DLog 2J] contiguous from x_eq3
    EqCheckArgs b1{(const EqOperand*)(dev + pl.d_eqnl), PI(pl.d_eqnlm), cons_nl, PX(pl.x_pbits), DI(pl.o_one),
                   PX(pl.x_eq3), pl.n_eq_nl};
    c->mark("eq_check", true);
    rc = c->hip_check(launch_eq_check(nl, b1, st), "eq_check nl");
    c->mark("eq_check", false);
    if (rc) return rc;
  }
  {
    AliceHashArgs a{(const uint64_t*)(dev + pl.d_ahn), (const uint64_t*)(dev + pl.d_ahc), PI(pl.o_az), PX(pl.x_u),
                    PX(pl.x_w), PI(pl.o_ae), nl, nn, nl, pl.el, (uint8_t*)(out_base + pl.x_rng), P, ah_state};
    c->mark("alice_hash", true);
    rc = c->hip_check(launch_alice_hash(a, st), "alice_hash");
    c->mark("alice_hash", false);
    if (rc) return rc;
  }
  if (c->span_armed && (rc = c->hip_check(hipEventRecord(c->span_end, st), "span event record"))) return rc;
  pl.launched = true;
  return FSDKR_OK;
}

static bool caps_ok(const fsdkr_verdicts& v, const Sess& x) {
  return v.feldman && v.pdl && v.range && v.ped && v.ck && (x.J == 0 || v.dlog) && v.cap_pairs >= x.P &&
         v.cap_msgs >= x.Mt && v.cap_joins >= x.J;
}

// Wait for the launched pipeline, read the verdict words back, assemble per session.
int collect_finish_impl(Ctx* c, fsdkr_verdicts* out, uint32_t count) {
  CollectPlan* plan = reinterpret_cast<CollectPlan*>(c->plan);
  if (!plan || !plan->launched) {
    c->fail("fsdkr_collect_finish: no launched batch");
    return FSDKR_E_ARG;
  }
  CollectPlan& pl = *plan;
  if (!out || count != pl.S) {
    c->fail("fsdkr_collect_finish: %u verdict blocks for %u sessions", count, pl.S);
    return FSDKR_E_ARG;
  }
  for (uint32_t s = 0; s < count; ++s)
    if (!caps_ok(out[s], pl.ss[s])) {
      c->fail("fsdkr_collect_finish: session %u: verdict arrays missing or too small", s);
      return FSDKR_E_ARG;
    }
  pl.launched = false;
  const uint32_t P = pl.P, Mt = pl.Mt, M = pl.M;
  uint8_t* const out_base = pl.dev + pl.out_off;
  hipStream_t st = c->stream;
  const std::vector<uint32_t>& e_pdl = pl.e_pdl;
  std::vector<uint32_t> ppanic(Mt), unn(pl.n_inv_nn), uzA(P), uzp(P), eq2(P), eq3(pl.n_eq_nl),
      eqck(pl.n_eq_ck), p2(pl.n_p2);
  std::vector<uint8_t> fel(P), pdlv(P), rng(P);
  int rc;
  auto D2Hp = [&](void* dst, const void* src, size_t bytes) {
    if (!bytes) return (int)FSDKR_OK;
    return c->hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st), "D2H verdicts");
  };
  auto D2H = [&](void* dst, size_t off, size_t bytes) { return D2Hp(dst, out_base + off, bytes); };
  if ((rc = D2H(ppanic.data(), pl.x_ppanic, Mt * 4)) ||
      (rc = D2Hp(unn.data(), pl.r_unn, unn.size() * 4)) || (rc = D2Hp(uzA.data(), pl.r_uzA, P * 4)) ||
      (rc = D2Hp(uzp.data(), pl.r_uzp, P * 4)) || (rc = D2H(eq2.data(), pl.x_eq2, P * 4)) ||
      (rc = D2H(eq3.data(), pl.x_eq3, eq3.size() * 4)) || (rc = D2H(eqck.data(), pl.x_eqck, eqck.size() * 4)) ||
      (rc = D2H(p2.data(), pl.x_p2, p2.size() * 4)) || (rc = D2Hp(fel.data(), pl.r_fel, P)) ||
      (rc = D2Hp(pdlv.data(), pl.r_pdlv, P)) || (rc = D2H(rng.data(), pl.x_rng, P)))
    return rc;
  if ((rc = c->sync())) return rc;
  if (c->span_armed) {
    c->span_armed = false;
    if (hipEventElapsedTime(&c->span_ms, c->span_beg, c->span_end) != hipSuccess) {
      c->span_ms = -1.0f;
      (void)hipGetLastError();   // best effort: not reported by the next launch check
    }
  }
  // PDL unit test of c: c^eA witnesses it unless eA == 0 / the Alice proof was rejected early
  // (joint: unn is c's own unit flag)
  std::vector<uint32_t> unit_c_pdl(unn.begin(), unn.begin() + P);
  for (size_t k = 0; k < pl.cpdl_extra.size(); ++k) unit_c_pdl[pl.cpdl_extra[k]] = unn[P + k];
  for (uint32_t s = 0; s < count; ++s) {
    const Sess& x = pl.ss[s];
    fsdkr_verdicts& v = out[s];
    for (uint32_t lp = 0; lp < x.P; ++lp) {
      const uint32_t p = x.pbase + lp;
      bool ez = true;
      for (int k = 0; k < 8; ++k) ez = ez && e_pdl[(size_t)p * 8 + k] == 0;
      // reference panics (mod_inv(..).unwrap(), zk_pdl_with_slack.rs:180) when e != 0 and c or z is not a unit
      const bool panic = !ez && (!unit_c_pdl[p] || !uzp[p]);
      uint8_t bits = (uint8_t)(pdlv[p] & 1u);
      if (eq2[p]) bits |= 2;
      if (eq3[p]) bits |= 4;
      if (panic) bits |= 8;
      v.pdl[lp] = bits;
      v.feldman[lp] = fel[p];
      // Alice: pre-checks, invertibility of z^e and c^e, transcript hash (range_proofs.rs:125-163);
      // joint: c^e is a unit iff e == 0 or c is
      const bool unit_ce = pl.joint ? (pl.ae_zero[p] || unn[p]) : unn[p] != 0;
      v.range[lp] = (rng[p] && unit_ce && uzA[p]) ? 1 : 0;
    }
    for (uint32_t lm = 0; lm < x.Mt; ++lm) {
      const uint32_t m = x.mbase + lm;
      uint32_t* eqm = &eq3[P + (size_t)m * M];
      if (pl.ped_mode[m] == 1)
        for (uint32_t k = 0; k < M; ++k) eqm[k] = 1;   // odd part 1
      if (pl.ped_p2_first[m] != ~0u)
        for (uint32_t k = 0; k < M; ++k) eqm[k] = eqm[k] && p2[pl.ped_p2_first[m] + k];
      // panic index: challenge shorter than M bits (BitVec) or Z shorter than M, whichever first
      uint32_t pw = ppanic[m];
      if (pl.ped_zlen[m] < M) pw = pw ? std::min(pw, pl.ped_zlen[m] + 1) : pl.ped_zlen[m] + 1;
      v.ped[lm] = pl.ped_mode[m] == 2 ? 2 : ped_verdict(eqm, M, pw);   // A short / modulus 0: panic
      bool ck = pl.ck_pre[m];
      for (uint32_t k = 0; k < CK_M2; ++k) ck = ck && eqck[(size_t)m * CK_M2 + k];
      v.ck[lm] = pl.ck_short[m] ? 2 : ((ck || pl.ck_one[m]) ? 1 : 0);
    }
    for (uint32_t lj = 0; lj < x.J; ++lj) {
      const uint32_t j = x.jbase + lj;
      const size_t base = P + (size_t)Mt * M + 2 * (size_t)j;
      uint8_t d = 0;
      for (int which = 0; which < 2; ++which) {
        bool ok = (pl.dlog_pre[j] >> which) & 1u;
        ok = ok && (pl.dlog_trivial[j] || eq3[base + which]);
        if (pl.dlog_p2_first[j] != ~0u) ok = ok && p2[pl.dlog_p2_first[j] + which];
        if (ok) d |= (uint8_t)(1u << which);
      }
      v.dlog[lj] = d;
    }
  }
  return FSDKR_OK;
}

}  // namespace fsdkr
