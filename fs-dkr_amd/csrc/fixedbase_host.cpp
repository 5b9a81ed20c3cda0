// Launch sequencing of fixed-base jobs (fbjob.hpp) and the stand-alone C ABI
// entry fsdkr_fixed_base_modexp.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "fbjob.hpp"
#include "fsdkr/fsdkr.h"
#include "kernels.h"

namespace fsdkr {

static int fb_group(Ctx* c, size_t count) {
  if (c->modexp_group == 2 || c->modexp_group == 4 || c->modexp_group == 8) return (int)c->modexp_group;
  constexpr size_t kLaneCapacity = 256ull * 4 * 2 * 64;   // CUs x SIMDs x resident waves x lanes
  // 4 lanes (L = 18, no in-cycle normalisation) is the most efficient per MAC
  // (8 lanes at n = 64: no faster, profiles/r04/r04g_*)
  return count * 8 <= kLaneCapacity ? 8 : 4;
}

static int comb_path(Ctx* c, const FbJob& j, const FbDev& d, const uint32_t* consts, hipStream_t st,
                     const char* tag, const uint32_t* chain, hipEvent_t ready, hipEvent_t comb_ready);

int fb_launch(Ctx* c, const FbJob& j, const FbDev& d, const uint32_t* consts, hipStream_t st, const char* tag,
              hipStream_t table_st, const FbPre* pre) {
  if (j.count() == 0) return FSDKR_OK;
  const bool comb = !j.cgroups.empty() && d.comb;
  const uint8_t* I = d.img;
  auto U64 = [&](size_t o) { return reinterpret_cast<const uint64_t*>(I + o); };
  auto U32 = [&](size_t o) { return reinterpret_cast<const uint32_t*>(I + o); };
  const uint32_t nb = (uint32_t)j.bases(), ni = (uint32_t)j.count();
  int rc;
  // the table chains (own stream, from t = 0 beside fb_sched), unless prestarted
  hipStream_t ts = table_st ? table_st : st;
  hipEvent_t ready = pre ? pre->ready : nullptr;
  bool own = false;
  if (!pre) {
    FbTableArgs ta{U64(j.off.b_ptr), U32(j.off.b_len), U32(j.off.b_mod), U32(j.off.b_toff), U32(j.off.b_h), consts,
                   d.table, j.w, nb, j.table_prio};
    size_t m = c->tbeg("fb_table", ts);
    rc = c->hip_check(launch_fb_table(j.k32, ta, ts), "fb_table launch");
    c->tend(m, ts);
    if (rc) return rc;
    if (ts != st) {
      if ((rc = c->hip_check(hipEventCreateWithFlags(&ready, hipEventDisableTiming), "event")) ||
          (rc = c->hip_check(hipEventRecord(ready, ts), "event record")))
        return rc;
      own = true;
    }
  }
  if (comb) {
    rc = comb_path(c, j, d, consts, st, tag, pre ? pre->table : d.table, ready, pre ? pre->comb_ready : nullptr);
    if (own) (void)hipEventDestroy(ready);
    return rc;
  }
  FbSchedArgs sa{U64(j.off.e_ptr), U32(j.off.e_len), U32(j.off.i_h), d.sched, d.nsteps, j.stride, j.w, ni};
  if ((rc = c->hip_check(launch_fb_sched(sa, st), "fb_sched launch"))) return rc;
  if (ready) (void)hipStreamWaitEvent(st, ready, 0);
  FbExpArgs ea{U32(j.off.i_toff), U32(j.off.e_mod), U64(j.off.o_ptr), consts, d.table, d.sched, d.nsteps, j.stride,
               ni, pre ? pre->table : nullptr, pre ? pre->entries : 0u};
  size_t m = c->tbeg("fb_exp", st);
  rc = c->hip_check(launch_fb_exp(j.k32, ea, fb_group(c, ni), st), tag);
  c->tend(m, st);
  if (own) (void)hipEventDestroy(ready);
  return rc;
}

CombParams comb_choose(uint32_t bits, uint32_t w, uint32_t avail, double per_base, size_t nbases, size_t entry_bytes,
                       size_t cap) {
  CombParams best;
  if (bits < 64 || per_base < 8.0) return best;
  const uint32_t wb = fb_window(bits);
  double best_cost = 0.9 * ((double)((bits + wb - 1) / wb) + (double)((1u << wb) - 1));
  const uint32_t step = w ? w : 1u;
  for (uint32_t h = 2; h <= 12; ++h)
    for (uint32_t v = 1; v <= 8; ++v) {
      const uint32_t hv = h * v;
      uint32_t b = (bits + hv - 1) / hv;
      b = (b + step - 1) / step * step;
      if ((hv * b + 31) / 32 > 256) continue;                         // comb_sched's exponent window
      if (avail && (uint64_t)(hv - 1) * (b / step) >= avail) continue;   // chain entries the tables need
      if (nbases * ((size_t)v << h) * entry_bytes > cap) continue;
      const double cost = (double)(b - 1) + (double)v * b + (double)v * (double)((1u << h) - 1 - h) / per_base;
      if (cost < best_cost) {
        best_cost = cost;
        best.h = h;
        best.v = v;
        best.b = b;
        best.pstep = w ? b / w : 1u;
      }
    }
  return best;
}

void CombJob::init(const CombParams& pp, uint32_t k, uint32_t nb, uint32_t cnt) {
  p = pp;
  k32 = k;
  nbase = nb;
  count = cnt;
  ulist.clear();
  level_off.assign(1, 0);
  ulist.push_back(0);
  for (uint32_t i = 0; i < p.h; ++i) ulist.push_back((uint16_t)(1u << i));
  level_off.push_back((uint32_t)ulist.size());
  for (uint32_t pc = 2; pc <= p.h; ++pc) {
    for (uint32_t u = 1; u < (1u << p.h); ++u)
      if ((uint32_t)__builtin_popcount(u) == pc) ulist.push_back((uint16_t)u);
    level_off.push_back((uint32_t)ulist.size());
  }
}

// fixed once per process, so a prestart and the prepare after it choose the same
// parameters for the same base classes
size_t comb_mem_cap(Ctx* c) {
  static size_t cap = 0;
  if (!cap) {
    size_t free_b = 0, total_b = 0;
    if (c->hip_check(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo")) return 0;
    cap = std::min(free_b / 4, (size_t)24 << 30);
  }
  return cap;
}

static int comb_sched_launch(Ctx* c, const CombJob& j, const CombDev& d, hipStream_t st) {
  CombSchedArgs sa{d.eptr, d.elen, d.sched, j.p.h, j.p.v, j.p.b, j.count};
  return c->hip_check(launch_comb_sched(sa, st), "comb_sched launch");
}

int comb_build_launch(Ctx* c, const CombJob& j, const CombDev& d, const uint32_t* chain, const uint32_t* consts,
                      hipStream_t st) {
  // the levels are short launches on the exponents' critical path: at issue
  // priority 3 the n = 64 call took 48.2 ms, at 0 51.1 (profiles/r04/r04m_ab_comb_v*)
  constexpr uint32_t prio = 3;
  for (uint32_t lv = 1; lv <= j.p.h; ++lv) {
    const uint32_t o = j.level_off[lv - 1], nu = j.level_off[lv] - o;
    CombBuildArgs ba{chain, d.ptoff, d.bmod, consts, d.comb, d.ulist + o, nu, j.p.h, j.p.v, j.p.pstep, j.nbase, prio,
                     lv == 1 ? 1u : 0u};
    int rc = c->hip_check(launch_comb_build(j.k32, ba, st), "comb_build launch");
    if (rc) return rc;
  }
  return FSDKR_OK;
}

// one comb_exp launch over n jobs of the same width
static int comb_exp_launch(Ctx* c, const CombJob* const* jobs, const CombDev* devs, uint32_t n,
                           const uint32_t* consts, hipStream_t st, const char* tag) {
  CombExpArgs ea{};   // default issue priority (1 or 2 measured no faster, profiles/r04/r04p_*)
  ea.consts = consts;
  size_t total = 0;
  for (uint32_t k = 0; k < n; ++k) {
    const CombJob& j = *jobs[k];
    const CombDev& d = devs[k];
    if (!j.count) continue;
    ea.g[ea.ngroups++] = CombGroupDev{d.comb, d.sched, d.ibase, d.imod, d.optr, j.p.h, j.p.v, j.p.steps(), j.count, 0};
    total += j.count;
  }
  if (!ea.ngroups) return FSDKR_OK;
  size_t m = c->tbeg("comb_exp", st);
  int rc = c->hip_check(launch_comb_exp(jobs[0]->k32, ea, fb_group(c, total), st), tag);
  c->tend(m, st);
  return rc;
}

int comb_launch(Ctx* c, const CombJob& j, const CombDev& d, const uint32_t* chain, const uint32_t* consts,
                hipStream_t st, hipEvent_t chain_ready, const char* tag, const uint32_t* pre_tables) {
  if (!j.count) return FSDKR_OK;
  int rc;
  if ((rc = comb_sched_launch(c, j, d, st))) return rc;
  if (chain_ready) (void)hipStreamWaitEvent(st, chain_ready, 0);
  CombDev dd = d;
  if (pre_tables) {
    dd.comb = const_cast<uint32_t*>(pre_tables);
  } else {
    size_t m = c->tbeg("comb_build", st);
    rc = comb_build_launch(c, j, d, chain, consts, st);
    c->tend(m, st);
    if (rc) return rc;
  }
  const CombJob* jp = &j;
  return comb_exp_launch(c, &jp, &dd, 1, consts, st, tag);
}

// The job's comb groups: every schedule first (they need only the exponents),
// then, once the chains exist, every group's table levels and one comb_exp launch.
static int comb_path(Ctx* c, const FbJob& j, const FbDev& d, const uint32_t* consts, hipStream_t st,
                     const char* tag, const uint32_t* chain, hipEvent_t ready, hipEvent_t comb_ready) {
  const uint8_t* I = d.img;
  auto U64 = [&](size_t o) { return reinterpret_cast<const uint64_t*>(I + o); };
  auto U32 = [&](size_t o) { return reinterpret_cast<const uint32_t*>(I + o); };
  const size_t ng = j.cgroups.size();
  std::vector<CombDev> devs(ng);
  std::vector<const CombJob*> jobs(ng);
  int rc;
  for (size_t k = 0; k < ng; ++k) {
    const FbJob::CombGrp& g = j.cgroups[k];
    devs[k] = CombDev{U32(g.o_ptoff), U32(g.o_bmod), U64(j.off.e_ptr) + g.i0, U32(j.off.e_len) + g.i0,
                      U32(g.o_ibase), U32(j.off.e_mod) + g.i0, U64(j.off.o_ptr) + g.i0,
                      reinterpret_cast<const uint16_t*>(I + g.o_ul),
                      g.pre_tables ? const_cast<uint32_t*>(g.pre_tables) : reinterpret_cast<uint32_t*>(d.comb + g.s_comb),
                      reinterpret_cast<uint16_t*>(d.comb + g.s_sched)};
    jobs[k] = &g.cj;
    if ((rc = comb_sched_launch(c, g.cj, devs[k], st))) return rc;
  }
  if (ready) (void)hipStreamWaitEvent(st, ready, 0);
  bool any_pre = false;
  for (const FbJob::CombGrp& g : j.cgroups) any_pre = any_pre || g.pre_tables;
  if (any_pre && comb_ready) (void)hipStreamWaitEvent(st, comb_ready, 0);
  size_t m = c->tbeg("comb_build", st);
  for (size_t k = 0; k < ng; ++k)
    if (!j.cgroups[k].pre_tables && (rc = comb_build_launch(c, j.cgroups[k].cj, devs[k], chain, consts, st)))
      return rc;
  c->tend(m, st);
  return comb_exp_launch(c, jobs.data(), devs.data(), (uint32_t)ng, consts, st, tag);
}

bool FbJob::plan_comb(int mode, size_t cap, const std::vector<CombPre>* pre) {
  cgroups.clear();
  comb_scratch = 0;
  if (mode == 0 || (k32 != 64 && k32 != 96) || count() == 0) return false;
  // groups: runs of consecutive bases with one exponent bound (hence one chain height)
  std::vector<uint32_t> gid(bases());
  std::vector<CombGrp> gs;
  for (const auto& r : base_runs(b_bits.data(), b_h.data(), (uint32_t)bases())) {
    gs.emplace_back();
    gs.back().b0 = r.first;
    gs.back().b1 = r.second;
    for (uint32_t b = r.first; b < r.second; ++b) gid[b] = (uint32_t)gs.size() - 1;
  }
  // instances grouped by their base's group (stable)
  std::vector<size_t> cnt(gs.size() + 1, 0);
  for (uint32_t b : e_base) ++cnt[gid[b] + 1];
  for (size_t k = 1; k <= gs.size(); ++k) cnt[k] += cnt[k - 1];
  std::vector<size_t> pos(cnt.begin(), cnt.end() - 1);
  bool sorted = true;
  for (size_t i = 1; i < count() && sorted; ++i) sorted = gid[e_base[i]] >= gid[e_base[i - 1]];
  if (!sorted) {
    std::vector<size_t> perm(count());
    for (size_t i = 0; i < count(); ++i) perm[pos[gid[e_base[i]]]++] = i;
    auto apply = [&](auto& v) {
      auto t = v;
      for (size_t i = 0; i < count(); ++i) t[i] = v[perm[i]];
      v.swap(t);
    };
    apply(e_ptr);
    apply(o_ptr);
    apply(e_len);
    apply(e_base);
    apply(e_mod);
    for (size_t i = 0; i < count(); ++i) {
      i_h[i] = b_h[e_base[i]];
      i_toff[i] = b_toff[e_base[i]];
    }
  }
  const size_t KD = (size_t)shape_digits(k32);
  size_t used = 0, ng = 0;
  for (size_t k = 0; k < gs.size(); ++k) {
    CombGrp& g = gs[k];
    g.i0 = cnt[k];
    g.i1 = cnt[k + 1];
    if (g.i1 == g.i0) continue;   // bases without instances need no tables
    const uint32_t nb = g.b1 - g.b0;
    const double per_base = mode == 2 ? 1e9 : (double)(g.i1 - g.i0) / nb;
    const CombParams p = comb_choose(b_bits[g.b0], w, b_h[g.b0], per_base, nb, KD * 4, cap);
    if (!p.h || ++ng > (size_t)kCombGroups) return false;
    g.cj.init(p, k32, nb, (uint32_t)(g.i1 - g.i0));
    for (size_t q = 0; pre && q < pre->size() && !g.pre_tables; ++q)
      if ((*pre)[q].b0 == g.b0 && (*pre)[q].b1 == g.b1 && same_params((*pre)[q].p, p)) g.pre_tables = (*pre)[q].tables;
    if (!g.pre_tables) used += g.cj.table_bytes();
    if (used > cap) return false;
  }
  for (CombGrp& g : gs) {
    if (g.i1 == g.i0) continue;
    g.s_comb = comb_scratch;
    if (!g.pre_tables) comb_scratch += (g.cj.table_bytes() + 255) & ~(size_t)255;
    g.s_sched = comb_scratch;
    comb_scratch += (g.cj.sched_bytes() + 255) & ~(size_t)255;
    cgroups.push_back(std::move(g));
  }
  return true;
}

int comb_mode(const Ctx* c) {
  return (c->flags & FSDKR_CFG_FB_BGMW) ? 0 : (c->flags & FSDKR_CFG_FB_COMB) ? 2 : 1;
}

bool batch_inv_on(const Ctx* c) { return !(c->flags & FSDKR_CFG_INV_EACH); }

// Stand-alone fixed-base job as a comb: the chains P_m = b^(2^(m b)) (fb_table
// with window b, h v entries per base), then comb_launch.  false: not taken.
static bool comb_run(Ctx* c, FbJob& j, const uint32_t* consts, const char* tag, int* rc_out) {
  const int mode = comb_mode(c);
  if (mode == 0 || (j.k32 != 64 && j.k32 != 96)) return false;
  uint32_t bits = 1;
  for (uint32_t b : j.b_bits) bits = std::max(bits, b);
  const int KD = shape_digits(j.k32);
  const double per_base = mode == 2 ? 1e9 : (double)j.count() / (double)j.bases();
  CombParams p = comb_choose(bits, 0, 0, per_base, j.bases(), (size_t)KD * 4, comb_mem_cap(c));
  if (!p.h) return false;
  CombJob cj;
  cj.init(p, j.k32, (uint32_t)j.bases(), (uint32_t)j.count());
  const uint32_t nb = cj.nbase, ni = cj.count, hv = p.h * p.v;
  std::vector<uint32_t> ptoff(nb), bh(nb, hv), ibase(ni);
  for (uint32_t q = 0; q < nb; ++q) ptoff[q] = q * hv;
  for (uint32_t i = 0; i < ni; ++i) ibase[i] = j.e_base[i];
  std::vector<uint8_t> img;
  auto put = [&](const void* src, size_t bytes) {
    const size_t o = (img.size() + 255) & ~(size_t)255;
    img.resize(o + ((bytes + 255) & ~(size_t)255) + 256, 0);
    if (bytes) memcpy(img.data() + o, src, bytes);
    return o;
  };
  const size_t o_bptr = put(j.b_ptr.data(), nb * 8), o_blen = put(j.b_len.data(), nb * 4),
               o_bmod = put(j.b_mod.data(), nb * 4), o_ptoff = put(ptoff.data(), nb * 4), o_bh = put(bh.data(), nb * 4),
               o_eptr = put(j.e_ptr.data(), (size_t)ni * 8), o_elen = put(j.e_len.data(), (size_t)ni * 4),
               o_ibase = put(ibase.data(), (size_t)ni * 4), o_imod = put(j.e_mod.data(), (size_t)ni * 4),
               o_optr = put(j.o_ptr.data(), (size_t)ni * 8), o_ul = put(cj.ulist.data(), cj.ulist.size() * 2);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_chain = al(img.size()), o_comb = o_chain + al((size_t)nb * hv * KD * 4),
               o_sched = o_comb + al(cj.table_bytes()), total = o_sched + al(cj.sched_bytes());
  std::string name = std::string("comb_") + tag;
  uint8_t* dev = (uint8_t*)c->buf(name.c_str(), total);
  if (!dev) {
    c->fail("%s: device allocation failed (%zu bytes)", tag, total);
    *rc_out = FSDKR_E_OOM;
    return true;
  }
  int rc = c->hip_check(hipMemcpyAsync(dev, img.data(), img.size(), hipMemcpyHostToDevice, c->stream), "H2D comb");
  auto U64 = [&](size_t o) { return reinterpret_cast<const uint64_t*>(dev + o); };
  auto U32 = [&](size_t o) { return reinterpret_cast<const uint32_t*>(dev + o); };
  uint32_t* chain = reinterpret_cast<uint32_t*>(dev + o_chain);
  if (!rc) {
    FbTableArgs ta{U64(o_bptr), U32(o_blen), U32(o_bmod), U32(o_ptoff), U32(o_bh), consts, chain, p.b, nb, 0};
    rc = c->hip_check(launch_fb_table(j.k32, ta, c->stream), "comb chain launch");
  }
  if (!rc) {
    CombDev d{U32(o_ptoff), U32(o_bmod), U64(o_eptr), U32(o_elen), U32(o_ibase), U32(o_imod), U64(o_optr),
              reinterpret_cast<const uint16_t*>(dev + o_ul), reinterpret_cast<uint32_t*>(dev + o_comb),
              reinterpret_cast<uint16_t*>(dev + o_sched)};
    rc = comb_launch(c, cj, d, chain, consts, c->stream, nullptr, tag);
  }
  // `img` is a local host buffer: the async copy must finish before it goes away
  if (!rc) rc = c->hip_check(hipStreamSynchronize(c->stream), "sync comb");
  *rc_out = rc;
  return true;
}

int fb_run(Ctx* c, FbJob& j, const uint32_t* consts, const char* tag) {
  if (j.count() == 0) return FSDKR_OK;
  int crc = 0;
  if (comb_run(c, j, consts, tag, &crc)) return crc;
  const int KD = shape_digits(j.k32);
  std::vector<uint8_t> img;
  j.pack(img);
  const size_t o_tab = (img.size() + 255) & ~(size_t)255;
  const size_t o_sch = o_tab + ((j.table_bytes(KD) + 255) & ~(size_t)255);
  const size_t o_ns = o_sch + ((j.sched_bytes() + 255) & ~(size_t)255);
  const size_t total = o_ns + j.nsteps_bytes() + 256;
  std::string name = std::string("fb_") + tag;
  uint8_t* dev = (uint8_t*)c->buf(name.c_str(), total);
  if (!dev) {
    c->fail("%s: device allocation failed (%zu bytes)", tag, total);
    return FSDKR_E_OOM;
  }
  int rc = c->hip_check(hipMemcpyAsync(dev, img.data(), img.size(), hipMemcpyHostToDevice, c->stream), "H2D fb");
  if (rc) return rc;
  FbDev d{dev, (uint32_t*)(dev + o_tab), (uint16_t*)(dev + o_sch), (uint32_t*)(dev + o_ns)};
  rc = fb_launch(c, j, d, consts, c->stream, tag);
  if (rc) return rc;
  // `img` is a local host buffer: the async copy must finish before it goes away
  return c->hip_check(hipStreamSynchronize(c->stream), "sync fb");
}

}  // namespace fsdkr

using namespace fsdkr;

extern "C" int fsdkr_fixed_base_modexp(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t n_bases, const uint32_t* bases,
                                       const uint32_t* base_mod_idx, const uint32_t* mods, uint32_t n_mod,
                                       uint32_t count, const uint32_t* base_idx, const uint32_t* exp,
                                       uint32_t exp_limbs, uint32_t* out) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  if (count == 0) return FSDKR_OK;
  if (!bases || !base_mod_idx || !mods || !base_idx || !exp || !out || !n_bases || !n_mod || !exp_limbs) {
    c->fail("fsdkr_fixed_base_modexp: bad argument");
    return FSDKR_E_ARG;
  }
  if (mod_limbs != 64 && mod_limbs != 96) {
    c->fail("fsdkr_fixed_base_modexp: unsupported modulus width %u limbs", mod_limbs);
    return FSDKR_E_UNSUPPORTED;
  }
  for (uint32_t m = 0; m < n_mod; ++m)
    if (!(mods[(size_t)m * mod_limbs] & 1u)) {
      c->fail("fsdkr_fixed_base_modexp: modulus %u is even", m);
      return FSDKR_E_ARG;
    }
  for (uint32_t b = 0; b < n_bases; ++b)
    if (base_mod_idx[b] >= n_mod) {
      c->fail("fsdkr_fixed_base_modexp: base_mod_idx[%u] out of range", b);
      return FSDKR_E_ARG;
    }
  const size_t nb = (size_t)n_bases * mod_limbs * 4, nm = (size_t)n_mod * mod_limbs * 4;
  const size_t ne = (size_t)count * exp_limbs * 4, no = (size_t)count * mod_limbs * 4;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  uint8_t* d = (uint8_t*)c->buf("fbx_io", al(nb) + al(nm) + al(ne) + al(no));
  if (!d) {
    c->fail("fsdkr_fixed_base_modexp: device allocation failed");
    return FSDKR_E_OOM;
  }
  uint8_t *d_b = d, *d_m = d + al(nb), *d_e = d_m + al(nm), *d_o = d_e + al(ne);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(d_b, bases, nb, hipMemcpyHostToDevice, c->stream), "H2D bases")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_m, mods, nm, hipMemcpyHostToDevice, c->stream), "H2D mods")) ||
      (rc = c->hip_check(hipMemcpyAsync(d_e, exp, ne, hipMemcpyHostToDevice, c->stream), "H2D exp")))
    return rc;
  uint32_t* consts = nullptr;
  if ((rc = setup_moduli(c, mod_limbs, (const uint32_t*)d_m, n_mod, &consts, "fbx"))) return rc;
  FbJob j;
  j.k32 = mod_limbs;
  for (uint32_t b = 0; b < n_bases; ++b)
    j.add_base((uint64_t)(uintptr_t)(d_b + (size_t)b * mod_limbs * 4), mod_limbs, base_mod_idx[b]);
  for (uint32_t i = 0; i < count; ++i) {
    if (base_idx[i] >= n_bases) {
      c->fail("fsdkr_fixed_base_modexp: base_idx[%u] out of range", i);
      return FSDKR_E_ARG;
    }
    const uint32_t* e = exp + (size_t)i * exp_limbs;
    uint32_t bits = 0;
    for (int k = (int)exp_limbs - 1; k >= 0; --k)
      if (e[k]) {
        bits = 32u * (uint32_t)k + 32u - (uint32_t)__builtin_clz(e[k]);
        break;
      }
    j.add(base_idx[i], (uint64_t)(uintptr_t)(d_e + (size_t)i * exp_limbs * 4), exp_limbs, bits,
          (uint64_t)(uintptr_t)(d_o + (size_t)i * mod_limbs * 4));
  }
  j.finalize();
  if ((rc = fb_run(c, j, consts, "fbx"))) return rc;
  if ((rc = c->hip_check(hipMemcpyAsync(out, d_o, no, hipMemcpyDeviceToHost, c->stream), "D2H out"))) return rc;
  return c->sync();
}
