// Host side of a fixed-base exponentiation job (fixedbase.hip): bases shared by
// many exponents, each instance writing base^exp mod N to its own address.
// Used by the collect() pipeline (h1_i, h2_i, ring-Pedersen T) and by the
// stand-alone ring-Pedersen / fixed-base entry points.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <utility>
#include <vector>

#include "ctx.hpp"
#include "fixedbase.h"

namespace fsdkr {

// Lim-Lee comb job (comb.hip) over `nbase` bases whose squaring chains are
// already laid out in `chain` (P_m of base q at entry ptoff[q] + m * pstep):
// the u order of the table levels (level 1: 0 and the single bits, then by
// popcount) and the byte sizes of its scratch.
struct CombJob {
  CombParams p;
  uint32_t k32 = 0, nbase = 0, count = 0;
  std::vector<uint16_t> ulist;
  std::vector<uint32_t> level_off;   // [h + 1]: level p's u values at [level_off[p-1], level_off[p])
  void init(const CombParams& pp, uint32_t k, uint32_t nb, uint32_t cnt);
  size_t table_bytes() const { return (size_t)nbase * p.entries_per_base() * shape_digits(k32) * 4; }
  size_t sched_bytes() const { return (size_t)count * p.steps() * 2; }
};
// Comb tables built ahead (fsdkr_collect_prestart) for the bases [b0, b1) of a
// job laid out like collect()'s FbJob, with parameters p.
struct CombPre {
  uint32_t b0 = 0, b1 = 0;
  CombParams p;
  const uint32_t* tables = nullptr;
};
inline bool same_params(const CombParams& a, const CombParams& b) {
  return a.h == b.h && a.v == b.v && a.b == b.b && a.pstep == b.pstep;
}
// base classes of a fixed-base job: runs of consecutive bases with one exponent
// bound and chain height ([first, last) pairs)
inline std::vector<std::pair<uint32_t, uint32_t>> base_runs(const uint32_t* bits, const uint32_t* h, uint32_t nb) {
  std::vector<std::pair<uint32_t, uint32_t>> r;
  for (uint32_t b = 0; b < nb; ++b) {
    if (r.empty() || bits[b] != bits[r.back().first] || h[b] != h[r.back().first]) r.emplace_back(b, b);
    r.back().second = b + 1;
  }
  return r;
}

struct FbJob {
  uint32_t k32 = 0;
  uint32_t table_prio = 3;   // s_setprio of the table chain (a long serial chain, few waves)
  // bases
  std::vector<uint64_t> b_ptr;
  std::vector<uint32_t> b_len, b_mod, b_bits;
  // instances
  std::vector<uint64_t> e_ptr, o_ptr;
  std::vector<uint32_t> e_len, e_base, e_mod;
  // finalize() results
  uint32_t w = 1, stride = 0;
  size_t entries = 0;
  std::vector<uint32_t> b_h, b_toff, i_h, i_toff;
  // comb plan (plan_comb, after finalize): the instances grouped by base class
  // (runs of bases with one exponent bound, e.g. collect()'s [h1_i | T_m | h2_i]),
  // each group a Lim-Lee comb over its bases' BGMW chains (P_m = entry m pstep)
  struct CombGrp {
    uint32_t b0 = 0, b1 = 0;   // bases [b0, b1)
    size_t i0 = 0, i1 = 0;     // instances [i0, i1)
    CombJob cj;
    const uint32_t* pre_tables = nullptr;                     // built ahead (CombPre): no table levels
    size_t o_ptoff = 0, o_bmod = 0, o_ibase = 0, o_ul = 0;   // packed image offsets
    size_t s_comb = 0, s_sched = 0;                           // comb scratch offsets
  };
  std::vector<CombGrp> cgroups;   // non-empty: fb_launch runs the job as combs
  size_t comb_scratch = 0;
  // plan the comb groups (reorders the instances by group); false: BGMW.  pre:
  // tables built ahead for these bases (a group with the same bases and
  // parameters takes them)
  bool plan_comb(int mode, size_t cap, const std::vector<CombPre>* pre = nullptr);

  uint32_t add_base(uint64_t ptr, uint32_t len, uint32_t mod) {
    b_ptr.push_back(ptr);
    b_len.push_back(len);
    b_mod.push_back(mod);
    b_bits.push_back(1);
    return (uint32_t)b_ptr.size() - 1;
  }
  // ebits: bound on the exponent's bit length (sizes the base's table)
  void add(uint32_t base, uint64_t exp, uint32_t elen, uint32_t ebits, uint64_t out) {
    e_ptr.push_back(exp);
    e_len.push_back(elen);
    e_base.push_back(base);
    e_mod.push_back(b_mod[base]);
    o_ptr.push_back(out);
    b_bits[base] = std::max(b_bits[base], std::max(ebits, 1u));
  }
  // append `cnt` instances to be filled in place (e_ptr, e_len, e_base, e_mod,
  // o_ptr at [offset, offset + cnt)); the caller raises b_bits itself
  size_t grow(size_t cnt) {
    const size_t o = count();
    e_ptr.resize(o + cnt);
    e_len.resize(o + cnt);
    e_base.resize(o + cnt);
    e_mod.resize(o + cnt);
    o_ptr.resize(o + cnt);
    return o;
  }
  size_t count() const { return e_ptr.size(); }
  size_t bases() const { return b_ptr.size(); }

  void finalize() {
    uint32_t maxb = 1;
    for (uint32_t b : b_bits) maxb = std::max(maxb, b);
    w = fb_window(maxb);
    b_h.resize(bases());
    b_toff.resize(bases());
    entries = 0;
    uint32_t hmax = 1;
    for (size_t b = 0; b < bases(); ++b) {
      b_h[b] = std::max(1u, (b_bits[b] + w - 1) / w);
      b_toff[b] = (uint32_t)entries;
      entries += b_h[b];
      hmax = std::max(hmax, b_h[b]);
    }
    stride = (hmax + (1u << w) + 1) & ~1u;
    i_h.resize(count());
    i_toff.resize(count());
    for (size_t i = 0; i < count(); ++i) {
      i_h[i] = b_h[e_base[i]];
      i_toff[i] = b_toff[e_base[i]];
    }
  }

  // device image: descriptor arrays (inputs) appended to `img` at 256-byte
  // alignment; offsets recorded for bind()
  struct Offsets {
    size_t b_ptr, b_len, b_mod, b_toff, b_h, e_ptr, e_len, i_h, i_toff, e_mod, o_ptr;
  } off{};
  void pack(std::vector<uint8_t>& img) {
    auto put = [&](const void* src, size_t bytes) {
      const size_t o = (img.size() + 255) & ~(size_t)255;
      img.resize(o + ((bytes + 255) & ~(size_t)255) + 256, 0);
      if (bytes) memcpy(img.data() + o, src, bytes);
      return o;
    };
    off.b_ptr = put(b_ptr.data(), b_ptr.size() * 8);
    off.b_len = put(b_len.data(), b_len.size() * 4);
    off.b_mod = put(b_mod.data(), b_mod.size() * 4);
    off.b_toff = put(b_toff.data(), b_toff.size() * 4);
    off.b_h = put(b_h.data(), b_h.size() * 4);
    off.e_ptr = put(e_ptr.data(), e_ptr.size() * 8);
    off.e_len = put(e_len.data(), e_len.size() * 4);
    off.i_h = put(i_h.data(), i_h.size() * 4);
    off.i_toff = put(i_toff.data(), i_toff.size() * 4);
    off.e_mod = put(e_mod.data(), e_mod.size() * 4);
    off.o_ptr = put(o_ptr.data(), o_ptr.size() * 8);
    for (CombGrp& g : cgroups) {
      std::vector<uint32_t> ib(g.i1 - g.i0);
      for (size_t i = g.i0; i < g.i1; ++i) ib[i - g.i0] = e_base[i] - g.b0;
      g.o_ptoff = put(b_toff.data() + g.b0, (size_t)(g.b1 - g.b0) * 4);
      g.o_bmod = put(b_mod.data() + g.b0, (size_t)(g.b1 - g.b0) * 4);
      g.o_ibase = put(ib.data(), ib.size() * 4);
      g.o_ul = put(g.cj.ulist.data(), g.cj.ulist.size() * 2);
    }
  }
  // bytes pack() adds for the comb groups (an upper bound, alignment included)
  size_t comb_desc_bytes() const {
    size_t s = 0;
    for (const CombGrp& g : cgroups) s += (size_t)(g.b1 - g.b0) * 8 + (g.i1 - g.i0) * 4 + g.cj.ulist.size() * 2 + 4 * 512;
    return s;
  }
  // scratch the kernels write: table, schedules, step counts
  size_t table_bytes(int KD) const { return entries * (size_t)KD * 4; }
  size_t sched_bytes() const { return count() * (size_t)stride * 2; }
  size_t nsteps_bytes() const { return count() * 4; }
};

// Device addresses of one packed FbJob.
struct FbDev {
  const uint8_t* img = nullptr;   // base of the packed descriptor image
  uint32_t* table = nullptr;
  uint16_t* sched = nullptr;
  uint32_t* nsteps = nullptr;
  uint8_t* comb = nullptr;        // comb scratch (FbJob::comb_scratch bytes) when cgroups is set
};

// table, schedule and exponent kernels.  table_st: stream of the table chain
// (nullptr = st; the schedule kernel runs beside it on st), and fb_exp on st
// waits for it.  pre: every base's table was built ahead into pre->table
// (fsdkr_collect_prestart, same layout), complete at pre->ready.
struct FbPre {
  const uint32_t* table = nullptr;
  uint32_t entries = 0;
  hipEvent_t ready = nullptr;
  hipEvent_t comb_ready = nullptr;   // the CombPre tables (FbJob::CombGrp::pre_tables) exist
};
int fb_launch(Ctx* c, const FbJob& j, const FbDev& d, const uint32_t* consts, hipStream_t st, const char* tag,
              hipStream_t table_st = nullptr, const FbPre* pre = nullptr);

// Device inputs of a CombJob: per base ptoff / mod_idx, per instance exponent
// address / limbs, table set, modulus row, destination; the ulist upload; scratch.
struct CombDev {
  const uint32_t *ptoff, *bmod;
  const uint64_t* eptr;
  const uint32_t *elen, *ibase, *imod;
  const uint64_t* optr;
  const uint16_t* ulist;
  uint32_t* comb;
  uint16_t* sched;
};
// schedules on st, then (after chain_ready, if given) the table levels and the
// exponentiations, all on st; pre_tables: the tables exist (at chain_ready), no levels
int comb_launch(Ctx* c, const CombJob& j, const CombDev& d, const uint32_t* chain, const uint32_t* consts,
                hipStream_t st, hipEvent_t chain_ready, const char* tag, const uint32_t* pre_tables = nullptr);
// the table levels alone (a prestart builds them ahead of the exponents)
int comb_build_launch(Ctx* c, const CombJob& j, const CombDev& d, const uint32_t* chain, const uint32_t* consts,
                      hipStream_t st);
// device bytes the comb tables may take (a fraction of the free memory)
size_t comb_mem_cap(Ctx* c);
// the context's fixed-base engine: 0 = BGMW only (FSDKR_CFG_FB_BGMW), 2 = the comb
// whenever it is possible (FSDKR_CFG_FB_COMB), else (default, 1) the comb where
// comb_choose finds it cheaper
struct Ctx;
int comb_mode(const Ctx* c);
// upload + launch + wait (stand-alone callers)
int fb_run(Ctx* c, FbJob& j, const uint32_t* consts, const char* tag);

}  // namespace fsdkr
