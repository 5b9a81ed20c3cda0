// Fixed-base (BGMW) exponentiation kernels (fixedbase.hip): argument blocks and
// launchers.  Device addresses are uint64_t so the host can build descriptor
// arrays and upload them with the rest of a batch image.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace fsdkr {

struct FbTableArgs {            // table[toff[b] + j] = base_b^(2^(w j)) * R mod N, j < h[b]
  const uint64_t* base_ptr;     // [count]
  const uint32_t* base_len;     // [count] limbs
  const uint32_t* mod_idx;      // [count] row of consts
  const uint32_t* toff;         // [count] first table entry of the base
  const uint32_t* h;            // [count] entries (windows) of the base
  const uint32_t* consts;       // mod_setup rows
  uint32_t* table;              // [sum h][KD] digits
  uint32_t w;
  uint32_t count;
  uint32_t prio;                // s_setprio level of the chain's waves
};

struct FbSchedArgs {            // per-instance BGMW product schedule
  const uint64_t* exp_ptr;      // [count]
  const uint32_t* exp_len;      // [count] limbs
  const uint32_t* h;            // [count] windows of the instance's base table
  uint16_t* sched;              // [count][stride]
  uint32_t* nsteps;             // [count]
  uint32_t stride;              // >= max h + 2^w - 1
  uint32_t w;
  uint32_t count;
};

struct FbExpArgs {              // out = base^exp mod N from the base's table
  const uint32_t* toff;         // [count] first table entry of the instance's base
  const uint32_t* mod_idx;      // [count]
  const uint64_t* out_ptr;      // [count] destination (K32 limbs)
  const uint32_t* consts;
  const uint32_t* table;
  const uint16_t* sched;        // from fb_sched
  const uint32_t* nsteps;
  uint32_t stride;
  uint32_t count;
  // entries [0, split) live in table_pre (tables built ahead by
  // fsdkr_collect_prestart), the rest in `table` from entry `split` on
  const uint32_t* table_pre;
  uint32_t split;
};

uint32_t fb_window(uint32_t ebits);
hipError_t launch_fb_table(uint32_t k32, const FbTableArgs& a, hipStream_t st);
hipError_t launch_fb_sched(const FbSchedArgs& a, hipStream_t st);
hipError_t launch_fb_exp(uint32_t k32, const FbExpArgs& a, int group, hipStream_t st);

// ---- Lim-Lee comb (comb.hip): many exponents per base ----------------------------
// Exponent bit t = (i v + j) b + k (row i < h, block j < v, column k < b).  Per
// base, table j holds G[j][u] = prod_{i: bit i of u} P_{i v + j} for u < 2^h with
// P_m = base^(2^(m b)) (G[j][0] = 1), so base^e = prod_{k = b-1..0} (square,
// then multiply by G[j][u_jk] for j < v): b - 1 squarings and v b products per
// exponent instead of BGMW's ceil(bits / w) + 2^w - 1.
struct CombParams {
  uint32_t h = 0, v = 0, b = 0;   // h = 0: not worth it / not possible
  uint32_t pstep = 1;             // P_m = chain entry m * pstep (chain entries every b / pstep squarings)
  uint32_t steps() const { return v * b; }
  size_t entries_per_base() const { return (size_t)v << h; }
};
// Cheapest (h, v) for exponents below 2^bits with `per_base` exponents per base,
// from a squaring chain whose entries are w squarings apart (`avail` of them per
// base; 0 = the chain is built for the comb), tables of at most `cap` bytes in
// all for `nbases` bases of `entry_bytes`.  h = 0 unless it beats BGMW (fb_window)
// by 10 %.
CombParams comb_choose(uint32_t bits, uint32_t w, uint32_t avail, double per_base, size_t nbases, size_t entry_bytes,
                       size_t cap);

struct CombBuildArgs {          // one popcount level of the tables
  const uint32_t* chain;        // chain entries (Montgomery form), base b's P_m at ptoff[b] + m * pstep
  const uint32_t* ptoff;        // [nbase]
  const uint32_t* mod_idx;      // [nbase] row of consts
  const uint32_t* consts;
  uint32_t* comb;               // [nbase][v][2^h][KD]
  const uint16_t* ulist;        // [nu] the level's u values (level 1: 0 and the single bits)
  uint32_t nu, h, v, pstep, nbase;
  uint32_t prio;                // s_setprio of the level's waves (short, latency-bound launches)
  uint32_t ulist_level1;        // 1: level 1 (u = 0 and the single bits: copies), else products
};
struct CombSchedArgs {          // per instance, step s = (b - 1 - k) v + j: u_jk (u16)
  const uint64_t* exp_ptr;      // [count]
  const uint32_t* exp_len;      // [count] limbs
  uint16_t* sched;              // [count][v b]
  uint32_t h, v, b, count;
};
// One comb_exp launch over up to kCombGroups instance groups (each with its own
// tables and (h, v, b)): group k owns blocks [block0, next group's block0), so
// every wave runs one group's schedule shape in lockstep.
constexpr int kCombGroups = 4;
struct CombGroupDev {
  const uint32_t* comb;         // the group's tables [nbase][v][2^h][KD]
  const uint16_t* sched;        // [count][steps]
  const uint32_t* ibase;        // [count] base (table set) of the instance, group-local
  const uint32_t* mod_idx;      // [count]
  const uint64_t* out_ptr;      // [count] destination (K32 limbs)
  uint32_t h, v, steps, count, block0;
};
struct CombExpArgs {
  CombGroupDev g[kCombGroups];
  uint32_t ngroups;
  const uint32_t* consts;
  uint32_t prio;
};
hipError_t launch_comb_build(uint32_t k32, const CombBuildArgs& a, hipStream_t st);
hipError_t launch_comb_sched(const CombSchedArgs& a, hipStream_t st);
// fills the groups' block0 (blocks of the launch's size) and launches
hipError_t launch_comb_exp(uint32_t k32, CombExpArgs& a, int group, hipStream_t st);

}  // namespace fsdkr
