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

}  // namespace fsdkr
