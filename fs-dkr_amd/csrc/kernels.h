// Internal kernel entry points (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fsdkr {

constexpr int BLOCK = 256;

struct ModexpArgs {
  const uint32_t* base;     // [count][K32]
  const uint32_t* exps;     // [count][exp_limbs]
  uint32_t exp_limbs;
  uint32_t nwin;            // windows of `window` bits, taken from bit nwin*window-1 down
  uint32_t window;
  const uint32_t* mod_idx;  // [count]
  const uint32_t* consts;   // [n_mod][3*KD+4]  from mod_setup
  uint32_t* out;            // [count][K32]
  uint32_t* table;          // [count][2^window][KD] scratch
  uint32_t count;
};

int shape_digits(uint32_t k32);   // KD for a K32-limb modulus class (0 if unsupported)
hipError_t mod_setup(uint32_t k32, const uint32_t* mods, uint32_t n_mod, uint32_t* consts, hipStream_t st);
hipError_t modexp(uint32_t k32, const ModexpArgs& a, hipStream_t st);

}  // namespace fsdkr
