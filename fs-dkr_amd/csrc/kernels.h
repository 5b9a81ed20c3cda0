// Internal kernel entry points (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fsdkr {

constexpr int BLOCK = 256;

// ---- per-modulus constants (mod_setup_kernel) ----------------------------------
// Row of modulus m: [N | R mod N | R^2 mod N | ninv, pad x3] for the class's KD
// digits, then the same block for N' = N (-N^-1 mod 2^29) (quotient-scaled rows;
// written when SCALED_OK), R = 2^(29 KD).
constexpr int cons_stride(int kd) { return 6 * kd + 8; }
constexpr int cons_scaled(int kd) { return 3 * kd + 4; }
// N' < 2^(32 K32 + 29) must leave R > 4N': 32 K32 + 31 <= 29 KD
constexpr bool scaled_ok(int kd, int k32) { return 32 * k32 + 31 <= 29 * kd; }

// One batched-modexp launch.  Operands are addressed per instance so a launch
// can mix proof fields, device-computed challenges and other kernels' outputs.
struct ModexpArgs {
  const uint64_t* base_ptr;  // [count] device addresses of little-endian u32 limbs
  const uint32_t* base_len;  // [count] limbs (<= K32)
  const uint64_t* exp_ptr;   // [count]
  const uint32_t* exp_len;   // [count] limbs
  uint32_t nwin;             // windows of `window` bits, taken from bit nwin*window-1 down
  uint32_t window;
  const uint32_t* nwin_i;    // [count] per-instance window count (overrides nwin; merged launches)
  const uint32_t* mod_idx;   // [count] row of `consts`
  const uint32_t* consts;    // [n_mod][3*KD+4]  from mod_setup
  uint32_t* out;             // [count][K32]
  uint32_t* table;           // [count][2^window][KD] scratch
  uint32_t count;
  uint32_t prio;             // > 0: latency-critical launch, its waves raise their issue priority to s_setprio(prio)
  uint32_t group;            // lanes per instance (0 = choose by batch size)
  uint32_t ct;               // 1: regular access for secret exponents (every window-table read
                             // scans the whole table; every instance runs `nwin` windows)
  uint32_t slide;            // 1: sliding windows of up to `window` bits (odd-power table of
                             // 2^(window-1) + 1 entries); the caller guarantees that the
                             // instances of every wave share their exponent (modexp_slide_kernel)
  const uint32_t* out_idx;   // [count] output row of each instance (nullptr: row = instance)
  // Split sliding-window chains (slide shapes, QS): a HEAD launch (lo_bit > 0, tail
  // = 0) runs the exponent bits >= lo_bit, always builds the odd-power table and
  // writes its accumulator (the chain's Montgomery form) to state; the TAIL launch
  // (tail = 1, same descriptors, table and w) resumes from state and runs the bits
  // < lo_bit, jointly with base2^exp2 per instance (4-bit fixed windows over a
  // 16-entry table in table2) when base2_ptr is set: out = base^exp * base2^exp2.
  uint32_t lo_bit = 0;
  uint32_t tail = 0;
  uint32_t* state = nullptr;        // [count][KD]
  const uint64_t* base2_ptr = nullptr;   // [count] K32 limbs, reduced
  const uint64_t* exp2_ptr = nullptr;    // [count]
  const uint32_t* exp2_len = nullptr;    // [count] limbs, exp2 < 2^lo_bit
  uint32_t* table2 = nullptr;       // [count][16][KD]
};

int shape_digits(uint32_t k32);   // KD for a K32-limb modulus class (0 if unsupported)
// The 32-lane 4096-bit latency shape uses KD = 160 digits (L = 5 per lane), so its
// Montgomery constants (R = 2^(29 KD)) differ from the 144-digit class: a launch
// with group kWideGroup needs consts from mod_setup_g(k32, kWideGroup, ...).
constexpr uint32_t kWideGroup = 32;
// One instance per wave64 (modexp_wave_kernel), 4096-bit class only; it uses the
// class's own KD = 144 constants (mod_setup), table entries of 192 words.
constexpr uint32_t kWaveGroup = 64;
int shape_digits_g(uint32_t k32, uint32_t group);   // digits of the Montgomery constants
int table_digits(uint32_t k32, uint32_t group);     // words per window-table entry
hipError_t mod_setup(uint32_t k32, const uint32_t* mods, uint32_t n_mod, uint32_t* consts, hipStream_t st);
hipError_t mod_setup_wave(uint32_t k32, const uint32_t* mods, uint32_t n_mod, uint32_t* consts, hipStream_t st);
hipError_t mod_setup_g(uint32_t k32, uint32_t group, const uint32_t* mods, uint32_t n_mod, uint32_t* consts,
                       hipStream_t st);
hipError_t modexp(uint32_t k32, const ModexpArgs& a, hipStream_t st);

// Miller–Rabin witness tail (prime.hip): x = b^d mod c from modexp, c - 1 = d 2^s.
struct MrTailArgs {
  const uint32_t* x;        // [count][K32] exact
  const uint32_t* consts;   // [count][3*KD+4]: candidate i is modulus i
  const uint32_t* s;        // [count]
  uint32_t s_max;           // max s over the launch (uniform loop bound)
  uint32_t* verdict;        // [count] 1 = strong probable prime to this base
  uint32_t count;
};
// Modulus widths of key generation: 32 limbs (1024-bit primes, KD = 36) beside
// the verifier's classes.  Not accepted by the collect() entry points.
constexpr uint32_t kPrimeLimbs = 32;
hipError_t mr_tail(uint32_t k32, const MrTailArgs& a, hipStream_t st);

}  // namespace fsdkr
