/*
 * fsdkr.h — C ABI of the MI355X (gfx950) batch verifier for FS-DKR's
 * key-refresh hot path (Leo-Li009/fs-dkr, reference mounted at
 * /root/reference).
 *
 * The reference has no FFI: its operator API is the Rust signatures of
 * RefreshMessage::collect and the proof verifiers it calls.  This header is
 * the boundary a thin Rust wrapper binds under those
 * unchanged signatures.  Every entry point cites the reference interface it
 * replaces.
 *
 * Conventions
 *  - Big integers are little-endian arrays of uint32_t limbs, fixed width per
 *    call (mod_limbs in {64, 96, 128, 192}: 2048/3072/4096/6144-bit moduli).
 *  - All pointers are borrowed host pointers unless the name says _device.
 *  - Return value: 0 = FSDKR_OK, negative = FSDKR_E_*.  An invalid proof is
 *    DATA (a verdict bit), never an error code.  fsdkr_last_error() gives text.
 *  - Calls are blocking and not thread-safe per context (one context per
 *    calling thread).  Nothing unwinds across the boundary.
 */
#ifndef FSDKR_FSDKR_H
#define FSDKR_FSDKR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FSDKR_OK 0
#define FSDKR_E_ARG (-1)          /* bad argument (null pointer, size, even modulus, ...) */
#define FSDKR_E_HIP (-2)          /* HIP runtime failure (no device, launch failure)      */
#define FSDKR_E_OOM (-3)          /* device allocation failed                              */
#define FSDKR_E_UNSUPPORTED (-4)  /* operand shape outside what the kernels implement     */

typedef struct fsdkr_ctx fsdkr_ctx;

typedef struct fsdkr_cfg {
  int32_t device;  /* HIP device ordinal (-1: current device)                 */
  uint32_t flags;  /* FSDKR_CFG_TIMING: record HIP events around every kernel */
} fsdkr_cfg;

#define FSDKR_CFG_TIMING 1u

/* Context: owns the HIP stream, device buffers and per-modulus constant
 * tables.  Replaces nothing in the reference (which holds no state between
 * calls); it exists so repeated collect() calls reuse device memory. */
int fsdkr_ctx_create(const fsdkr_cfg* cfg, fsdkr_ctx** out);
void fsdkr_ctx_destroy(fsdkr_ctx* ctx);
const char* fsdkr_last_error(const fsdkr_ctx* ctx);
/* 1 if the shared library was built with gfx950 kernels and a device is present. */
int fsdkr_device_available(void);

/* ---- Job 2 building block: batched modular exponentiation -----------------
 * out[i] = base[i] ^ exp[i] mod mods[mod_idx[i]]   (exact, fully reduced)
 *
 * Replaces curv-kzen 0.10 BigInt::mod_pow (GMP mpz_powm) as called from
 *   zk_pdl_with_slack.rs:177-186 (commitment_unknown_order),
 *   range_proofs.rs:129,136-137,142,148 (AliceProof::verify),
 *   ring_pedersen_proof.rs:144-148 (RingPedersenProof::verify),
 *   kzen-paillier encrypt_with_chosen_randomness (refresh_message.rs:75-81).
 * base[i] < 2^(32*mod_limbs) (need not be reduced), exp[i] >= 0 of exp_limbs
 * limbs, every modulus odd.  mod_idx[i] < n_mod. */
int fsdkr_modexp_batch(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* base,
                       const uint32_t* exp, uint32_t exp_limbs, const uint32_t* mod_idx,
                       const uint32_t* mods, uint32_t n_mod, uint32_t* out);

/* Device-resident variant for benchmarking/integration: all pointers are
 * device pointers already in HBM; runs on the context stream and returns
 * after the kernels complete.  `exp_bits` bounds the exponent bit length. */
int fsdkr_modexp_batch_device(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* d_base,
                              const uint32_t* d_exp, uint32_t exp_limbs, uint32_t exp_bits,
                              const uint32_t* d_mod_idx, const uint32_t* d_mods, uint32_t n_mod,
                              uint32_t* d_out);

/* Kernel timing (needs FSDKR_CFG_TIMING): accumulated milliseconds and launch
 * count of kernel `name` since the last reset ("modexp", "mod_setup", ...). */
int fsdkr_kernel_time(const fsdkr_ctx* ctx, const char* name, double* ms, uint32_t* launches);
void fsdkr_kernel_time_reset(fsdkr_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* FSDKR_FSDKR_H */
