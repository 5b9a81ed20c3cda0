// Argument blocks of the verification kernels (verify.hip).  Device
// addresses are carried as uint64_t so descriptor arrays can be built on the
// host and uploaded in one copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "kernels.h"

namespace fsdkr {

struct BinomArgs {          // out = 1 + s * n
  const uint64_t* s_ptr;
  const uint64_t* n_ptr;
  uint32_t s_len, n_len, out_limbs;
  uint32_t* out;
  uint32_t count;
};

struct PedHashArgs {        // ring-Pedersen challenge bits
  const uint32_t* A;        // [count][M][a_len]
  uint32_t M, a_len;
  uint32_t* bits;           // [count][ceil(M/32)]
  uint32_t* panic;          // [count] 0, or 1 + bits readable before the reference's index panic
  uint32_t count;
};

struct AliceHashArgs {      // H(N, N+1, c, z, u, w) == e
  const uint64_t* n_ptr;    // receiver N
  const uint64_t* c_ptr;    // ciphertext
  const uint32_t *z, *u, *w, *e;
  uint32_t n_len, c_len, z_len, e_len;
  uint8_t* verdict;         // in: host pre-checks, out: AND hash equality
  uint32_t count;
  uint32_t* state;          // [count][32] SHA-256 state after H(N, N+1, c, z) (alice_prefix), or null
};

struct InverseArgs {
  const uint64_t* y_ptr;    // value to invert (reduced, K32 limbs)
  const uint64_t* m_ptr;    // odd modulus (K32 limbs)
  uint32_t* out;            // [count][K32] inverse (may be null)
  uint32_t* unit;           // [count] 1 if gcd(y, m) == 1
  uint32_t* scratch;        // unused (lane-cooperative inverse keeps its state in registers)
  uint32_t count;
};

// Montgomery's simultaneous inversion: the instances of one modulus (a group)
// share ONE inverse -- prefix products, the inverse of the last, a backward pass
// of two products per element -- with a per-element fallback (inverse_coop's
// algorithm) for a group whose product is not a unit.  y_ptr / out / unit are
// indexed as InverseArgs; order lists the instances group by group.
struct BatchInverseArgs {
  const uint64_t* y_ptr;    // [count] values (reduced)
  const uint64_t* m_ptr;    // [count] moduli (every instance of a group: the same odd modulus)
  const uint32_t* order;    // [count] instance indices, grouped by modulus
  const uint32_t* gstart;   // [ngroups + 1] group offsets into order
  uint32_t* out;            // [count][K32] inverses (may be null: unit flags only)
  uint32_t* unit;           // [count] 1 if gcd(y, m) == 1
  uint32_t* scratch;        // [count][KD] prefix products (device)
  uint32_t ngroups;
};

struct EqOperand {
  uint64_t a, b, c, d;      // device addresses
  uint32_t a_len, b_len, c_len, d_len;
  uint32_t sel;             // bit index into sel_bits choosing d (set) or 1 (clear); ~0 = always d
  uint32_t flags;           // bit0: require c < N
};

struct EqCheckArgs {        // a*b == c*d (mod N)
  const EqOperand* ops;
  const uint32_t* mod_idx;
  const uint32_t* consts;
  const uint32_t* sel_bits;
  uint64_t one;             // address of the constant 1 (K32 limbs)
  uint32_t* out;            // [count] 1/0
  uint32_t count;
};

struct Prod3Operand {
  uint64_t a, b, c;
  uint32_t a_len, b_len, c_len, pad;
};

struct Prod3Args {          // out = a*b*c mod N
  const Prod3Operand* ops;
  const uint32_t* mod_idx;
  const uint32_t* consts;
  uint32_t* out;            // [count][K32]
  uint32_t count;
};

struct PdlU1Args {          // G*(s1 mod q) + Q*(q - e) == u1
  const uint32_t *s1, *e, *Q, *u1;
  uint32_t s1_len;
  uint8_t* verdict;         // bit0 written
  uint32_t count;
};

// One Feldman share check: S == sum_j A[off + j] * idx^j over ncoef commitments.
struct FeldmanInfo {
  uint32_t off;             // first commitment point (index into vss)
  uint32_t ncoef;           // commitments of the message (0: curv's unwrap panics)
  uint32_t idx;             // evaluation point i + 1
  uint32_t pad;
};

struct FeldmanArgs {
  const uint32_t* vss;      // [points][16]
  const uint32_t* S;        // [count][16]
  const FeldmanInfo* info;  // [count]
  uint8_t* verdict;         // [count] bit0 ok, bit1 panic
  uint32_t count;
  uint32_t prio;            // s_setprio of the Horner threads (one long serial chain each)
};

// 2-adic half of a check modulo an even modulus N = 2^k * m (m odd):
//   a^ea * b^eb == c * d^[bit]   (mod 2^k)
// (the odd half runs in the Montgomery kernels modulo m).  Used for even
// ring-Pedersen and composite-DLog moduli, which the reference exponentiates
// with GMP like any other (ring_pedersen_proof.rs:144-148, zk-paillier
// CompositeDLogProof::verify).  Null addresses stand for the value 1.
struct Pow2Op {
  uint64_t a, ea, b, eb, c, d;
  uint32_t a_len, ea_len, b_len, eb_len, c_len, d_len;
  uint32_t sel;             // ~0: d always; else challenge bit index (d used iff set)
  uint32_t kbits;           // k (1 .. 32 * 96)
};

struct Pow2Args {
  const Pow2Op* ops;
  const uint32_t* sel_bits;
  uint32_t* out;            // [count] 1/0
  uint32_t count;
};

struct EcMsmArgs {          // out[o] = sum_j scalars[o][j] * P[o][j]
  const uint64_t* pt_ptr;   // [count][terms] affine points (16 limbs)
  const uint32_t* scalars;  // [count][terms][8]
  uint32_t terms;
  uint32_t* out;            // [count][16] affine
  uint32_t count;
  uint32_t* scratch;        // [count][terms][24] Jacobian terms
  uint32_t prio;            // s_setprio level (0..3)
};

hipError_t launch_binom(const BinomArgs& a, hipStream_t st);
hipError_t launch_ped_hash(const PedHashArgs& a, hipStream_t st);
hipError_t launch_alice_hash(const AliceHashArgs& a, hipStream_t st);
hipError_t launch_alice_prefix(const AliceHashArgs& a, hipStream_t st);
hipError_t launch_inverse(uint32_t k32, const InverseArgs& a, hipStream_t st);
// lane-cooperative Pornin inverse (inverse.hip): registers + DPP
hipError_t launch_inverse_coop(uint32_t k32, const InverseArgs& a, hipStream_t st);
hipError_t launch_inverse_batch(uint32_t k32, const BatchInverseArgs& a, hipStream_t st);
// Montgomery's simultaneous inversion where instances share a modulus (one
// binary-GCD inverse per modulus instead of one per instance); FSDKR_CFG_INV_EACH:
// one inverse each (tests, A/B)
struct Ctx;
bool batch_inv_on(const Ctx* c);
size_t inverse_batch_scratch_words(uint32_t k32);
hipError_t launch_eq_check(uint32_t k32, const EqCheckArgs& a, hipStream_t st);
hipError_t launch_prod3(uint32_t k32, const Prod3Args& a, hipStream_t st);
hipError_t launch_pdl_u1(const PdlU1Args& a, hipStream_t st);
hipError_t launch_feldman(const FeldmanArgs& a, hipStream_t st);
hipError_t launch_ec_msm(const EcMsmArgs& a, hipStream_t st);
hipError_t launch_pow2_check(const Pow2Args& a, hipStream_t st);

}  // namespace fsdkr
