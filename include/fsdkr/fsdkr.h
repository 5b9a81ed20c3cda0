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
  uint32_t flags;  /* FSDKR_CFG_* below                                        */
} fsdkr_cfg;

/* record HIP events around every kernel (fsdkr_kernel_timing) */
#define FSDKR_CFG_TIMING 1u
/* Algorithm switches for parity tests and A/B runs.  Results are identical
 * under every setting; the default (0) is the fastest measured.
 *   FB_BGMW   fixed-base exponentiations by BGMW windows only (no Lim-Lee comb)
 *   FB_COMB   a Lim-Lee comb wherever one fits, even where it saves nothing
 *   INV_EACH  one binary-GCD inverse per element (no simultaneous inversion) */
#define FSDKR_CFG_FB_BGMW 2u
#define FSDKR_CFG_FB_COMB 4u
#define FSDKR_CFG_INV_EACH 8u

/* Context: owns the HIP stream, device buffers and per-modulus constant
 * tables.  Replaces nothing in the reference (which holds no state between
 * calls); it exists so repeated collect() calls reuse device memory. */
int fsdkr_ctx_create(const fsdkr_cfg* cfg, fsdkr_ctx** out);
void fsdkr_ctx_destroy(fsdkr_ctx* ctx);
const char* fsdkr_last_error(const fsdkr_ctx* ctx);
/* Lanes cooperating on one modexp instance (2, 4, 8, 16, and 32 or 64 for the
 * 4096-bit generic modexp, 64 being one instance per wavefront; unsupported
 * values for a width fall back to the automatic choice); 0 = choose by batch
 * size. */
int fsdkr_ctx_set_modexp_group(fsdkr_ctx* ctx, uint32_t lanes);
/* Switch per-kernel HIP-event timing (FSDKR_CFG_TIMING) on or off after
 * creation.  The events cost ~9 ms per n = 64 collect (eight streams, one
 * event pair per launch), so timed benchmark regions run with it off. */
int fsdkr_ctx_set_timing(fsdkr_ctx* ctx, int on);
/* Replace the context's fsdkr_cfg flags (FSDKR_CFG_*) after creation.  Waits
 * for outstanding work first. */
int fsdkr_ctx_set_flags(fsdkr_ctx* ctx, uint32_t flags);

/* Multi-GPU shards: run the s^N mod N^2 chains (GA, the longest dependent
 * chains of collect()) on `ga_cus` CUs spread over the 8 XCDs and every other
 * stream on the complement, so a rank's small batch keeps its critical chains
 * off the SIMDs of the throughput jobs (0 = no split, the single-GPU default).
 * A multiple of 8, at most 224.  Waits for outstanding work, re-creates the
 * context's streams.  Performance setting only: results are unchanged. */
int fsdkr_ctx_set_cu_split(fsdkr_ctx* ctx, uint32_t ga_cus);
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

/* fsdkr_modexp_batch for SECRET exponents (the prover's alpha, gamma, rho, a_i,
 * lambda, xhi, sigma's N^-1 mod phi; key generation's candidates; decryption's
 * p - 1, q - 1): identical results, but the kernel's memory addresses and
 * instruction stream do not depend on the exponent.  Every window-table read
 * scans the whole table through a mask, and every instance runs the window
 * count of the widest exponent of the call (only exp_limbs is visible).  GMP's
 * mpz_powm, behind the reference's curv BigInt::mod_pow, has no such property
 * (mpz_powm_sec does). */
int fsdkr_modexp_batch_ct(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* base,
                          const uint32_t* exp, uint32_t exp_limbs, const uint32_t* mod_idx,
                          const uint32_t* mods, uint32_t n_mod, uint32_t* out);

/* out[i] = y[i]^-1 mod m[i] and unit[i] = (gcd(y[i], m[i]) == 1); y[i] < m[i],
 * every m[i] odd, all [count][mod_limbs].  out may be NULL (unit test only).
 * Replaces curv BigInt::mod_inv (GMP mpz_invert) at zk_pdl_with_slack.rs:180
 * (PDL: unwrap, panics on a non-unit) and range_proofs.rs:129,142 (Alice). */
int fsdkr_mod_inverse(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* y, const uint32_t* m,
                      uint32_t* out, uint32_t* unit);

/* Device-resident variant for benchmarking/integration: all pointers are
 * device pointers already in HBM; runs on the context stream and returns
 * after the kernels complete.  `exp_bits` bounds the exponent bit length. */
int fsdkr_modexp_batch_device(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* d_base,
                              const uint32_t* d_exp, uint32_t exp_limbs, uint32_t exp_bits,
                              const uint32_t* d_mod_idx, const uint32_t* d_mods, uint32_t n_mod,
                              uint32_t* d_out);

/* fsdkr_modexp_batch_device with ONE exponent per modulus (key): d_exp is
 * [n_mod][exp_limbs], instance i computes d_base[i]^d_exp[mod_idx[i]] mod
 * d_mods[mod_idx[i]] -- the r^N mod N^2 of Paillier encryption under key N
 * (paillier EncryptWithChosenRandomness behind the reference's
 * Paillier::encrypt_with_chosen_randomness calls, refresh_message.rs:75-81).
 * The instances are regrouped by key so each wave shares its exponent and the
 * 4096-bit launch runs sliding windows; results land in the caller's order. */
int fsdkr_modexp_keyed_device(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* d_base,
                              const uint32_t* d_exp, uint32_t exp_limbs, uint32_t exp_bits,
                              const uint32_t* d_mod_idx, const uint32_t* d_mods, uint32_t n_mod,
                              uint32_t* d_out);

/* ---- Key generation: batched Miller–Rabin -------------------
 * verdict[i] = 1 iff cand[i] is a strong probable prime to base bases[i]:
 * with cand - 1 = d 2^s, b^d == 1 or b^(d 2^j) == cand - 1 for some j < s
 * (mod cand).  cand: [count][mod_limbs], odd and >= 5; bases: [count][mod_limbs]
 * (any value; 2 <= b <= cand - 2 for a meaningful round).  mod_limbs in
 * {32, 64, 96} (1024/2048/3072-bit candidates).  Replaces the primality test
 * inside kzen-paillier 0.4.3 Paillier::keypair_with_modulus_size, called at
 * refresh_message.rs:118 (distribute), ring_pedersen_proof.rs:50
 * (RingPedersenStatement::generate) and add_party_message.rs:51
 * (generate_h1_h2_n_tilde).  fsdkr.keygen drives the prime walk above it. */
int fsdkr_miller_rabin(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t count, const uint32_t* cand,
                       const uint32_t* bases, uint32_t* verdict);


/* ---- Job 2: batched verification of RefreshMessage::collect ----------------
 * One call verifies every proof collect() checks (refresh_message.rs:321-437):
 * n^2 Feldman share checks (:177-188), R*n PDL-with-slack + Alice range proofs
 * (:330-350), R+J ring-Pedersen proofs (:353-365), R+J Paillier correct-key
 * proofs + modulus sizes (:375-396), J pairs of composite-DLog proofs
 * (:398-437).  The caller's batching layer gathers the messages into the SoA
 * arrays below (pairs p = k*n + i, k < R sender slice order, i < n receiver);
 * big integers use fixed per-field limb widths chosen by the caller.
 * Points are affine x||y (8+8 limbs), (0,0) encodes the point at infinity. */
typedef struct fsdkr_collect_batch {
  uint32_t n_refresh;    /* R */
  uint32_t n_join;       /* J;  n = R + J receivers (new_n, :327)                 */
  uint32_t t;            /* local_key.t                                           */
  uint32_t m_security;   /* M of RingPedersenProof (256)                          */
  uint32_t key_bits;     /* PAILLIER_KEY_SIZE (lib.rs:26)                         */
  uint32_t nl;           /* limbs of N, N~, h1, h2, ring-Pedersen N (64 = 2048 bit) */
  uint32_t s1l, s3l, el, zl, yl; /* limb widths of PDL/Alice s1, s3|s2, Alice e, RP Z, DLog y */
  const uint32_t* party_index;   /* [R+J] message party indices (joins: 0 = unassigned) */
  const uint32_t* msg_lens;      /* [R][3] pdl_proof_vec / points_committed / points_encrypted lengths */
  /* receivers: local_key.paillier_key_vec[i].n and h1_h2_n_tilde_vec[i] */
  const uint32_t *recv_n, *recv_ntilde, *recv_h1, *recv_h2;          /* [n][nl]   */
  /* pairs */
  const uint32_t* enc;      /* [P][2nl] points_encrypted_vec[i]       */
  const uint32_t* commit;   /* [P][16]  points_committed_vec[i]       */
  const uint32_t *pdl_z, *pdl_u3, *pdl_s2;                            /* [P][nl]   */
  const uint32_t* pdl_u1;   /* [P][16]  */
  const uint32_t* pdl_u2;   /* [P][2nl] */
  const uint32_t* pdl_s1;   /* [P][s1l] */
  const uint32_t* pdl_s3;   /* [P][s3l] */
  const uint32_t *rp_z, *rp_s;                                        /* [P][nl]   */
  const uint32_t* rp_e;     /* [P][el]  */
  const uint32_t* rp_s1;    /* [P][s1l] */
  const uint32_t* rp_s2;    /* [P][s3l] */
  const uint32_t* vss;      /* [R][t+1][16] coefficients_committed_vec commitments */
  /* ring-Pedersen statement + proof of the R refresh then J join messages */
  const uint32_t *ped_S, *ped_T, *ped_N;                              /* [R+J][nl] */
  const uint32_t* ped_A;    /* [R+J][M][nl] */
  const uint32_t* ped_Z;    /* [R+J][M][zl] */
  /* NiCorrectKeyProof: ek.n and sigma_vec of the R then J messages */
  const uint32_t* ck_n;     /* [R+J][ckl]     (ckl below; 0 = nl) */
  const uint32_t* ck_sigma; /* [R+J][11][ckl] */
  /* join messages: dlog_statement {N, g, ni} and the two CompositeDLogProofs */
  const uint32_t *dlog_N, *dlog_g, *dlog_ni, *dlog_x1, *dlog_x2;      /* [J][nl]  */
  const uint32_t *dlog_y1, *dlog_y2;                                  /* [J][yl]  */
  /* receivers; 0 means R + J.  A multi-GPU shard passes a slice of the refresh
   * messages (and of the joins' proofs) with the full receiver set n. */
  uint32_t n_recv;
  /* Optional (NULL / 0 = the regular shape):
   *  vss_len    [R] number of commitments of each coefficients_committed_vec; vss is
   *             then ragged (sum vss_len points).  curv validate_share_public runs
   *             Horner over each message's own vector (refresh_message.rs:180-182);
   *             an empty vector panics (unwrap).  NULL: t+1 each.
   *  range_lens [R] range_proofs lengths; range_proofs[i] with i >= len panics
   *             (refresh_message.rs:342).  rp_* rows past the length are placeholders.
   *  ckl        limbs of ck_n / ck_sigma (64, 96, 128, 192); 0 = nl.  Lets a batch of
   *             2048-bit receivers carry an oversize ek.n whose correct-key proof the
   *             reference verifies before it reports ModuliTooSmall (:376-391).
   *  recv_avail receivers that local_key holds keys for (0 = all n); the reference
   *             indexes paillier_key_vec[i] / h1_h2_n_tilde_vec[i] (:334-339) and panics
   *             at the first pair with i >= recv_avail (rows past it are placeholders).
   *  ped_lens   [R+J][2] lengths of ring_pedersen_proof.A and .Z: A shorter than M
   *             panics in the challenge hash, Z shorter at check len(Z)
   *             (ring_pedersen_proof.rs:131-144); missing rows are placeholders.
   *  ck_lens    [R+J] lengths of dk_correctness_proof.sigma_vec (< 11 panics in
   *             zk-paillier's verify); missing rows are placeholders.
   *  pdl_s3_neg [R*n] nonzero: the pair's PDL s3 is negative and pdl_s3 holds |s3|.
   *             commitment_unknown_order then raises h2^-1 to |s3|
   *             (zk_pdl_with_slack.rs:177-184); the u3 check is evaluated as
   *             h1^s1 == u3 * z^e * h2^|s3| (mod N~), equivalent when h2 is a unit.
   *             The caller reports the pairs whose h2 is not a unit (mod_inv
   *             unwrap panics) itself; their u3 bit here is meaningless.
   *  neg_bits   [R*n] bit 0: the pair's PDL z is negative, bit 1: its Alice z is,
   *             bit 2: its ciphertext c is; pdl_z / rp_z / enc then hold the
   *             magnitude.  The challenges hash |v| (curv to_bytes); the arithmetic
   *             takes the residue -|v| mod N~ (z^e) or mod N^2 (c^e, c^-1), as GMP
   *             reduces a negative base (zk_pdl_with_slack.rs:114-122,136-157;
   *             range_proofs.rs:129-157).  The caller's share decryption reduces its
   *             own ciphertexts (Paillier::mul / add work mod N^2, :221-234).
   *  ped_a_neg  [R+J][M] nonzero: ring-Pedersen A_k is negative and ped_A holds |A_k|:
   *             the challenge hashes |A_k|, the check T^Z_k == A_k S^e_k (mod N)
   *             takes -|A_k| mod N (BigInt::mod_mul reduces it;
   *             ring_pedersen_proof.rs:130-153). */
  const uint32_t* vss_len;
  const uint32_t* range_lens;
  uint32_t ckl;
  uint32_t recv_avail;
  const uint32_t* ped_lens;
  const uint32_t* ck_lens;
  const uint8_t* pdl_s3_neg;
  const uint8_t* neg_bits;
  const uint8_t* ped_a_neg;
} fsdkr_collect_batch;

/* Verdicts (caller-allocated). 1 bits mean "check passed".  cap_* are the
 * element capacities of the arrays; a call fails with FSDKR_E_ARG if the
 * prepared batch needs more (R*n pairs, R+J messages, J joins).  The device
 * pass never sets range bit1 / dlog bit2: the host layer sets them for
 * instances whose negative operand makes the reference panic (a negative
 * exponent in curv's mod_pow), and fsdkr_collect_first_error maps them. */
typedef struct fsdkr_verdicts {
  uint8_t* feldman;  /* [R*n]  bit0 validate_share_public ok; bit1: reference panics  */
  uint8_t* pdl;      /* [R*n]  bit0 u1, bit1 u2, bit2 u3 equal; bit3: reference panics */
  uint8_t* range;    /* [R*n]  bit0 AliceProof::verify ok; bit1: reference panics        */
  uint8_t* ped;      /* [R+J]  bit0 RingPedersenProof::verify ok; bit1: panics         */
  uint8_t* ck;       /* [R+J]  bit0 NiCorrectKeyProof::verify ok; bit1: reference panics */
  uint8_t* dlog;     /* [J]    bit0 base-h1 proof ok, bit1 base-h2 proof ok, bit2: reference
                      *         panics (may be NULL if J = 0) */
  uint32_t cap_pairs, cap_msgs, cap_joins;
} fsdkr_verdicts;

int fsdkr_verify_collect(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch, fsdkr_verdicts* out);

/* The same as phases: prepare = host pre-pass + ONE host->device copy of the
 * batch image (kept in the context); run = the kernel pipeline on the
 * device-resident batch + verdict readback (= launch + finish: launch only
 * enqueues the kernels and returns, so the caller can overlap host work or the
 * share-recovery calls, which run on their own stream).  run may be repeated;
 * a failed prepare leaves no batch (run then returns FSDKR_E_ARG). */
int fsdkr_collect_prepare(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch);
int fsdkr_collect_run(fsdkr_ctx* ctx, fsdkr_verdicts* out);
int fsdkr_collect_launch(fsdkr_ctx* ctx);
int fsdkr_collect_finish(fsdkr_ctx* ctx, fsdkr_verdicts* out);

/* Optional head start: launches the pipeline's longest job -- s2^N and s^N mod
 * N^2 of every (message, receiver) pair (zk_pdl_with_slack.rs:129-135,
 * range_proofs.rs:148), 2 R n chains of 2048-bit exponents at 4096 bits -- from
 * the only fields it reads (n_refresh, n_join, n_recv, nl, recv_n, pdl_s2,
 * rp_s), so it runs while the caller packs the rest of the batch.  The next
 * fsdkr_collect_prepare of a single batch with equal values of those fields
 * reuses the results (anything else recomputes them).  Fails with FSDKR_E_ARG
 * while a launched batch is not finished.  Does not validate: a batch it cannot
 * start is left to prepare.  The fixed-base tables (recv_ntilde, recv_h1,
 * recv_h2, ped_T, ped_N and the exponent widths) and the correct-key job (ck_n,
 * ck_sigma) start too when present, and with the exponents themselves (pdl_s1,
 * pdl_s3, rp_s1, rp_s2, ped_Z) every fixed-base exponentiation behind the tables.  Called again with the same GA fields while
 * those chains run (a caller that packed them first), it leaves GA running and
 * starts only the parts that are new.  Once the tables are started, a call that
 * finds the challenge jobs' fields (enc, commit, pdl_z, pdl_u1, pdl_u2, pdl_u3,
 * rp_z, rp_e, el, vss with the table call's pdl_s1 / rp_s1) starts them: the PDL
 * challenges (hashed on the host), c^e mod N^2 and z^e mod N~ of the PDL and
 * Alice proofs with their inverses, pdl_u1 and the Feldman checks.  prepare
 * reuses each started part only if every row that part read is equal. */
int fsdkr_collect_prestart(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch);

/* out[i] = base[i]^E[mod_idx[i]] * base2[i]^exp2[i] mod N[mod_idx[i]] (4096-bit
 * moduli, 128 limbs; E: one exponent per modulus, exp_limbs limbs; exp2: 8 limbs,
 * below 2^256; base2 reduced) through collect()'s split GA chains: a head over E's
 * bits >= 256 and a joint tail, which is how collect() computes s2^N c^-e mod N^2
 * (zk_pdl_with_slack.rs:136-142) and s^N c^-e mod N^2 (range_proofs.rs:140-148)
 * with base2 = c^-1.  Parity tests of that path; odd moduli. */
int fsdkr_modexp_joint_batch(fsdkr_ctx* ctx, uint32_t count, const uint32_t* base, const uint32_t* base2,
                             const uint32_t* exp2, const uint32_t* mod_idx, const uint32_t* mods,
                             const uint32_t* mod_exp, uint32_t exp_limbs, uint32_t n_mod, uint32_t* out);

/* Which prestarted parts the last fsdkr_collect_prepare[_multi] reused (bit
 * mask): 1 GA chains, 2 fixed-base tables, 4 correct-key job, 8 ring-Pedersen
 * T^Z exponents (multi-session).  0 before any prepare.  Diagnostic (tests
 * check that a changed batch is recomputed); the reference has no counterpart. */
uint32_t fsdkr_collect_reuse_mask(const fsdkr_ctx* ctx);

/* Device span of the last finished collect() call (single or multi-session), in
 * ms from HIP timing events: from the call's first device work (the end of the
 * prestart's upload, or the pipeline launch when nothing was prestarted) to the
 * end of the pipeline's last kernel.  -1 before the first finish.  Diagnostic
 * only; the reference has no counterpart. */
double fsdkr_collect_last_span_ms(const fsdkr_ctx* ctx);

/* ---- Many independent collect() calls in ONE device pass -------------------
 * `count` sessions (e.g. BASELINE configs[4]: 1024 custody wallets, t=1 n=3,
 * 3072-bit keys), each the batch its own RefreshMessage::collect
 * (refresh_message.rs:321-326) would verify; out[s] receives session s's
 * verdicts.  Sessions may differ in R, J, n, t and limb widths (the device
 * image uses the widest); m_security must agree.  The reference has no such
 * entry point: it verifies one session per call.  fsdkr_collect_first_error
 * then maps each session's verdicts on its own. */
int fsdkr_verify_collect_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count,
                               fsdkr_verdicts* out);
int fsdkr_collect_prepare_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count);
int fsdkr_collect_finish_multi(fsdkr_ctx* ctx, fsdkr_verdicts* out, uint32_t count);
/* fsdkr_collect_prestart for many sessions: starts every session's s2^N and
 * s^N mod N^2 chains (GA) in one launch from recv_n, pdl_s2, rp_s (and the
 * counts, nl) of each batch; a later fsdkr_collect_prepare_multi of batches
 * with the same values and shapes consumes the results (otherwise it computes
 * them itself).  Lets the caller pack the other fields of 1024 custody
 * sessions (BASELINE configs[4]) while the longest chains run.  When every
 * batch also carries recv_ntilde, recv_h1, recv_h2, ped_T, ped_N (and the s1l,
 * s3l, zl widths) the fixed-base table chains start too; when every batch
 * carries ck_n, ck_sigma and ckl (no ck_lens), so does the correct-key job
 * (sigma_k^n mod n, zk-paillier NiCorrectKeyProof::verify).  Each part is
 * reused only if prepare's values match it exactly. */
int fsdkr_collect_prestart_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count);
/* After fsdkr_collect_prestart[_multi] started the fixed-base tables: every
 * message's ring-Pedersen T^Z_k mod N (ring_pedersen_proof.rs:144) as fixed-base
 * exponents behind the T tables, from ped_Z / zl / m_security of the same
 * batches (no ped_lens).  The Z rows are copied to the device before the call
 * returns.  A later prepare of batches with the same T, N and Z rows (compared
 * by a 64-bit digest of the Z rows) reads these results instead of computing
 * them, and takes the Z rows from the prestart's copy.  Does nothing when the
 * tables were not prestarted or an exponent exceeds their bound. */
int fsdkr_collect_prestart_rp(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count);

/* FsDkrError variants, in error.rs declaration order (error.rs:6-60). */
#define FSDKR_ERR_NONE 0
#define FSDKR_ERR_PARTIES_THRESHOLD_VIOLATION 1
#define FSDKR_ERR_PUBLIC_SHARE_VALIDATION 2
#define FSDKR_ERR_SIZE_MISMATCH 3
#define FSDKR_ERR_PDL_W_SLACK_PROOF 4
#define FSDKR_ERR_RING_PEDERSEN_PROOF 5
#define FSDKR_ERR_RANGE_PROOF 6
#define FSDKR_ERR_MODULI_TOO_SMALL 7
#define FSDKR_ERR_PAILLIER_VERIFICATION 8
#define FSDKR_ERR_NEW_PARTY_UNASSIGNED_INDEX 9
#define FSDKR_ERR_BROADCASTED_PUBLIC_KEY 10
#define FSDKR_ERR_DLOG_PROOF_VALIDATION 11
#define FSDKR_ERR_RING_PEDERSEN_PROOF_VALIDATION 12

typedef struct fsdkr_error {
  int32_t variant;        /* FSDKR_ERR_*                                                 */
  int32_t panic;          /* 1: the reference panics at this point instead of returning */
  uint32_t f[4];          /* payload fields in declaration order                         */
  uint32_t keys_applied;  /* messages (R first, then J) whose ek was written into
                             local_key.paillier_key_vec before the error (:394, :436)   */
} fsdkr_error;

/* Map verdicts to the FIRST failing check in collect() order:
 * threshold, sizes, Feldman (k, i), [PDL then range (or its index panic)] (k, i), ring-Pedersen
 * (refresh, then join), per refresh message correct-key then modulus size,
 * per join message index, correct-key, DLog, modulus size.  `verdicts` may be
 * NULL when the threshold or size check already fails.  Pure host logic. */
int fsdkr_collect_first_error(const fsdkr_collect_batch* batch, const fsdkr_verdicts* verdicts, fsdkr_error* out);
/* fsdkr_collect_first_error for `count` sessions of a multi-session batch
 * (fsdkr_collect_prepare_multi / fsdkr_verify_collect_multi): out[s] from
 * batches[s] and verdicts[s], in one call (each session's collect() outcome is
 * its own, refresh_message.rs:321-467 per session).  Stops at the first session
 * whose mapping fails and returns that code.  Pure host logic. */
int fsdkr_collect_first_error_multi(const fsdkr_collect_batch* batches, const fsdkr_verdicts* verdicts, uint32_t count,
                                    fsdkr_error* out);

/* Fixed-base batch: out[i] = bases[base_idx[i]] ^ exp[i] mod mods[base_mod_idx[base_idx[i]]]
 * (exact).  The GPU builds one squaring chain of base^(2^(w j)) per base and
 * evaluates every exponent with Brickell-Gordon-McCurley-Wilson windowing, or,
 * when many exponents share a base, with a Lim-Lee comb over the chain (tables
 * of 2^h products per base: b - 1 squarings and v b products per exponent;
 * the context flag FSDKR_CFG_FB_BGMW forces BGMW); results are identical to fsdkr_modexp_batch.  This is the engine behind the bases the
 * reference exponentiates many times with curv BigInt::mod_pow: h1, h2 of a
 * receiver's DLogStatement (zk_pdl_with_slack.rs:144-157, range_proofs.rs:129-137)
 * and ring-Pedersen T (ring_pedersen_proof.rs:144).  mod_limbs in {64, 96}. */
int fsdkr_fixed_base_modexp(fsdkr_ctx* ctx, uint32_t mod_limbs, uint32_t n_bases, const uint32_t* bases,
                            const uint32_t* base_mod_idx, const uint32_t* mods, uint32_t n_mod, uint32_t count,
                            const uint32_t* base_idx, const uint32_t* exp, uint32_t exp_limbs, uint32_t* out);

/* ---- Stand-alone checks (JoinMessage::collect, per-proof callers) ---------
 * Feldman share checks of validate_collect (refresh_message.rs:177-188, curv
 * VerifiableSS::validate_share_public): verdict[k*n + i] = 1 iff
 * commit[k*n + i] == sum_j vss[k][j] * (i+1)^j.  vss: [n_msgs][t+1][16],
 * commit: [n_msgs*n][16] affine points ((0,0) = infinity). */
/* PDLwSlackProof::verify's u1 equation (zk_pdl_with_slack.rs:124-127, :158):
 * verdict[p] = 1 iff G*(s1[p] mod q) + Q[p]*(q - e[p] mod q) == u1[p].  s1:
 * [count][s1_len] limbs (any width), e: [count][8], Q / u1: [count][16] affine
 * points ((0,0) = infinity).  The collect() pipeline runs the same kernel
 * (pdl_u1_kernel: four lanes per pair over the GLV split of both scalars). */
int fsdkr_pdl_u1_check(fsdkr_ctx* ctx, uint32_t count, const uint32_t* s1, uint32_t s1_len, const uint32_t* e,
                       const uint32_t* Q, const uint32_t* u1, uint8_t* verdict);
int fsdkr_feldman_check(fsdkr_ctx* ctx, uint32_t n_msgs, uint32_t n, uint32_t t, const uint32_t* vss,
                        const uint32_t* commit, uint8_t* verdict);
/* RingPedersenProof::verify (ring_pedersen_proof.rs:126-157) for `count`
 * independent proofs: S, T, N: [count][nl]; A: [count][M][nl]; Z: [count][M][zl].
 * verdict[m] bit0 = Ok(()), bit1 = the reference panics (challenge shorter
 * than M bits and every check before the panicking index passes, or N = 0);
 * 0 = Err(RingPedersenProofError).  Any N: an even N = 2^k m is checked modulo
 * m (Montgomery) and modulo 2^k (pow2.hip).  Called by JoinMessage::collect
 * (add_party_message.rs:146-167). */
int fsdkr_ring_pedersen_verify(fsdkr_ctx* ctx, uint32_t nl, uint32_t count, uint32_t m_security, uint32_t zl,
                               const uint32_t* S, const uint32_t* T, const uint32_t* N, const uint32_t* A,
                               const uint32_t* Z, uint8_t* verdict);

/* The prime walk above it (kzen-paillier Paillier::keypair_with_modulus_size's
 * prime generation, restated: the walk oracle/keygen.py follows).  `count`
 * probable primes of `bits` bits (bits >= 64; top two bits set) by independent
 * walks: walk w draws a start s (`draw`: bits uniform random bits, OR-ed with
 * 3 << (bits-2) | 1) and returns the first of s, s+2, ..., s+2(span-1) that has
 * no odd prime factor below 2000, passes a Miller-Rabin round to base 2 and
 * MR rounds 8 more rounds to bases 2 + (SHA-256("fsdkr-mr" | c | j | ctr)
 * stream mod (c - 3)); a walk with no prime draws a new start after every walk
 * of its pass is settled.  Draw order: every walk's start first, in walk order.
 * The base-2 rounds of `window` survivors of every unsettled walk run as one GPU
 * launch (fsdkr_miller_rabin), then the extra rounds of each walk's first
 * passer.  span 0 = 4 * bits, window 0 = max(32, bits / 8).  out: [count][limbs],
 * limbs >= ceil(bits / 32).  `draw` returns 0 on success (non-zero aborts with
 * FSDKR_E_ARG). */
typedef int (*fsdkr_draw_bits_fn)(void* user, uint32_t bits, uint32_t* out, uint32_t limbs);
int fsdkr_sample_primes(fsdkr_ctx* ctx, uint32_t bits, uint32_t count, uint32_t window, uint32_t span,
                        fsdkr_draw_bits_fn draw, void* user, uint32_t* out, uint32_t limbs);

/* ---- Job 1: Paillier encryption of the shares (refresh_message.rs:72-84) ----
 * out[k] = (1 + m[k] N) * r[k]^N mod N^2, N = ns[n_idx[k]]  (kzen-paillier
 * encrypt_with_chosen_randomness).  m: [count][ml], r: [count][nl] (< N),
 * ns: [n_keys][nl], out: [count][2nl]. */
int fsdkr_paillier_encrypt(fsdkr_ctx* ctx, uint32_t nl, uint32_t count, const uint32_t* m, uint32_t ml,
                           const uint32_t* r, const uint32_t* n_idx, const uint32_t* ns, uint32_t n_keys,
                           uint32_t* out);

/* ---- share recovery building blocks (refresh_message.rs:367-373, 439-464) ---
 * Both run on the context's recovery stream, so they overlap a batch started
 * with fsdkr_collect_launch (collect() recovers the share speculatively while
 * the proofs are verified and discards it if a check fails).
 * Paillier decryption of `count` ciphertexts [count][2nl] under one key
 * dk = (p, q) (each [nl], zero-padded), kzen-paillier CRT form
 * (Paillier::decrypt, refresh_message.rs:439); the exponentiations and the
 * CRT constants' inverses run on the GPU.  m_out: [count][nl]. */
int fsdkr_paillier_decrypt(fsdkr_ctx* ctx, uint32_t nl, uint32_t count, const uint32_t* c, const uint32_t* p,
                           const uint32_t* q, uint32_t* m_out);
/* The same for many keys (one per session of fsdkr_verify_collect_multi):
 * ciphertext k is decrypted under key key_idx[k] of p, q: [n_keys][nl]. */
int fsdkr_paillier_decrypt_multi(fsdkr_ctx* ctx, uint32_t nl, uint32_t count, const uint32_t* c,
                                 const uint32_t* key_idx, const uint32_t* p, const uint32_t* q, uint32_t n_keys,
                                 uint32_t* m_out);
/* out[o] = sum_j scalars[o][j] * points[o][j] on secp256k1 (affine 16-limb
 * points, 8-limb scalars reduced mod q on device): pk_vec entries and G*x.
 * One GPU thread per term, then one per output. */
int fsdkr_ec_msm(fsdkr_ctx* ctx, uint32_t count, uint32_t terms, const uint32_t* points, const uint32_t* scalars,
                 uint32_t* out);

/* Share recovery of collect() in one call, for `count` independent jobs (one
 * party of RefreshMessage::collect, JoinMessage::collect, or one session of a
 * multi-session batch): refresh_message.rs:367-373 (get_ciphertext_sum) and
 * :439-464 (Paillier::decrypt, x_i, y, pk_vec), add_party_message.rs:183-213.
 * Job j: the Lagrange weights l_k of the first t_vss+1 messages' old indices
 * (curv map_share_to_new_params), the decryption of the party's ciphertext
 * from each of them under (p, q), new share = (sum_k l_k Dec(c_k) mod N) mod q
 * (decryption is a homomorphism on units of Z_{N^2}: the reference's decryption
 * of prod_k c_k^l_k * Enc(0)), y = G*share and pk_vec[i] = sum_{k <= t'}
 * l_k * points[i][k] for i < n_new, t' = min(t_key, t_vss).  The decryptions and
 * multi-scalar multiplications run on the GPU on the recovery stream (they
 * overlap a launched collect batch).  Index checks the reference performs by
 * indexing its own vectors (the party's ciphertext, t_vss+1 messages) belong to
 * the caller, which extracts the arrays below. */
typedef struct fsdkr_recover_job {
  uint32_t nl;                /* limbs of N = p q: 64, 96, 128 or 192 */
  uint32_t t_vss;             /* VSS threshold of local_key.vss_scheme: t_vss+1 messages combine */
  uint32_t t_key;             /* local_key.t: the pk_vec sums run k = 0..t_key (:460) */
  uint32_t n_new;             /* pk_vec entries to rebuild (refresh + join messages) */
  const uint32_t* old_index;  /* [t_vss+1] old_party_index of message k (1-based) */
  const uint32_t* cts;        /* [t_vss+1][2nl] points_encrypted_vec[i-1] of message k, each below
                                 2^(64 nl): the caller reduces a wider ciphertext mod N^2 first
                                 (Paillier::mul / add / decrypt work mod N^2, so c + k N^2
                                 recovers like c) */
  const uint32_t* p;          /* [nl] */
  const uint32_t* q;          /* [nl] */
  const uint32_t* points;     /* [n_new][min(t_key,t_vss)+1][16] points_committed_vec[i] of message k
                                 (n_new rows of the caller's choosing: a multi-GPU rank passes
                                 its slice of the new parties) */
  uint32_t flags;             /* FSDKR_RECOVER_* flags below (0: the whole recovery) */
} fsdkr_recover_job;
/* job flag: only the pk_vec rows; no decryption (share and y are zero).  The
 * ranks of a sharded collect() split the pk_vec rows and one of them decrypts
 * (fsdkr/shard.py); the results travel with the verdict all-reduce. */
#define FSDKR_RECOVER_NO_DECRYPT 1u
/* status of a recovered job */
#define FSDKR_RECOVER_OK 0
#define FSDKR_RECOVER_PANIC_LI 1       /* t_key > t_vss: li_vec[k] out of bounds in the pk_vec loop (:460-462) */
#define FSDKR_RECOVER_PANIC_DECRYPT 2  /* the decryption key is degenerate (p == q, even, 1): Paillier::decrypt */
typedef struct fsdkr_recovered {
  uint32_t share[8];          /* new x_i, reduced mod q */
  uint32_t y[16];             /* G * x_i (affine; (0,0) = infinity) */
  uint32_t* pk_vec;           /* caller's [n_new][16] */
  int32_t status;             /* FSDKR_RECOVER_* */
} fsdkr_recovered;
int fsdkr_collect_recover(fsdkr_ctx* ctx, const fsdkr_recover_job* jobs, uint32_t count, fsdkr_recovered* out);
/* The same as two calls, so the recovery overlaps the caller's other work: _launch
 * copies every input, does the host pre-pass (Lagrange weights, CRT constants,
 * ciphertext reductions) and enqueues the GPU work (the decryption
 * exponentiations, the pk_vec MSM) on the recovery stream, then returns;
 * _finish waits for it and fills `out` as fsdkr_collect_recover does.  One
 * recovery in flight per context; collect() launches it before its own
 * pipeline (refresh_message.rs:439-464 only reads inputs the caller holds
 * before verification). */
int fsdkr_collect_recover_launch(fsdkr_ctx* ctx, const fsdkr_recover_job* jobs, uint32_t count);
int fsdkr_collect_recover_finish(fsdkr_ctx* ctx, fsdkr_recovered* out);

/* Kernel timing (needs FSDKR_CFG_TIMING): accumulated milliseconds and launch
 * count of kernel `name` since the last reset ("modexp", "mod_setup", ...). */
int fsdkr_kernel_time(const fsdkr_ctx* ctx, const char* name, double* ms, uint32_t* launches);
void fsdkr_kernel_time_reset(fsdkr_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* FSDKR_FSDKR_H */
