// Internal declarations of the batched collect() verification, shared by
// collect_prestart.cpp (fsdkr_collect_prestart[_multi]: GA chains and fixed-base
// tables started from the stage-1 fields), collect_prepare.cpp (the host pre-pass
// and the device image), collect_launch.cpp (the kernel pipeline and the verdict
// readback) and collect.cpp (first-error mapping and the C ABI).
//
// Reference: /root/reference/src/refresh_message.rs:321-467 (collect),
// :147-191 (validate_collect); zk_pdl_with_slack.rs:113-188; range_proofs.rs:112-164;
// ring_pedersen_proof.rs:126-157; zk-paillier NiCorrectKeyProof / CompositeDLogProof.
#pragma once
#include <hip/hip_runtime.h>
#include <openssl/evp.h>

#include "evp_sha.hpp"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "ctx.hpp"
#include "fbjob.hpp"
#include "fsdkr/fsdkr.h"
#include "hostbn.hpp"
#include "kernels.h"
#include "sha256.hpp"
#include "verify.h"

namespace fsdkr {


constexpr uint32_t CK_M2 = 11;      // zk-paillier correct_key_ni M2
constexpr uint32_t CK_ALPHA = 6370; // zk-paillier primorial bound [dep, unverified]
const uint8_t SALT[4] = {75, 90, 101, 110};  // SALT_STRING "KZen" [dep, unverified]

const uint32_t Q_LIMBS_H[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                               0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

inline const std::vector<uint32_t>& small_primes() {
  static std::vector<uint32_t> ps = [] {
    std::vector<uint32_t> v;
    std::vector<bool> comp(CK_ALPHA, false);
    for (uint32_t i = 2; i < CK_ALPHA; ++i) {
      if (comp[i]) continue;
      v.push_back(i);
      for (uint32_t j = i * i; j < CK_ALPHA; j += i) comp[j] = true;
    }
    return v;
  }();
  return ps;
}

// the primorial check of the correct-key proof over keys of up to 192 limbs
inline const hbn::SmallFactorSieve& small_factor_sieve() {
  static const hbn::SmallFactorSieve sv(small_primes(), 192);
  return sv;
}

// q^3 (the Alice s1 bound, range_proofs.rs:125) as limbs
inline const hbn::Limbs& q_cubed() {
  static hbn::Limbs q3 = [] {
    const hbn::Limbs q = hbn::from(Q_LIMBS_H, 8);
    return hbn::mul(hbn::mul(q, q), q);
  }();
  return q3;
}

inline bool is_odd(const uint32_t* p) { return (p[0] & 1u) != 0; }

// to_bytes(x) absorbed for a small non-negative integer
inline void absorb_u32(Sha256& h, uint32_t v) { h.bigint(&v, 1); }

// curv BigInt::to_bytes of little-endian u32 limbs: the minimal big-endian
// magnitude, zero as one 0x00 byte
inline void put_bigint(std::vector<uint8_t>& out, const uint32_t* x, uint32_t n) {
  int top = (int)n - 1;
  while (top >= 0 && x[top] == 0) --top;
  if (top < 0) {
    out.push_back(0);
    return;
  }
  int sh = 24;
  while (sh > 0 && ((x[top] >> sh) & 0xffu) == 0) sh -= 8;
  for (; sh >= 0; sh -= 8) out.push_back((uint8_t)(x[top] >> sh));
  for (int k = top - 1; k >= 0; --k) {
    const uint32_t v = x[k];
    const uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    out.insert(out.end(), b, b + 4);
  }
}

// BigInt::from_bytes(P.to_bytes(true)) re-encoded by to_bytes: 33 bytes for a
// finite point (x limbs 0..7, y limbs 8..15, prefix 2 + y mod 2), 0x00 for infinity
inline void put_point(std::vector<uint8_t>& out, const uint32_t* p16) {
  bool inf = true;
  for (int i = 0; i < 16; ++i) inf = inf && p16[i] == 0;
  if (inf) {
    out.push_back(0);
    return;
  }
  out.push_back((uint8_t)(2 + (p16[8] & 1u)));
  for (int i = 7; i >= 0; --i) {
    const uint32_t v = p16[i];
    const uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    out.insert(out.end(), b, b + 4);
  }
}

// the secp256k1 generator G, compressed (zk_pdl_with_slack.rs:114: G.to_bytes(true))
const uint8_t G_COMPRESSED[33] = {0x02, 0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0,
                                  0x62, 0x95, 0xCE, 0x87, 0x0B, 0x07, 0x02, 0x9B, 0xFC, 0xDB, 0x2D,
                                  0xCE, 0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98};

// SHA-256 digest as a 256-bit little-endian limb array (BigInt::from_bytes(digest))
inline void digest_le(const uint8_t* d, uint32_t* e8) {
  for (int i = 0; i < 8; ++i)
    e8[i] = ((uint32_t)d[28 - 4 * i] << 24) | ((uint32_t)d[29 - 4 * i] << 16) | ((uint32_t)d[30 - 4 * i] << 8) |
            (uint32_t)d[31 - 4 * i];
}

// One thread's SHA-256 context (OpenSSL: SHA-NI / AVX2 code paths where the CPU has them)
struct HostSha {
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  std::vector<uint8_t> buf;
  ~HostSha() { EVP_MD_CTX_free(ctx); }
  bool digest(uint32_t* e8) {
    uint8_t d[32];
    unsigned int len = 0;
    const bool ok = ctx && EVP_DigestInit_ex(ctx, sha256_md(), nullptr) == 1 &&
                    EVP_DigestUpdate(ctx, buf.data(), buf.size()) == 1 && EVP_DigestFinal_ex(ctx, d, &len) == 1 &&
                    len == 32;
    if (ok) digest_le(d, e8);
    return ok;
  }
};

using RowsSha = std::array<uint8_t, 32>;

// PDL challenge e = H(G, Q, c, z, u1, u2, u3) of pair lp of batch b as 8 little-endian
// limbs (zk_pdl_with_slack.rs:114-122; every value as curv's to_bytes)
inline bool pdl_challenge(HostSha& sha, const fsdkr_collect_batch* b, size_t lp, uint32_t* e8) {
  const uint32_t w = b->nl;
  sha.buf.clear();
  sha.buf.insert(sha.buf.end(), G_COMPRESSED, G_COMPRESSED + 33);
  put_point(sha.buf, b->commit + lp * 16);
  put_bigint(sha.buf, b->enc + lp * 2 * w, 2 * w);
  put_bigint(sha.buf, b->pdl_z + lp * w, w);
  put_point(sha.buf, b->pdl_u1 + lp * 16);
  put_bigint(sha.buf, b->pdl_u2 + lp * 2 * w, 2 * w);
  put_bigint(sha.buf, b->pdl_u3 + lp * w, w);
  return sha.digest(e8);
}

// f(begin, end) over [0, n) on up to host_threads() threads (inline when small)
template <class F>
inline void parallel_for(size_t n, size_t grain, F&& f) {
  const size_t want = grain ? (n + grain - 1) / grain : 1;
  const size_t chunks = std::min<size_t>(host_threads(), want);
  if (chunks <= 1) {
    f((size_t)0, n);
    return;
  }
  struct Part {
    F* f;
    size_t n, chunks;
  } part{&f, n, chunks};
  host_pool_run(chunks, [](void* a, size_t c) {
    const Part& x = *static_cast<const Part*>(a);
    (*x.f)(x.n * c / x.chunks, x.n * (c + 1) / x.chunks);
  }, &part);
}

// a[0, words) == b[0, words), compared in parallel chunks
inline bool words_equal(const uint32_t* a, const uint32_t* b, size_t words) {
  if (words < (1u << 16)) return memcmp(a, b, words * 4) == 0;
  std::atomic<bool> eq{true};
  parallel_for((words + 65535) / 65536, 1, [&](size_t c0, size_t c1) {
    const size_t lo = c0 * 65536, hi = std::min(words, c1 * 65536);
    if (eq.load(std::memory_order_relaxed) && memcmp(a + lo, b + lo, (hi - lo) * 4) != 0) eq = false;
  });
  return eq;
}

// FSDKR_PREP_PROFILE=1: host pre-pass phase times on stderr (diagnostics)
struct PhaseClock {
  bool on = getenv("FSDKR_PREP_PROFILE") != nullptr;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  void lap(const char* what) {
    if (!on) return;
    const auto t1 = std::chrono::steady_clock::now();
    fprintf(stderr, "[prep] %-16s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
    t0 = t1;
  }
};

// Image planner: offsets are assigned first, the bytes are written into the
// pinned arena afterwards (rows re-packed to the merged limb width, in parallel).
struct Img {
  struct Op {
    size_t dst;
    const uint8_t* src;
    size_t rows, src_stride, dst_stride;   // bytes
  };
  std::vector<Op> ops;
  std::vector<std::vector<uint8_t>> owned;
  size_t size = 0;
  static size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
  size_t reserve(size_t bytes) {
    const size_t o = al(size);
    size = o + al(bytes ? bytes : 1);
    return o;
  }
  // `rows` rows of w_src words written at `dst` with stride w_dst >= w_src words (zero-padded)
  void rows_at(size_t dst, const uint32_t* src, size_t rows, uint32_t w_src, uint32_t w_dst) {
    if (!rows) return;
    ops.push_back({dst, reinterpret_cast<const uint8_t*>(src), rows, (size_t)w_src * 4, (size_t)w_dst * 4});
  }
  size_t own_at(size_t dst, std::vector<uint8_t>&& b) {
    owned.push_back(std::move(b));
    const std::vector<uint8_t>& v = owned.back();
    if (!v.empty()) ops.push_back({dst, v.data(), 1, v.size(), v.size()});
    return dst;
  }
  template <class T>
  size_t own(const std::vector<T>& v) {
    std::vector<uint8_t> b(v.size() * sizeof(T));
    if (!b.empty()) memcpy(b.data(), v.data(), b.size());
    const size_t o = reserve(b.size());
    return own_at(o, std::move(b));
  }
  void materialize(uint8_t* base) const {
    // split big row copies into ~1 MB pieces so the threads share the work
    struct Piece {
      const Op* op;
      size_t r0, r1;
    };
    std::vector<Piece> pieces;
    for (const Op& op : ops) {
      const size_t per = std::max<size_t>(1, (1u << 20) / std::max<size_t>(op.dst_stride, 1));
      for (size_t r = 0; r < op.rows; r += per) pieces.push_back({&op, r, std::min(op.rows, r + per)});
    }
    parallel_for(pieces.size(), 4, [&](size_t b, size_t e) {
      for (size_t k = b; k < e; ++k) {
        const Op& op = *pieces[k].op;
        if (op.src_stride == op.dst_stride) {
          memcpy(base + op.dst + pieces[k].r0 * op.dst_stride, op.src + pieces[k].r0 * op.src_stride,
                 (pieces[k].r1 - pieces[k].r0) * op.dst_stride);
          continue;
        }
        for (size_t r = pieces[k].r0; r < pieces[k].r1; ++r) {
          uint8_t* d = base + op.dst + r * op.dst_stride;
          memcpy(d, op.src + r * op.src_stride, op.src_stride);
          memset(d + op.src_stride, 0, op.dst_stride - op.src_stride);
        }
      }
    });
  }
};

// one session's place in the merged image
struct Sess {
  const fsdkr_collect_batch* b;
  uint32_t R, J, n, Mt, P, V;
  uint32_t rbase, mbase, jbase, pbase, vbase;
  uint32_t ckl;
};

inline uint32_t ncoef_of(const fsdkr_collect_batch* b, uint32_t k) { return b->vss_len ? b->vss_len[k] : b->t + 1; }

// ------------------------------------------------------------------------------
// Everything launch()/finish() need after the host pre-pass and the upload.
struct CollectPlan {
  // merged shape
  uint32_t S = 0, n = 0, P = 0, Mt = 0, J = 0, M = 0, nl = 0, nn = 0, ckl = 0, s1l = 0, el = 0;
  std::vector<Sess> ss;               // per-session offsets (batch pointers are not kept)
  size_t out_off = 0, total = 0;
  uint8_t* dev = nullptr;
  // input offsets used by launches
  size_t o_Q, o_enc, o_pz, o_pu1, o_pu2, o_pu3, o_ps1, o_pA, o_az, o_ae, o_vss, o_NN, o_mods, o_ckmods, o_one, o_epdl;
  size_t d_finfo = 0, d_p2 = 0;
  uint32_t n_mods_nl = 0, n_p2 = 0;
  // output offsets
  size_t x_pbits, x_ppanic, x_Bpdl, x_gs1, x_invc, x_invz, x_unn, x_uzA, x_uzp, x_eq2, x_eq3, x_eqck, x_u,
      x_w, x_fel, x_pdlv, x_rng, x_p2;
  // modexp jobs: 0 GA (nn long), 1 GD (nl: DLog), 2 J2 (nn short), 3 J5 (nl short), 4 GC (ckl: correct key)
  static constexpr int NJOB = 5;
  size_t d_J[NJOB], x_J[NJOB];
  uint32_t jk32[NJOB], jcount[NJOB], jbits[NJOB], jflags[NJOB] = {};   // jflags: launch_modexp_desc desc_flags
  // descriptor offsets
  size_t d_bs, d_bn, d_iynn, d_imnn, d_iynl, d_imnl, d_eqnn, d_eqnnm, d_eqnl, d_eqnlm, d_eqck, d_eqckm, d_p3nn, d_p3nl,
      d_p3m, d_ahn, d_ahc, d_alpre;
  size_t d_p3mnl = 0;    // moduli of the nl prod3 rows (d_p3m, + the negative-s3 rows)
  uint32_t n_p3nl = 0;   // P + pairs with a negative PDL s3
  uint32_t n_inv_nn = 0, n_eq_nn = 0, n_eq_nl = 0, n_eq_ck = 0;
  // the pairs grouped by receiver (Montgomery's simultaneous inversion of the
  // per-pair inverses: c^-1 mod N_i^2, (z^e)^-1 mod Ñ_i; inverse_batch_kernel)
  size_t d_binv_order = 0, d_binv_gstart = 0;
  uint32_t binv_ngroups = 0;
  // host-side pre-verdicts
  std::vector<uint32_t> cpdl_extra;
  std::vector<uint8_t> ck_pre, dlog_pre;   // dlog_pre: bit0 / bit1 per proof
  std::vector<uint8_t> ped_mode;           // 0 regular, 1 odd part 1 (Montgomery half holds), 2 modulus 0 (abort)
  std::vector<uint8_t> dlog_trivial;       // odd part of the DLog N is 1
  std::vector<uint32_t> ped_p2_first, dlog_p2_first;   // first 2-adic op of an even message / join (~0: none)
  std::vector<uint32_t> ped_zlen;          // readable Z entries (M: all); A short: ped_mode 2
  std::vector<uint8_t> ck_short;           // sigma_vec shorter than 11 (or n = 0): zk-paillier panics
  std::vector<uint8_t> ck_one;             // n = 1: the proof verifies trivially
  std::vector<uint32_t> e_pdl;             // PDL challenges [P][8] (host, prepare), also uploaded at o_epdl
  // s^N mod N^2 results computed by fsdkr_collect_prestart (ga_hit): the eq / prod3
  // operands read them from the prestart buffer once ga_done has fired
  bool ga_hit = false;
  hipEvent_t ga_done = nullptr;
  // the prestart's Montgomery constants of the N_i^2 (the same rows launch() needs
  // for J2 / eq / prod3), ready at ga_setup: launch() reuses them instead of
  // running its own mod_setup on the main chain
  const uint32_t* pre_cons_nn = nullptr;
  bool pre_cons_wide = false;
  hipEvent_t ga_setup = nullptr;
  // h1 / h2 fixed-base tables built by fsdkr_collect_prestart (fb_hit)
  bool fb_hit = false;
  FbPre fb_pre;
  // correct-key sigma^n mod n computed by fsdkr_collect_prestart_multi (ck_hit):
  // the correct-key equalities read them once ck_done has fired
  bool ck_hit = false;
  hipEvent_t ck_done = nullptr;
  // ring-Pedersen T^Z computed by fsdkr_collect_prestart_rp (tz_hit): the RP
  // equalities read them once tz_done has fired
  bool tz_hit = false;
  hipEvent_t tz_done = nullptr;
  // GA's joint tail (ga_split_ok): J2 is not run; GA computes s2^N c^-e_pdl | s^N c^-e_A,
  // the nn inverse is c's own (unit flags of c); job slot 2 then holds J9
  bool joint = false;
  size_t d_desc2 = 0;                  // the tail's descriptor block (in the image)
  struct GaTail {                      // a split prestarted head's launch (ga_hit && joint)
    const uint8_t* desc = nullptr;
    const uint32_t* cons = nullptr;
    uint32_t* out = nullptr;
    uint32_t count = 0, bits = 0, group = 0, flags = 0;
  } ga_tail;
  std::vector<uint8_t> ae_zero;        // Alice e == 0: c^0 = 1 whatever c is
  // device words finish reads back (the plan's output region)
  const void *r_unn = nullptr, *r_uzA = nullptr, *r_uzp = nullptr, *r_pdlv = nullptr, *r_fel = nullptr;
  FbJob fb;
  size_t d_FB = 0;
  uint32_t* fb_table = nullptr;
  uint16_t* fb_sched = nullptr;
  uint32_t* fb_nsteps = nullptr;
  uint8_t* fb_comb = nullptr;   // comb scratch of fb's comb groups (FbJob::plan_comb)
  bool launched = false;
};


// The long-exponent job GA's J1 half (s2^N | s^N mod N^2 per pair, 2P 4096-bit
// chains: the critical path of the pipeline) started by fsdkr_collect_prestart
// from the few fields it reads, while the caller still packs the rest of the
// batch.  A later prepare of a batch with the same values consumes the results.
struct GaPre {
  bool valid = false;
  uint32_t nl = 0, n = 0, R = 0;
  std::vector<uint32_t> recv_n, s2, s;   // the inputs (each session at its own nl), for the match in prepare
  struct Sess {
    uint32_t nl, n, R;
    size_t rbase, pbase;   // first global receiver / pair of the session
  };
  std::vector<Sess> sess;
  uint32_t* out = nullptr;               // [2P][nn]: J1 instance order (s2^N rows, then s^N rows)
  hipEvent_t done = nullptr;
  // split GA (ga_split_ok): the prestart ran the HEAD; prepare launches the joint tail
  // with these descriptors (ga_rows: out_idx of every instance, pads = 2P)
  bool split = false;
  uint32_t ga_group = 0, ga_flags = 0, ga_count = 0, ga_bits = 0;
  const uint8_t* ga_desc = nullptr;
  std::vector<uint32_t> ga_rows;
  hipEvent_t ga_setup = nullptr;   // GA's Montgomery constants ready (before its chains)
  hipEvent_t ga_rows_up = nullptr;  // the pair rows and descriptors copied up (beside the moduli setup)
  const uint32_t* cons = nullptr;   // those constants (KD 160 when `wide`, else the width's KD)
  bool wide = false;
  // the fixed-base tables of h1_i, h2_i (bases 2i, 2i+1 of prepare's FbJob), built
  // for exponents of up to bits_h1 / bits_h2 bits with window w
  bool fb_valid = false;
  std::vector<uint32_t> ntilde, h1, h2, T, pedmod;   // bases, and the T_m moduli rows
  std::vector<uint64_t> fb_bptr;                      // device rows of the bases [h1_i | T_m | h2_i]
  uint32_t Mt = 0, fb_w = 0, bits_h1 = 0, bits_h2 = 0, bits_z = 0, fb_entries = 0;
  uint32_t* fb_table = nullptr;
  hipEvent_t fb_done = nullptr;     // every table built
  hipEvent_t fb_setup = nullptr;    // the table chains' moduli constants ready (fb_cons)
  // Lim-Lee comb tables of the base classes (FbJob::plan_comb), built on the
  // chains' stream after them: prepare's and prestart_rp's combs take them
  std::vector<CombPre> comb_pre;
  hipEvent_t comb_done = nullptr;
  // correct-key sigma_k^n mod n of every message (prepare's GC job), when stage 1
  // packed ck_n and ck_sigma: rows at width ck_l, in prepare's message order
  bool ck_valid = false;
  uint32_t ck_l = 0, ck_bits = 0, ck_Mt = 0;
  std::vector<uint32_t> ck_n, ck_sigma;   // the inputs (zero-extended to ck_l), for the match
  uint32_t* ck_out = nullptr;             // [Mt * 11][ck_l]
  hipEvent_t ck_done = nullptr;
  // the constants of the table chains' moduli [Ntilde_i | RP modulus_m] (rows n + m: T_m's)
  const uint32_t* fb_cons = nullptr;
  // ring-Pedersen T_m^Z_{m,k} of every message (fsdkr_collect_prestart_rp): the
  // fixed-base exponents behind the prestarted T tables, rows m*M + k at width nl;
  // prepare drops them from its fixed-base job when the T rows and the Z rows' SHA-256 match
  bool tz_valid = false;
  uint32_t tz_Mt = 0, tz_M = 0;
  std::vector<RowsSha> tz_sha;             // SHA-256 of the Z rows, per block of kShaRows rows
  uint32_t* tz_out = nullptr;
  const uint32_t* tz_z = nullptr;        // the device copy of the Z rows [Mt*M][tz_zl]
  uint32_t tz_zl = 0;
  hipEvent_t tz_done = nullptr;
};

// SHA-256 of a sequence of rows, one digest per block of kShaRows consecutive rows
// (computed in parallel, one block per task).  A row enters as its length in words
// without trailing zero words (u32) and those words, so rows of equal value hash
// alike at any packed width and the encoding is injective.  Prestart and prepare
// compare the ring-Pedersen Z rows with it: equal digest vectors mean equal rows
// up to a SHA-256 collision.  `row(r)` returns {pointer, width} of global row r.
constexpr size_t kShaRows = 2048;
std::vector<RowsSha> rows_sha256(size_t rows, const std::function<std::pair<const uint32_t*, uint32_t>(size_t)>& row);

// collect()'s fixed-base tables, base order [h1_i | T_m | h2_i] (FbJob::finalize
// sizes: one entry per w exponent bits, at least one)
struct FbLayout {
  std::vector<uint32_t> h, toff, mod;
  uint32_t entries = 0;
};
inline FbLayout fb_layout(uint32_t n, uint32_t Mt, uint32_t w, uint32_t bits_h1, uint32_t bits_h2, uint32_t bits_z) {
  FbLayout L;
  auto add = [&](uint32_t bits, uint32_t mod) {
    const uint32_t h = std::max(1u, (bits + w - 1) / w);
    L.h.push_back(h);
    L.toff.push_back(L.entries);
    L.mod.push_back(mod);
    L.entries += h;
  };
  for (uint32_t r = 0; r < n; ++r) add(bits_h1, r);
  for (uint32_t m = 0; m < Mt; ++m) add(bits_z, n + m);
  for (uint32_t r = 0; r < n; ++r) add(bits_h2, r);
  return L;
}

// Modulus row of message m's ring-Pedersen T^Z checks, as prepare's pre-pass
// derives it: the odd part of N, or the placeholder 3 when the proof panics
// before any check (A shorter than M, N = 0) or the odd part is 1.
inline void ped_modulus(const fsdkr_collect_batch* b, uint32_t m, uint32_t M, uint32_t nl, uint32_t* on) {
  const uint32_t* N = b->ped_N + (size_t)m * b->nl;
  std::fill(on, on + nl, 0u);
  const bool panics = (b->ped_lens && b->ped_lens[2 * m] < M) || hbn::is_zero_raw(N, b->nl);
  if (!panics) {
    memcpy(on, N, (size_t)b->nl * 4);
    const uint32_t tz = hbn::ctz_raw(N, b->nl);
    if (tz) hbn::shr_raw(on, nl, tz);
    if (!(on[0] == 1 && hbn::is_zero_raw(on + 1, nl - 1))) return;
  }
  std::fill(on, on + nl, 0u);
  on[0] = 3;
}

// GA lanes per instance.  GA's chains are the pipeline's critical path and share
// the chip with every other stream.  With quotient-scaled rows (modexp.hip QS)
// the 16-lane 4096-bit shape issues fewer instructions per row than 8 lanes and
// fits three waves per SIMD (98 VGPRs): n = 64 (7 680 chains) went from 57.4 to
// 51.5 ms per call against 8 lanes (profiles/r04/r04d_ab_lanes_v*).  Small
// batches (multi-GPU shards) keep 16 lanes too: with the sliding windows and the
// joint tail (which the one-wave-per-chain modexp_wave_kernel and the fixed-window
// 32-lane shape lack) an emulated 8-way n = 64 rank-0 call takes 18.6 ms against
// 22.3 (wave shape) and 20.5-21.2 (32-lane sliding windows), and 4-way ranks
// 24.0-24.8 against 26.3-26.9 (profiles/r05/r05k_*, r05l_*, r05m_*).  Past 16 384
// chains the launch fills the chip several times over and the most MAC-efficient
// 4-lane shape wins: n = 256 (131 072 chains) 592 ms per call at 8 lanes, 571 ms
// at 4, 628 ms at 16 (profiles/r04/r04e_ab_n256_lanes_v*).  Used by the prestart
// and by launch().
inline uint32_t ga_lanes(uint32_t count, uint32_t nn) {
  if (nn != 128) return (uint64_t)count * 16 <= 65536u ? 16 : 8;
  return count <= 16384u ? 16 : 4;
}

// J2 (c^e mod N^2, 256-bit exponents) lanes per instance, when the joint tail
// does not absorb it
inline uint32_t j2_lanes(size_t count, uint32_t nn) {
  return nn == 128 ? (count <= 1024 ? kWaveGroup : count <= 16384 ? 16 : 8) : 8;
}

// GA's chains per wave when they are padded to whole waves per receiver: only the
// 4096-bit shapes have a sliding-window kernel that pads buy; the other widths
// (configs[4]'s 6144-bit GA, 6 chains per receiver) run fixed windows, where a
// pad is a whole duplicate chain (+33 % GA work at 8 per wave, profiles/r06/r06o_*)
inline uint32_t ga_per_wave(uint32_t group, uint32_t nn) { return (nn == 128 && group <= 64) ? 64 / group : 0u; }

// the descriptor flags of a regrouped GA job launched with `group` lanes
inline uint32_t ga_desc_flags(bool aligned_for, uint32_t group) {
  const bool slide_shape = group == 4 || group == 8 || group == 16 || group == kWideGroup;
  return kDescOutIdx | ((aligned_for && slide_shape) ? kDescSlide : 0u);
}

// GA's joint tail (modexp.hip modexp_tail_kernel): the chains s2^N | s^N mod N^2 run
// as a head over N's bits >= kGaSplit and a tail that multiplies c^-e_pdl | c^-e_A in
// along its squarings (e < 2^256), so no separate c^e chain (J2) runs.  For the
// sliding-window GA shapes (4096-bit, 4 / 8 / 16 / 32 lanes): n = 64 -0.8 ms,
// configs[3] -8 % against a separate J2 (profiles/r05/r05e_*, r05f_*)
constexpr uint32_t kGaSplit = 256;
// GA's issue priority (s_setprio of the prestarted chains and of the joint tail;
// priority 3 measured 0.5-1 ms slower at n = 64, profiles/r04/r04g_*)
inline uint32_t ga_prio() { return 2u; }
inline bool ga_split_ok(uint32_t nn, uint32_t group, uint32_t flags) {
  return nn == 128 && (flags & kDescSlide) && (flags & kDescOutIdx) &&
         (group == 4 || group == 8 || group == 16 || group == kWideGroup);
}
// the tail's per-instance descriptor block: base2_ptr u64 | exp2_ptr u64 | exp2_len u32
constexpr size_t kTailDescBytes = 20;

// collect_prestart.cpp
int prestart_ga(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count, uint32_t* n_out, uint32_t* P_out);
int collect_prestart_impl(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count);
int collect_prestart_rp_impl(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count);
bool ga_pre_matches(const Ctx* c, const fsdkr_collect_batch* bs, uint32_t count);
// collect_prepare.cpp
int collect_prepare_impl(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count);
// collect_launch.cpp
int collect_launch_impl(Ctx* c);
int collect_finish_impl(Ctx* c, fsdkr_verdicts* out, uint32_t count);
// collect.cpp
int first_error_impl(const fsdkr_collect_batch* b, const fsdkr_verdicts* v, fsdkr_error* e);

}  // namespace fsdkr
