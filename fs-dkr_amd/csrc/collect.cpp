// Host orchestration of the batched RefreshMessage::collect verification
// (fsdkr_verify_collect[_multi], prepare / launch / finish) and the first-error
// mapping (fsdkr_collect_first_error).
//
// Reference: /root/reference/src/refresh_message.rs:321-467 (collect),
// :147-191 (validate_collect); zk_pdl_with_slack.rs:113-188; range_proofs.rs:112-164;
// ring_pedersen_proof.rs:126-157; zk-paillier NiCorrectKeyProof / CompositeDLogProof.
//
// One call verifies one or many independent collect() sessions in ONE device
// pass: the sessions' pairs, receivers, messages and joins are concatenated
// into a single image (little-endian u32 limbs, one fixed width per field);
// every descriptor addresses rows of that image.  Pipeline (streams in
// launch()): ped_hash -> binom -> modexp jobs (GA, GD, GC, J2, J5, FB)
// -> inverses -> eq_check / prod3 -> alice_hash; pdl_u1, Feldman and the 2-adic
// checks of even moduli beside them -> one D2H of the verdict words (finish()).
#include <hip/hip_runtime.h>
#include <openssl/evp.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
namespace {

constexpr uint32_t CK_M2 = 11;      // zk-paillier correct_key_ni M2
constexpr uint32_t CK_ALPHA = 6370; // zk-paillier primorial bound [dep, unverified]
const uint8_t SALT[4] = {75, 90, 101, 110};  // SALT_STRING "KZen" [dep, unverified]

const uint32_t Q_LIMBS_H[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                               0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};

const std::vector<uint32_t>& small_primes() {
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

// q^3 (the Alice s1 bound, range_proofs.rs:125) as limbs
const hbn::Limbs& q_cubed() {
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
void put_bigint(std::vector<uint8_t>& out, const uint32_t* x, uint32_t n) {
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
void put_point(std::vector<uint8_t>& out, const uint32_t* p16) {
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
void digest_le(const uint8_t* d, uint32_t* e8) {
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
    const bool ok = ctx && EVP_DigestInit_ex(ctx, EVP_sha256(), nullptr) == 1 &&
                    EVP_DigestUpdate(ctx, buf.data(), buf.size()) == 1 && EVP_DigestFinal_ex(ctx, d, &len) == 1 &&
                    len == 32;
    if (ok) digest_le(d, e8);
    return ok;
  }
};

// f(begin, end) over [0, n) on up to host_threads() threads (inline when small)
template <class F>
void parallel_for(size_t n, size_t grain, F&& f) {
  const size_t want = grain ? (n + grain - 1) / grain : 1;
  const size_t chunks = std::min<size_t>(host_threads(), want);
  if (chunks <= 1) {
    f((size_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(chunks - 1);
  for (size_t c = 1; c < chunks; ++c) th.emplace_back([&, c] { f(n * c / chunks, n * (c + 1) / chunks); });
  f((size_t)0, n / chunks);
  for (auto& t : th) t.join();
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

}  // namespace

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
  uint32_t jk32[NJOB], jcount[NJOB], jbits[NJOB];
  // descriptor offsets
  size_t d_bs, d_bn, d_iynn, d_imnn, d_iynl, d_imnl, d_eqnn, d_eqnnm, d_eqnl, d_eqnlm, d_eqck, d_eqckm, d_p3nn, d_p3nl,
      d_p3m, d_ahn, d_ahc, d_alpre;
  uint32_t n_inv_nn = 0, n_eq_nn = 0, n_eq_nl = 0, n_eq_ck = 0;
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
  // h1 / h2 fixed-base tables built by fsdkr_collect_prestart (fb_hit)
  bool fb_hit = false;
  FbPre fb_pre;
  FbJob fb;
  size_t d_FB = 0;
  uint32_t* fb_table = nullptr;
  uint16_t* fb_sched = nullptr;
  uint32_t* fb_nsteps = nullptr;
  bool launched = false;
};

void free_collect_plan(Ctx* c) {
  delete reinterpret_cast<CollectPlan*>(c->plan);
  c->plan = nullptr;
}

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
  hipEvent_t ga_setup = nullptr;   // GA's Montgomery constants ready (before its chains)
  // the fixed-base tables of h1_i, h2_i (bases 2i, 2i+1 of prepare's FbJob), built
  // for exponents of up to bits_h1 / bits_h2 bits with window w
  bool fb_valid = false;
  std::vector<uint32_t> ntilde, h1, h2, T, pedmod;   // bases, and the T_m moduli rows
  uint32_t Mt = 0, fb_w = 0, bits_h1 = 0, bits_h2 = 0, bits_z = 0, fb_entries = 0;
  uint32_t* fb_table = nullptr;
  hipEvent_t fb_done = nullptr;     // every table built
};

void free_ga_pre(Ctx* c) {
  GaPre* g = reinterpret_cast<GaPre*>(c->ga_pre);
  if (g && g->done) (void)hipEventDestroy(g->done);
  if (g && g->ga_setup) (void)hipEventDestroy(g->ga_setup);
  if (g && g->fb_done) (void)hipEventDestroy(g->fb_done);
  delete g;
  c->ga_pre = nullptr;
}

// collect()'s fixed-base tables, base order [h1_i | T_m | h2_i] (FbJob::finalize
// sizes: one entry per w exponent bits, at least one)
struct FbLayout {
  std::vector<uint32_t> h, toff, mod;
  uint32_t entries = 0;
};
static FbLayout fb_layout(uint32_t n, uint32_t Mt, uint32_t w, uint32_t bits_h1, uint32_t bits_h2, uint32_t bits_z) {
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
static void ped_modulus(const fsdkr_collect_batch* b, uint32_t m, uint32_t M, uint32_t nl, uint32_t* on) {
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

// The fixed-base table chains of collect()'s FbJob, in its base order: h1_i, h2_i
// of every receiver's DLogStatement (h2: one squaring per exponent bit of s3,
// ~2816 at 2048-bit keys), then every message's ring-Pedersen T, sized by the
// bit lengths of the exponents they serve (PDL / Alice s1, s3|s2; RP Z), on the
// table chain's stream.
static int prestart_fb_tables(Ctx* c, const fsdkr_collect_batch* b, GaPre& g, uint32_t n, uint32_t P) {
  if (!b->recv_ntilde || !b->recv_h1 || !b->recv_h2 || !b->s1l || !b->s3l || !b->ped_T || !b->ped_N || !b->zl ||
      !b->m_security)
    return FSDKR_OK;   // stage 1 did not pack them: prepare builds every table
  // exponent bit bounds: exact from the packed exponents, else their slot widths
  // (a slim stage 1 leaves s1 / s3 / Z to stage 2; tables at most 31 bits longer)
  const bool exact_s = b->pdl_s1 && b->pdl_s3 && b->rp_s1 && b->rp_s2;
  const uint32_t nl = b->nl, Mt = b->n_refresh + b->n_join, M = b->m_security;
  for (uint32_t i = 0; i < n; ++i)
    if (!is_odd(b->recv_ntilde + (size_t)i * nl)) return FSDKR_OK;
  uint32_t bh1 = 1, bh2 = 1, bz = 1;
  if (exact_s) {
    for (size_t p = 0; p < P; ++p) {
      bh1 = std::max(bh1, std::max(hbn::bitlen(b->pdl_s1 + p * b->s1l, b->s1l), hbn::bitlen(b->rp_s1 + p * b->s1l, b->s1l)));
      bh2 = std::max(bh2, std::max(hbn::bitlen(b->pdl_s3 + p * b->s3l, b->s3l), hbn::bitlen(b->rp_s2 + p * b->s3l, b->s3l)));
    }
  } else {
    bh1 = 32 * b->s1l;
    bh2 = 32 * b->s3l;
  }
  if (b->ped_Z)
    for (size_t k = 0; k < (size_t)Mt * M; ++k) bz = std::max(bz, hbn::bitlen(b->ped_Z + k * b->zl, b->zl));
  else
    bz = 32 * b->zl;
  const uint32_t w = fb_window(std::max(std::max(bh1, bh2), bz));
  const FbLayout L = fb_layout(n, Mt, w, bh1, bh2, bz);
  const uint32_t nb = 2 * n + Mt, entries = L.entries, nmod = n + Mt;
  const int KD = shape_digits(nl);
  auto al = Img::al;
  const size_t o_mod = 0, o_h1 = al((size_t)nmod * nl * 4), o_h2 = o_h1 + al((size_t)n * nl * 4),
               o_T = o_h2 + al((size_t)n * nl * 4), o_bp = o_T + al((size_t)Mt * nl * 4),
               o_bl = o_bp + al((size_t)nb * 8), o_bm = o_bl + al((size_t)nb * 4), o_bt = o_bm + al((size_t)nb * 4),
               o_bh = o_bt + al((size_t)nb * 4), o_tab = o_bh + al((size_t)nb * 4);
  const size_t total = o_tab + (size_t)entries * KD * 4;
  uint8_t* dev = (uint8_t*)c->buf("collect_fb_pre", total);
  if (!dev) {
    c->fail("fsdkr_collect_prestart: device allocation of %zu bytes failed", total);
    return FSDKR_E_OOM;
  }
  std::vector<uint8_t> img(o_tab, 0);
  uint32_t* mods = reinterpret_cast<uint32_t*>(img.data() + o_mod);   // [Ntilde_i | RP modulus_m]
  memcpy(mods, b->recv_ntilde, (size_t)n * nl * 4);
  for (uint32_t m = 0; m < Mt; ++m) ped_modulus(b, m, M, nl, mods + (size_t)(n + m) * nl);
  memcpy(img.data() + o_h1, b->recv_h1, (size_t)n * nl * 4);
  memcpy(img.data() + o_h2, b->recv_h2, (size_t)n * nl * 4);
  memcpy(img.data() + o_T, b->ped_T, (size_t)Mt * nl * 4);
  auto* bp = reinterpret_cast<uint64_t*>(img.data() + o_bp);
  for (uint32_t r = 0; r < n; ++r) {   // prepare's base order [h1_i | T_m | h2_i]
    bp[r] = (uint64_t)(uintptr_t)(dev + o_h1 + (size_t)r * nl * 4);
    bp[n + Mt + r] = (uint64_t)(uintptr_t)(dev + o_h2 + (size_t)r * nl * 4);
  }
  for (uint32_t m = 0; m < Mt; ++m) bp[n + m] = (uint64_t)(uintptr_t)(dev + o_T + (size_t)m * nl * 4);
  std::vector<uint32_t> blen(nb, nl);
  memcpy(img.data() + o_bl, blen.data(), (size_t)nb * 4);
  memcpy(img.data() + o_bm, L.mod.data(), (size_t)nb * 4);
  memcpy(img.data() + o_bt, L.toff.data(), (size_t)nb * 4);
  memcpy(img.data() + o_bh, L.h.data(), (size_t)nb * 4);
  // every table chain in one launch on launch()'s table-chain stream; launch()'s
  // fixed-base exponent stream waits for it through fb_done
  hipStream_t ts = c->side_stream(8);
  StreamScope scope(c, ts);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(dev, img.data(), img.size(), hipMemcpyHostToDevice, ts), "prestart fb H2D")) ||
      (rc = c->hip_check(hipStreamSynchronize(ts), "prestart fb H2D sync")))
    return rc;
  uint32_t* cons = nullptr;
  if ((rc = setup_moduli(c, nl, reinterpret_cast<const uint32_t*>(dev + o_mod), nmod, &cons, "collect_fbpre_nl")))
    return rc;
  if (!g.fb_done && (rc = c->hip_check(hipEventCreateWithFlags(&g.fb_done, hipEventDisableTiming), "event")))
    return rc;
  g.fb_table = reinterpret_cast<uint32_t*>(dev + o_tab);
  auto U64 = [&](size_t o) { return reinterpret_cast<const uint64_t*>(dev + o); };
  auto U32 = [&](size_t o) { return reinterpret_cast<const uint32_t*>(dev + o); };
  FbTableArgs tall{U64(o_bp), U32(o_bl), U32(o_bm), U32(o_bt), U32(o_bh), cons, g.fb_table, w, nb, 3};
  if ((rc = c->hip_check(launch_fb_table(nl, tall, ts), "prestart fb_table"))) return rc;
  if ((rc = c->hip_check(hipEventRecord(g.fb_done, ts), "event record"))) return rc;
  g.ntilde.assign(b->recv_ntilde, b->recv_ntilde + (size_t)n * nl);
  g.h1.assign(b->recv_h1, b->recv_h1 + (size_t)n * nl);
  g.h2.assign(b->recv_h2, b->recv_h2 + (size_t)n * nl);
  g.T.assign(b->ped_T, b->ped_T + (size_t)Mt * nl);
  g.pedmod.assign(mods + (size_t)n * nl, mods + (size_t)nmod * nl);
  g.Mt = Mt;
  g.fb_w = w;
  g.bits_h1 = bh1;
  g.bits_h2 = bh2;
  g.bits_z = bz;
  g.fb_entries = entries;
  g.fb_valid = true;
  return FSDKR_OK;
}

// GA lanes per instance: GA shares the chip with the other streams, so it takes
// the largest group that keeps it within about half the resident lanes
// (measured at n = 64: 8 lanes 64 ms/step vs 16 lanes 70 ms); small batches
// (multi-GPU shards) get 16 or 32 lanes (KD = 160 constants) for latency.
// Used by the prestart and by launch().
static uint32_t ga_lanes(uint32_t count, uint32_t nn) {
  uint32_t g = 8;
  for (uint32_t x : {16u, kWideGroup})
    if ((uint64_t)count * x <= 65536u) g = x;
  if (g == kWideGroup && nn != 128) g = 16;
  return g;
}

// GA prestart of `count` sessions (one: fsdkr_collect_prestart; many:
// fsdkr_collect_prestart_multi), in prepare's global order: session s's
// receivers and pairs after session s-1's, every row at the widest nl.
static int prestart_ga(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count, uint32_t* n_out, uint32_t* P_out) {
  if (!c->ga_pre) c->ga_pre = new GaPre();
  GaPre& g = *reinterpret_cast<GaPre*>(c->ga_pre);
  g.valid = false;
  g.fb_valid = false;
  *n_out = *P_out = 0;
  const CollectPlan* running = reinterpret_cast<const CollectPlan*>(c->plan);
  if (running && running->launched) {
    c->fail("fsdkr_collect_prestart: a batch is in flight (call finish first)");
    return FSDKR_E_ARG;
  }
  // a prepared plan that consumed the previous prestart reads its s^N rows and
  // fixed-base tables in place: this prestart overwrites (or reallocates) those
  // buffers, so the plan is dropped (a later launch reports "no prepared batch")
  if (running && (running->ga_hit || running->fb_hit)) free_collect_plan(c);
  if (!bs || count == 0) {
    c->fail("fsdkr_collect_prestart: no batch");
    return FSDKR_E_ARG;
  }
  uint32_t nl = 0, n = 0, P = 0;
  std::vector<GaPre::Sess> ss(count);
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    if (!(b->nl == 64 || b->nl == 96) || !b->recv_n || !b->pdl_s2 || !b->rp_s) {
      c->fail("fsdkr_collect_prestart: session %u needs nl, recv_n, pdl_s2 and rp_s", k);
      return FSDKR_E_ARG;
    }
    const uint32_t R = b->n_refresh, ns = b->n_recv ? b->n_recv : R + b->n_join;
    if (R == 0 || ns < R) return FSDKR_OK;   // nothing to start (prepare reports bad shapes)
    for (uint32_t i = 0; i < ns; ++i)
      if (!is_odd(b->recv_n + (size_t)i * b->nl)) return FSDKR_OK;   // prepare reports it
    ss[k] = GaPre::Sess{b->nl, ns, R, (size_t)n, (size_t)P};
    nl = std::max(nl, b->nl);
    n += ns;
    P += R * ns;
  }
  const uint32_t nn = 2 * nl;
  // the inputs, at each session's own width, for the match in prepare
  g.recv_n.clear();
  g.s2.clear();
  g.s.clear();
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    const GaPre::Sess& x = ss[k];
    g.recv_n.insert(g.recv_n.end(), b->recv_n, b->recv_n + (size_t)x.n * x.nl);
    g.s2.insert(g.s2.end(), b->pdl_s2, b->pdl_s2 + (size_t)x.R * x.n * x.nl);
    g.s.insert(g.s.end(), b->rp_s, b->rp_s + (size_t)x.R * x.n * x.nl);
  }
  // image: [N^2 | N | s2 | s | descriptors], outputs after it
  auto al = Img::al;
  const size_t o_NN = 0, o_rn = al((size_t)n * nn * 4), o_s2 = o_rn + al((size_t)n * nl * 4),
               o_s = o_s2 + al((size_t)P * nl * 4), o_desc = o_s + al((size_t)P * nl * 4);
  const size_t desc_bytes = (size_t)2 * P * 32, o_out = o_desc + al(desc_bytes);
  const size_t total = o_out + (size_t)2 * P * nn * 4;
  uint8_t* dev = (uint8_t*)c->buf("collect_ga", total);
  if (!dev) {
    c->fail("fsdkr_collect_prestart: device allocation of %zu bytes failed", total);
    return FSDKR_E_OOM;
  }
  std::vector<uint8_t> img(o_out, 0);
  uint32_t* NN = reinterpret_cast<uint32_t*>(img.data() + o_NN);
  uint32_t* RN = reinterpret_cast<uint32_t*>(img.data() + o_rn);
  uint32_t* S2 = reinterpret_cast<uint32_t*>(img.data() + o_s2);
  uint32_t* S1 = reinterpret_cast<uint32_t*>(img.data() + o_s);
  std::vector<uint32_t> rbits(n);
  std::vector<uint32_t> sess_of_recv(n);
  for (uint32_t k = 0; k < count; ++k) std::fill(sess_of_recv.begin() + ss[k].rbase, sess_of_recv.begin() + ss[k].rbase + ss[k].n, k);
  parallel_for(n, 64, [&](size_t r0, size_t r1) {
    for (size_t r = r0; r < r1; ++r) {
      const GaPre::Sess& x = ss[sess_of_recv[r]];
      const uint32_t* Np = bs[sess_of_recv[r]].recv_n + (r - x.rbase) * x.nl;
      const hbn::Limbs N = hbn::from(Np, x.nl);
      hbn::store(hbn::mul(N, N), NN + r * nn, nn);
      memcpy(RN + r * nl, Np, (size_t)x.nl * 4);
      rbits[r] = hbn::bitlen(Np, x.nl);
    }
  });
  uint32_t recvn_max = 1;
  for (uint32_t r = 0; r < n; ++r) recvn_max = std::max(recvn_max, rbits[r]);
  for (uint32_t k = 0; k < count; ++k) {   // pair rows, zero-extended to nl
    const GaPre::Sess& x = ss[k];
    const size_t cnt = (size_t)x.R * x.n;
    if (x.nl == nl) {
      memcpy(S2 + x.pbase * nl, bs[k].pdl_s2, cnt * nl * 4);
      memcpy(S1 + x.pbase * nl, bs[k].rp_s, cnt * nl * 4);
    } else {
      for (size_t q = 0; q < cnt; ++q) {
        memcpy(S2 + (x.pbase + q) * nl, bs[k].pdl_s2 + q * x.nl, (size_t)x.nl * 4);
        memcpy(S1 + (x.pbase + q) * nl, bs[k].rp_s + q * x.nl, (size_t)x.nl * 4);
      }
    }
  }
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };
  ModexpJob J1;
  J1.k32 = nn;
  for (int which = 0; which < 2; ++which)   // the order prepare's J1 uses
    for (uint32_t k = 0; k < count; ++k) {
      const GaPre::Sess& x = ss[k];
      for (uint32_t q = 0; q < x.R * x.n; ++q) {
        const size_t p = x.pbase + q, r = x.rbase + q % x.n;
        J1.add(DI((which == 0 ? o_s2 : o_s) + p * nl * 4), nl, DI(o_rn + r * nl * 4), nl, recvn_max, (uint32_t)r);
      }
    }
  std::vector<uint8_t> desc;
  J1.pack(desc);
  memcpy(img.data() + o_desc, desc.data(), desc.size());
  hipStream_t gs = c->side_stream(0);   // GA's stream in launch()
  StreamScope scope(c, gs);
  int rc;
  if ((rc = c->hip_check(hipMemcpyAsync(dev, img.data(), img.size(), hipMemcpyHostToDevice, gs), "prestart H2D")) ||
      (rc = c->hip_check(hipStreamSynchronize(gs), "prestart H2D sync")))   // img is pageable and local
    return rc;
  // the lanes launch() would give GA: 32 lanes (KD = 160 constants) for the small
  // batches of a multi-GPU shard, where GA's chain latency is the critical path
  const uint32_t group = ga_lanes(2 * P, nn);
  uint32_t* cons = nullptr;
  if ((rc = setup_moduli(c, nn, reinterpret_cast<const uint32_t*>(dev + o_NN), n, &cons,
                         group == kWideGroup ? "collect_ga_nn_w" : "collect_ga_nn", group == kWideGroup ? kWideGroup : 0u)))
    return rc;
  g.out = reinterpret_cast<uint32_t*>(dev + o_out);
  if (!g.ga_setup && (rc = c->hip_check(hipEventCreateWithFlags(&g.ga_setup, hipEventDisableTiming), "event")))
    return rc;
  (void)hipEventRecord(g.ga_setup, gs);   // GA's constants are ready
  // issue priority 3 (2 measured 1-2 ms slower per call, profiles/r02x_ab_full.jsonl)
  if ((rc = launch_modexp_desc(c, nn, 2 * P, recvn_max, dev + o_desc, cons, g.out, gs, "mxt_GApre", 3, group)))
    return rc;
  if (!g.done && (rc = c->hip_check(hipEventCreateWithFlags(&g.done, hipEventDisableTiming), "event"))) return rc;
  if ((rc = c->hip_check(hipEventRecord(g.done, gs), "event record"))) return rc;
  g.nl = nl;
  g.n = n;
  g.R = count == 1 ? bs->n_refresh : 0;
  g.sess = std::move(ss);
  g.valid = true;
  *n_out = n;
  *P_out = P;
  return FSDKR_OK;
}

static int collect_prestart_impl(Ctx* c, const fsdkr_collect_batch* b) {
  uint32_t n = 0, P = 0;
  int rc = prestart_ga(c, b, 1, &n, &P);
  if (rc || P == 0) return rc;
  return prestart_fb_tables(c, b, *reinterpret_cast<GaPre*>(c->ga_pre), n, P);
}

// does the prestarted GA belong to these sessions (same shapes, same inputs)?
static bool ga_pre_matches(const Ctx* c, const fsdkr_collect_batch* bs, uint32_t count) {
  const GaPre* g = reinterpret_cast<const GaPre*>(c->ga_pre);
  if (!g || !g->valid || g->sess.size() != count) return false;
  uint32_t nl = 0;
  for (uint32_t k = 0; k < count; ++k) nl = std::max(nl, bs[k].nl);
  if (g->nl != nl) return false;
  size_t on = 0, op = 0;
  for (uint32_t k = 0; k < count; ++k) {
    const fsdkr_collect_batch* b = bs + k;
    const GaPre::Sess& x = g->sess[k];
    const uint32_t ns = b->n_recv ? b->n_recv : b->n_refresh + b->n_join;
    if (x.nl != b->nl || x.n != ns || x.R != b->n_refresh) return false;
    const size_t rows = (size_t)x.R * x.n * x.nl;
    if (memcmp(g->recv_n.data() + on, b->recv_n, (size_t)x.n * x.nl * 4) != 0 ||
        memcmp(g->s2.data() + op, b->pdl_s2, rows * 4) != 0 || memcmp(g->s.data() + op, b->rp_s, rows * 4) != 0)
      return false;
    on += (size_t)x.n * x.nl;
    op += rows;
  }
  return true;
}

// ------------------------------------------------------------------------------
static int collect_prepare_impl(Ctx* c, const fsdkr_collect_batch* bs, uint32_t count) {
  free_collect_plan(c);   // a failed prepare leaves no plan behind
  if (!bs || count == 0) {
    c->fail("fsdkr_collect_prepare: no batch");
    return FSDKR_E_ARG;
  }
  std::unique_ptr<CollectPlan> plan(new CollectPlan());
  CollectPlan& pl = *plan;
  PhaseClock clk;
  // ---------------- shapes
  uint32_t nl = 0, s1l = 0, s3l = 0, el = 0, zl = 0, yl = 1, ckl = 0, M = 0;
  pl.ss.resize(count);
  uint32_t n = 0, P = 0, Mt = 0, J = 0, V = 0;
  for (uint32_t s = 0; s < count; ++s) {
    const fsdkr_collect_batch* b = bs + s;
    Sess& x = pl.ss[s];
    x.b = b;
    x.R = b->n_refresh;
    x.J = b->n_join;
    x.n = b->n_recv ? b->n_recv : x.R + x.J;
    x.Mt = x.R + x.J;
    x.P = x.R * x.n;
    x.ckl = b->ckl ? b->ckl : b->nl;
    if (x.n < x.R || x.n == 0 || b->m_security == 0 || !(b->nl == 64 || b->nl == 96) || b->s1l == 0 ||
        b->s3l == 0 || b->el == 0 || b->zl == 0 || (x.J && b->yl == 0) || !shape_digits(x.ckl) || x.ckl < b->nl ||
        (M && b->m_security != M) || !b->party_index) {
      c->fail("fsdkr_collect_prepare: session %u: unsupported shape (R=%u J=%u n=%u nl=%u ckl=%u M=%u)", s, x.R, x.J,
              x.n, b->nl, x.ckl, b->m_security);
      return FSDKR_E_UNSUPPORTED;
    }
    M = b->m_security;
    // the receivers' own keys (LocalKey state, not message data) must be odd for Montgomery
    for (uint32_t i = 0; i < x.n; ++i)
      if (!is_odd(b->recv_n + (size_t)i * b->nl) || !is_odd(b->recv_ntilde + (size_t)i * b->nl)) {
        c->fail("session %u receiver %u: even Paillier or DLog modulus in the LocalKey (unsupported)", s, i);
        return FSDKR_E_UNSUPPORTED;
      }
    x.V = 0;
    for (uint32_t k = 0; k < x.R; ++k) x.V += ncoef_of(b, k);
    x.rbase = n;
    x.mbase = Mt;
    x.jbase = J;
    x.pbase = P;
    x.vbase = V;
    n += x.n;
    Mt += x.Mt;
    J += x.J;
    P += x.P;
    V += x.V;
    nl = std::max(nl, b->nl);
    s1l = std::max(s1l, b->s1l);
    s3l = std::max(s3l, b->s3l);
    el = std::max(el, b->el);
    zl = std::max(zl, b->zl);
    if (x.J) yl = std::max(yl, b->yl);
    ckl = std::max(ckl, x.ckl);
  }
  const uint32_t nn = 2 * nl;
  pl.S = count;
  pl.n = n;
  pl.P = P;
  pl.Mt = Mt;
  pl.J = J;
  pl.M = M;
  pl.nl = nl;
  pl.nn = nn;
  pl.ckl = ckl;
  pl.s1l = s1l;
  pl.el = el;
  const uint32_t MW = (M + 31) / 32;
  // global index -> session
  std::vector<uint32_t> sess_of_pair(P), sess_of_recv(n), sess_of_msg(Mt), sess_of_join(J);
  for (uint32_t s = 0; s < count; ++s) {
    const Sess& x = pl.ss[s];
    std::fill(sess_of_pair.begin() + x.pbase, sess_of_pair.begin() + x.pbase + x.P, s);
    std::fill(sess_of_recv.begin() + x.rbase, sess_of_recv.begin() + x.rbase + x.n, s);
    std::fill(sess_of_msg.begin() + x.mbase, sess_of_msg.begin() + x.mbase + x.Mt, s);
    std::fill(sess_of_join.begin() + x.jbase, sess_of_join.begin() + x.jbase + x.J, s);
  }
  std::vector<uint32_t> recv_of_pair(P);   // global receiver row of each pair
  for (uint32_t p = 0; p < P; ++p) {
    const Sess& x = pl.ss[sess_of_pair[p]];
    recv_of_pair[p] = x.rbase + (p - x.pbase) % x.n;
  }
  // a prestarted GA of this batch: J1 is not launched again
  pl.ga_hit = ga_pre_matches(c, bs, count);
  GaPre* gpre = reinterpret_cast<GaPre*>(c->ga_pre);
  if (pl.ga_hit) {
    pl.ga_done = gpre->done;
    gpre->valid = false;   // consumed (the buffer lives until the next prestart)
  }
  clk.lap("shapes");

  // ---------------- host pre-pass (O(n) + O(P) scans, no big exponentiations; threaded)
  std::vector<uint32_t> NN((size_t)n * nn), NP1((size_t)n * nn), recv_bits(n);
  parallel_for(n, 64, [&](size_t b0, size_t b1) {
    for (size_t r = b0; r < b1; ++r) {
      const Sess& x = pl.ss[sess_of_recv[r]];
      const uint32_t* Np = x.b->recv_n + (size_t)(r - x.rbase) * x.b->nl;
      hbn::Limbs N = hbn::from(Np, x.b->nl);
      hbn::store(hbn::mul(N, N), NN.data() + r * nn, nn);
      hbn::store(hbn::add_small(N, 1), NP1.data() + r * nn, nn);
      recv_bits[r] = hbn::bitlen(Np, x.b->nl);
    }
  });
  const hbn::Limbs& q3 = q_cubed();
  std::vector<uint8_t> alice_pre(P), pdl_small(P);
  std::vector<uint32_t> ae_bits(P);
  struct Maxes {
    uint32_t s1 = 1, s3 = 1, as1 = 1, as2 = 1, ae = 1;
    bool big_s1 = false;
  };
  std::vector<Maxes> tmax(host_threads() + 1);
  std::atomic<uint32_t> slot{0};
  // PDL challenges e = H(G, Q, c, z, u1, u2, u3) (zk_pdl_with_slack.rs:114-122) on the
  // host threads of this scan: J2 (c^e), J5 (z^e) and pdl_u1 can start with the pipeline
  std::vector<uint32_t>& EPDL = pl.e_pdl;
  EPDL.assign((size_t)P * 8, 0u);
  std::atomic<bool> sha_fail{false};
  parallel_for(P, 256, [&](size_t b0, size_t b1) {
    Maxes mx;
    HostSha sha;
    for (size_t p = b0; p < b1; ++p) {
      const Sess& x = pl.ss[sess_of_pair[p]];
      const fsdkr_collect_batch* b = x.b;
      const size_t lp = p - x.pbase;
      const uint32_t w = b->nl;
      sha.buf.clear();
      sha.buf.insert(sha.buf.end(), G_COMPRESSED, G_COMPRESSED + 33);
      put_point(sha.buf, b->commit + lp * 16);
      put_bigint(sha.buf, b->enc + lp * 2 * w, 2 * w);
      put_bigint(sha.buf, b->pdl_z + lp * w, w);
      put_point(sha.buf, b->pdl_u1 + lp * 16);
      put_bigint(sha.buf, b->pdl_u2 + lp * 2 * w, 2 * w);
      put_bigint(sha.buf, b->pdl_u3 + lp * w, w);
      if (!sha.digest(EPDL.data() + p * 8)) sha_fail = true;
      const uint32_t* Np = b->recv_n + (size_t)(lp % x.n) * b->nl;
      const uint32_t* s1 = b->pdl_s1 + lp * b->s1l;
      // s1 < N -> (N+1)^s1 mod N^2 = 1 + s1*N  (binomial, bit-identical)
      const bool small = hbn::cmp_raw(s1, b->s1l, Np, b->nl) < 0;
      pdl_small[p] = small ? 1 : 0;
      mx.big_s1 = mx.big_s1 || !small;
      mx.s1 = std::max(mx.s1, hbn::bitlen(s1, b->s1l));
      mx.s3 = std::max(mx.s3, hbn::bitlen(b->pdl_s3 + lp * b->s3l, b->s3l));
      const uint32_t* as1 = b->rp_s1 + lp * b->s1l;
      ae_bits[p] = hbn::bitlen(b->rp_e + lp * b->el, b->el);
      const bool s1_ok = hbn::cmp_raw(as1, b->s1l, q3.data(), q3.size()) <= 0;
      alice_pre[p] = (s1_ok && ae_bits[p] <= 256) ? 1 : 0;
      if (alice_pre[p]) {  // exponents of rejected proofs are never used
        mx.as1 = std::max(mx.as1, hbn::bitlen(as1, b->s1l));
        mx.as2 = std::max(mx.as2, hbn::bitlen(b->rp_s2 + lp * b->s3l, b->s3l));
        mx.ae = std::max(mx.ae, ae_bits[p]);
      }
    }
    tmax[slot++ % tmax.size()] = mx;   // at most host_threads() chunks
  });
  Maxes mx;
  for (const Maxes& t : tmax) {
    mx.s1 = std::max(mx.s1, t.s1);
    mx.s3 = std::max(mx.s3, t.s3);
    mx.as1 = std::max(mx.as1, t.as1);
    mx.as2 = std::max(mx.as2, t.as2);
    mx.ae = std::max(mx.ae, t.ae);
    mx.big_s1 = mx.big_s1 || t.big_s1;
  }
  clk.lap("pair scan + PDL challenges");
  if (sha_fail) {
    c->fail("fsdkr_collect_prepare: SHA-256 (OpenSSL EVP) failed");
    return FSDKR_E_ARG;
  }
  // correct-key: rho_j = mask_generation(len(n), H(n, salt, j)) mod n; primorial gcd.
  // ring-Pedersen modulus split N = 2^k m (even N: 2-adic half in pow2.hip); S mod m.
  std::vector<uint32_t> RHO((size_t)Mt * CK_M2 * ckl, 0u), CKMODS((size_t)Mt * ckl, 0u), CKEXP((size_t)Mt * ckl, 0u),
      ck_bits(Mt);
  std::vector<uint32_t> PEDN((size_t)Mt * nl, 0u), PEDS((size_t)Mt * nl, 0u), ped_tz(Mt, 0u);
  pl.ck_pre.assign(Mt, 0);
  pl.ped_mode.assign(Mt, 0);
  pl.ped_zlen.assign(Mt, M);
  pl.ck_short.assign(Mt, 0);
  pl.ck_one.assign(Mt, 0);
  for (uint32_t m = 0; m < Mt; ++m) {
    const Sess& x = pl.ss[sess_of_msg[m]];
    const uint32_t lm = m - x.mbase;
    if (x.b->ped_lens) {
      if (x.b->ped_lens[2 * lm] < M) pl.ped_mode[m] = 2;   // A[i] indexed by the hash loop (:131-133)
      pl.ped_zlen[m] = std::min(M, x.b->ped_lens[2 * lm + 1]);
    }
    if (x.b->ck_lens && x.b->ck_lens[lm] < CK_M2) pl.ck_short[m] = 1;
  }
  parallel_for(Mt, 4, [&](size_t b0, size_t b1) {
    for (size_t m = b0; m < b1; ++m) {
      const Sess& x = pl.ss[sess_of_msg[m]];
      const fsdkr_collect_batch* b = x.b;
      const size_t lm = m - x.mbase;
      const uint32_t* ckn = b->ck_n + lm * x.ckl;
      memcpy(CKEXP.data() + m * ckl, ckn, (size_t)x.ckl * 4);
      uint32_t* dst = CKMODS.data() + m * ckl;
      memcpy(dst, ckn, (size_t)x.ckl * 4);
      ck_bits[m] = hbn::bitlen(ckn, x.ckl);
      if (ck_bits[m] == 0) pl.ck_short[m] = 1;                  // rho = mask % 0: division by zero panics
      const bool one = ck_bits[m] == 1;                          // n = 1: every value is 0 mod 1 -> Ok
      const bool ok = !one && ck_bits[m] != 0 && is_odd(ckn) && !hbn::has_small_factor(ckn, x.ckl, small_primes());
      if (one) pl.ck_one[m] = 1;
      if (ok) {
        const uint32_t msklen = ck_bits[m] / 256 + 1;
        const uint32_t salt_v =
            ((uint32_t)SALT[0] << 24) | ((uint32_t)SALT[1] << 16) | ((uint32_t)SALT[2] << 8) | SALT[3];
        const hbn::Limbs Nl = hbn::from(ckn, x.ckl);
        std::vector<uint32_t> mask((size_t)msklen * 8, 0);
        for (uint32_t j = 0; j < CK_M2; ++j) {
          Sha256 h;
          h.init();
          h.bigint(ckn, x.ckl);
          absorb_u32(h, salt_v);
          absorb_u32(h, j);
          uint32_t seed[8];
          h.finish_le(seed);
          for (uint32_t k = 0; k < msklen; ++k) {
            Sha256 hk;
            hk.init();
            hk.bigint(seed, 8);
            absorb_u32(hk, k);
            hk.finish_le(mask.data() + (size_t)k * 8);
          }
          hbn::store(hbn::mod(hbn::from(mask.data(), mask.size()), Nl), RHO.data() + (m * CK_M2 + j) * ckl, ckl);
        }
      } else {   // zero / even / smooth modulus: verdict false, placeholder modulus 3 for the kernels
        std::fill(dst, dst + ckl, 0u);
        dst[0] = 3;
      }
      pl.ck_pre[m] = ok ? 1 : 0;
      // ring-Pedersen statement modulus N = 2^tz * (odd part)
      const uint32_t* N = b->ped_N + lm * b->nl;
      uint32_t* on = PEDN.data() + m * nl;
      memcpy(on, N, (size_t)b->nl * 4);
      uint32_t* sd = PEDS.data() + m * nl;
      memcpy(sd, b->ped_S + lm * b->nl, (size_t)b->nl * 4);
      if (pl.ped_mode[m] == 2 || hbn::is_zero_raw(N, b->nl)) {   // A short / modulus 0: panic before any check
        pl.ped_mode[m] = 2;
        std::fill(on, on + nl, 0u);
        on[0] = 3;
        continue;
      }
      const uint32_t tz = hbn::ctz_raw(N, b->nl);
      ped_tz[m] = tz;
      if (tz) hbn::shr_raw(on, nl, tz);
      if (on[0] == 1 && hbn::is_zero_raw(on + 1, nl - 1)) {   // odd part 1: every congruence mod 1 holds
        pl.ped_mode[m] = 1;
        on[0] = 3;
        continue;
      }
      // S reduced mod the odd part (the eq kernel compares canonical residues of
      // A*S; the reference reduces S^e mod N itself, ring_pedersen_proof.rs:147)
      if (hbn::cmp_raw(sd, nl, on, nl) >= 0) hbn::store(hbn::mod(hbn::from(sd, nl), hbn::from(on, nl)), sd, nl);
    }
  });
  clk.lap("ck rho+primes");
  // DLog statements: N > 2^128, gcd(g, N) = gcd(ni, N) = 1, x < N; challenges e = H(x, g, N, ni)
  pl.dlog_pre.assign(J, 0);
  pl.dlog_trivial.assign(J, 0);
  std::vector<uint32_t> DE((size_t)J * 2 * 8), DLOGN((size_t)J * nl, 0u), dlog_tz(J, 0u);
  parallel_for(J, 2, [&](size_t b0, size_t b1) {
    for (size_t j = b0; j < b1; ++j) {
      const Sess& x = pl.ss[sess_of_join[j]];
      const fsdkr_collect_batch* b = x.b;
      const size_t lj = j - x.jbase, w = b->nl;
      const uint32_t *N = b->dlog_N + lj * w, *g = b->dlog_g + lj * w, *ni = b->dlog_ni + lj * w;
      const uint32_t bl = hbn::bitlen(N, w);
      bool ok = bl > 129 || (bl == 129 && !(N[4] == 1 && hbn::is_zero_raw(N, 4)));
      ok = ok && hbn::gcd_is_one(g, w, N, w) && hbn::gcd_is_one(ni, w, N, w);
      uint8_t pre = 0;
      if (ok && hbn::cmp_raw(b->dlog_x1 + lj * w, w, N, w) < 0) pre |= 1;
      if (ok && hbn::cmp_raw(b->dlog_x2 + lj * w, w, N, w) < 0) pre |= 2;
      pl.dlog_pre[j] = pre;
      for (int which = 0; which < 2; ++which) {
        const uint32_t* xx = (which == 0 ? b->dlog_x1 : b->dlog_x2) + lj * w;
        const uint32_t* gg = which == 0 ? g : ni;
        const uint32_t* nn_ = which == 0 ? ni : g;
        Sha256 h;
        h.init();
        h.bigint(xx, w);
        h.bigint(gg, w);
        h.bigint(N, w);
        h.bigint(nn_, w);
        h.finish_le(DE.data() + (j * 2 + which) * 8);
      }
      uint32_t* on = DLOGN.data() + j * nl;
      memcpy(on, N, w * 4);
      if (!ok) {   // the checks fail before any exponentiation: placeholder modulus
        std::fill(on, on + nl, 0u);
        on[0] = 3;
        continue;
      }
      const uint32_t tz = hbn::ctz_raw(N, w);
      dlog_tz[j] = tz;
      if (tz) hbn::shr_raw(on, nl, tz);
      if (on[0] == 1 && hbn::is_zero_raw(on + 1, nl - 1)) {
        pl.dlog_trivial[j] = 1;
        on[0] = 3;
      }
    }
  });
  // exponent-length bounds
  uint32_t z_max = 1, y_max = 1, ckn_max = 1, recvn_max = 1;
  for (uint32_t s = 0; s < count; ++s) {
    const Sess& x = pl.ss[s];
    const fsdkr_collect_batch* b = x.b;
    for (size_t k = 0; k < (size_t)x.Mt * M; ++k) z_max = std::max(z_max, hbn::bitlen(b->ped_Z + k * b->zl, b->zl));
    for (uint32_t j = 0; j < x.J; ++j) {
      y_max = std::max(y_max, hbn::bitlen(b->dlog_y1 + (size_t)j * b->yl, b->yl));
      y_max = std::max(y_max, hbn::bitlen(b->dlog_y2 + (size_t)j * b->yl, b->yl));
    }
  }
  for (uint32_t m = 0; m < Mt; ++m)
    if (pl.ck_pre[m]) ckn_max = std::max(ckn_max, ck_bits[m]);
  for (uint32_t r = 0; r < n; ++r) recvn_max = std::max(recvn_max, recv_bits[r]);
  // Feldman share checks: per pair (commitment offset, count, index)
  std::vector<FeldmanInfo> finfo(P);
  for (uint32_t s = 0; s < count; ++s) {
    const Sess& x = pl.ss[s];
    uint32_t voff = x.vbase;
    for (uint32_t k = 0; k < x.R; ++k) {
      const uint32_t nc = ncoef_of(x.b, k);
      for (uint32_t i = 0; i < x.n; ++i) finfo[x.pbase + (size_t)k * x.n + i] = {voff, nc, i + 1, 0};
      voff += nc;
    }
  }
  clk.lap("dlog+maxes");

  // ---------------- device layout: inputs (planned; bytes written after the device allocation)
  Img I;
  using B = fsdkr_collect_batch;
  // merged field: the rows of every session at the merged width W
  auto field = [&](const uint32_t* B::*f, auto rows_of, auto width_of, uint32_t W) {
    size_t tot = 0;
    for (const Sess& x : pl.ss) tot += rows_of(x);
    const size_t o = I.reserve(tot * W * 4);
    size_t r = 0;
    for (const Sess& x : pl.ss) {
      const size_t rows = rows_of(x);
      I.rows_at(o + r * W * 4, x.b->*f, rows, width_of(x), W);
      r += rows;
    }
    return o;
  };
  auto R_recv = [](const Sess& x) { return (size_t)x.n; };
  auto R_pair = [](const Sess& x) { return (size_t)x.P; };
  auto R_join = [](const Sess& x) { return (size_t)x.J; };
  auto W_nl = [](const Sess& x) { return x.b->nl; };
  auto W_nn = [](const Sess& x) { return 2 * x.b->nl; };
  auto W_16 = [](const Sess&) { return 16u; };
  auto W_s1 = [](const Sess& x) { return x.b->s1l; };
  auto W_s3 = [](const Sess& x) { return x.b->s3l; };
  auto W_el = [](const Sess& x) { return x.b->el; };
  auto W_yl = [](const Sess& x) { return x.b->yl; };
  const size_t o_rn = field(&B::recv_n, R_recv, W_nl, nl), o_rt = field(&B::recv_ntilde, R_recv, W_nl, nl);
  const size_t o_h1 = field(&B::recv_h1, R_recv, W_nl, nl), o_h2 = field(&B::recv_h2, R_recv, W_nl, nl);
  const size_t o_NN = I.own(NN), o_NP1 = I.own(NP1);
  const size_t o_enc = field(&B::enc, R_pair, W_nn, nn), o_Q = field(&B::commit, R_pair, W_16, 16);
  const size_t o_pz = field(&B::pdl_z, R_pair, W_nl, nl), o_pu1 = field(&B::pdl_u1, R_pair, W_16, 16);
  const size_t o_pu2 = field(&B::pdl_u2, R_pair, W_nn, nn), o_pu3 = field(&B::pdl_u3, R_pair, W_nl, nl);
  const size_t o_ps1 = field(&B::pdl_s1, R_pair, W_s1, s1l), o_ps2 = field(&B::pdl_s2, R_pair, W_nl, nl);
  const size_t o_ps3 = field(&B::pdl_s3, R_pair, W_s3, s3l);
  const size_t o_az = field(&B::rp_z, R_pair, W_nl, nl), o_ae = field(&B::rp_e, R_pair, W_el, el);
  const size_t o_as = field(&B::rp_s, R_pair, W_nl, nl), o_as1 = field(&B::rp_s1, R_pair, W_s1, s1l);
  const size_t o_as2 = field(&B::rp_s2, R_pair, W_s3, s3l);
  const size_t o_vss = I.reserve((size_t)V * 64);
  for (const Sess& x : pl.ss) I.rows_at(o_vss + (size_t)x.vbase * 64, x.b->vss, x.V, 16, 16);
  const size_t o_pSraw = I.reserve((size_t)Mt * nl * 4), o_pT = I.reserve((size_t)Mt * nl * 4);
  const size_t o_pA = I.reserve((size_t)Mt * M * nl * 4), o_pZ = I.reserve((size_t)Mt * M * zl * 4);
  for (const Sess& x : pl.ss) {
    I.rows_at(o_pSraw + (size_t)x.mbase * nl * 4, x.b->ped_S, x.Mt, x.b->nl, nl);
    I.rows_at(o_pT + (size_t)x.mbase * nl * 4, x.b->ped_T, x.Mt, x.b->nl, nl);
    I.rows_at(o_pA + (size_t)x.mbase * M * nl * 4, x.b->ped_A, (size_t)x.Mt * M, x.b->nl, nl);
    I.rows_at(o_pZ + (size_t)x.mbase * M * zl * 4, x.b->ped_Z, (size_t)x.Mt * M, x.b->zl, zl);
  }
  const size_t o_pS = I.own(PEDS);
  const size_t o_cks = I.reserve((size_t)Mt * CK_M2 * ckl * 4);
  for (const Sess& x : pl.ss)
    I.rows_at(o_cks + (size_t)x.mbase * CK_M2 * ckl * 4, x.b->ck_sigma, (size_t)x.Mt * CK_M2, x.ckl, ckl);
  const size_t o_ckn = I.own(CKEXP);          // exponent: the caller's ek.n
  const size_t o_ckmods = I.own(CKMODS);      // modulus: ek.n, or placeholder 3 where the verdict is forced
  const size_t o_rho = I.own(RHO);
  size_t o_dg = 0, o_dni = 0, o_dx1 = 0, o_dx2 = 0, o_dy1 = 0, o_dy2 = 0, o_de = 0;
  if (J) {
    o_dg = field(&B::dlog_g, R_join, W_nl, nl);
    o_dni = field(&B::dlog_ni, R_join, W_nl, nl);
    o_dx1 = field(&B::dlog_x1, R_join, W_nl, nl);
    o_dx2 = field(&B::dlog_x2, R_join, W_nl, nl);
    o_dy1 = field(&B::dlog_y1, R_join, W_yl, yl);
    o_dy2 = field(&B::dlog_y2, R_join, W_yl, yl);
    o_de = I.own(DE);
  }
  std::vector<uint32_t> ONE(std::max(nn, ckl), 0);
  ONE[0] = 1;
  const size_t o_one = I.own(ONE);
  // nl-width moduli table: Ntilde_i | ring-Pedersen N (odd part) | DLog N (odd part)
  const uint32_t n_mods_nl = n + Mt + J;
  const size_t o_mods = I.reserve((size_t)n_mods_nl * nl * 4);
  for (const Sess& x : pl.ss) I.rows_at(o_mods + (size_t)x.rbase * nl * 4, x.b->recv_ntilde, x.n, x.b->nl, nl);
  {
    std::vector<uint8_t> tail(((size_t)Mt + J) * nl * 4);
    memcpy(tail.data(), PEDN.data(), (size_t)Mt * nl * 4);
    if (J) memcpy(tail.data() + (size_t)Mt * nl * 4, DLOGN.data(), (size_t)J * nl * 4);
    I.own_at(o_mods + (size_t)n * nl * 4, std::move(tail));
  }
  const size_t o_finfo = I.own(finfo);
  const size_t o_epdl = I.own(EPDL);
  clk.lap("layout plan");

  // ---------------- device layout: outputs (offsets relative to the output region)
  size_t out_bytes = 0;
  auto OUT = [&](size_t bytes) {
    const size_t o = Img::al(out_bytes);
    out_bytes = o + Img::al(bytes ? bytes : 1);
    return o;
  };
  const size_t x_pbits = OUT((size_t)Mt * MW * 4), x_ppanic = OUT((size_t)Mt * 4);
  const size_t x_Bpdl = OUT((size_t)P * nn * 4), x_gs1 = OUT((size_t)P * nn * 4);
  //   GA (nn, long)  = s2^N | s^N  [2P]  ++  (N+1)^s1 for s1 >= N  [<= P]
  //   J2 (nn, short) = c^e_pdl | c^e_A  [2P]
  //   J5 (nl, short) = z^e_pdl | zA^e_A [2P]
  //   GD (nl, long)  = g^y1 | ni^y2 [2J] ++ ni^e1 | g^e2 [2J]
  //   GC (ckl)       = sigma^n [Mt*11]
  //   FB (nl, fixed bases h1_i, h2_i, T_m) = h2^s3 | h2^s2A [2P], h1^s1 | h1^s1A [2P], T^Z [Mt*M]
  const size_t x_GA = OUT((size_t)3 * P * nn * 4 + 4);
  const size_t x_J1 = x_GA, x_J9 = x_GA + (size_t)2 * P * nn * 4;
  // J1 result row k (device address): the GA job's output, or the prestart buffer
  auto J1_at = [&](size_t k) -> uint64_t {
    return pl.ga_hit ? (uint64_t)(uintptr_t)(gpre->out + k * nn) : 0;
  };
  const size_t x_J2 = OUT((size_t)2 * P * nn * 4);
  const size_t x_J5 = OUT((size_t)2 * P * nl * 4);
  const size_t x_GD = OUT(((size_t)4 * J + 1) * nl * 4);
  const size_t x_J7 = x_GD, x_J8 = x_J7 + (size_t)2 * J * nl * 4;
  const size_t x_GC = OUT(((size_t)Mt * CK_M2 + 1) * ckl * 4);
  const size_t x_FB = OUT(((size_t)4 * P + (size_t)Mt * M + 1) * nl * 4);
  const size_t x_J4 = x_FB, x_J3 = x_J4 + (size_t)2 * P * nl * 4, x_RP = x_J3 + (size_t)2 * P * nl * 4;
  const size_t x_invc = OUT((size_t)2 * P * nn * 4), x_invz = OUT((size_t)P * nl * 4);
  const size_t x_unn = OUT((size_t)2 * P * 4);
  const size_t x_uzA = OUT((size_t)P * 4), x_uzp = OUT((size_t)P * 4);
  const size_t x_eq2 = OUT((size_t)P * 4);
  const size_t n_eqnl = (size_t)P + (size_t)Mt * M + 2 * (size_t)J;
  const size_t x_eq3 = OUT(n_eqnl * 4);               // [u3 P | RP Mt*M | DLog 2J]
  const size_t x_eqck = OUT((size_t)Mt * CK_M2 * 4);
  const size_t x_u = OUT((size_t)P * nn * 4), x_w = OUT((size_t)P * nl * 4);
  const size_t x_fel = OUT(P), x_pdlv = OUT(P), x_rng = OUT(P);
  // 2-adic checks of even moduli
  uint32_t n_p2 = 0;
  pl.ped_p2_first.assign(Mt, ~0u);
  pl.dlog_p2_first.assign(J, ~0u);
  for (uint32_t m = 0; m < Mt; ++m)
    if (ped_tz[m] && pl.ped_mode[m] != 2) {
      pl.ped_p2_first[m] = n_p2;
      n_p2 += M;
    }
  for (uint32_t j = 0; j < J; ++j)
    if (dlog_tz[j] && pl.dlog_pre[j]) {
      pl.dlog_p2_first[j] = n_p2;
      n_p2 += 2;
    }
  const size_t x_p2 = OUT((size_t)n_p2 * 4);

  // single device allocation: [inputs | descriptors | outputs]
  const size_t in_bytes_pre = Img::al(I.size);
  const size_t n_eqall = (size_t)P + n_eqnl + (size_t)Mt * CK_M2;
  const size_t desc_bound =
      ((size_t)7 * P + 4 * (size_t)J + (size_t)Mt * CK_M2) * 32 +                        // modexp jobs
      (2 * (size_t)n + Mt) * 24 + (4 * (size_t)P + (size_t)Mt * M) * 32 + 24 * 512 +      // fixed-base job
      4 * (size_t)P * 8 + 4 * (size_t)P * 16 +                                            // binom, inverses
      n_eqall * (sizeof(EqOperand) + 4) + 2 * (size_t)P * sizeof(Prod3Operand) + 4 * (size_t)P +
      2 * (size_t)P * 8 + P + (size_t)n_p2 * sizeof(Pow2Op) + 32 * 256 + 64 * 1024;
  const size_t out_off = Img::al(in_bytes_pre + desc_bound);
  const size_t total = out_off + out_bytes;
  uint8_t* dev = (uint8_t*)c->buf("collect_arena", total);
  if (!dev) {
    c->fail("fsdkr_verify_collect: device allocation of %zu bytes failed", total);
    return FSDKR_E_OOM;
  }
  uint8_t* const out_base = dev + out_off;
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };        // input address
  auto DX = [&](size_t o) { return (uint64_t)(uintptr_t)(out_base + o); };   // output address

  // ---------------- modexp jobs (descriptors addressed into the image)
  ModexpJob J1, J2, J5, J7, J8, J9, GC;
  J1.k32 = J2.k32 = J9.k32 = nn;
  J5.k32 = J7.k32 = J8.k32 = nl;
  GC.k32 = ckl;
  FbJob& FB = pl.fb;
  FB = FbJob();
  FB.k32 = nl;
  // base order [h1_i | T_m | h2_i] and instance order [h1 | T | h2]: group A (the
  // short h1 chains and the T chains) and group B (the long h2 chains) are
  // contiguous, so group A's exponents run as soon as its tables exist
  std::vector<uint32_t> fb_h1(n), fb_h2(n), fb_T(Mt);
  for (uint32_t r = 0; r < n; ++r) fb_h1[r] = FB.add_base(DI(o_h1 + (size_t)r * nl * 4), nl, r);
  for (uint32_t m = 0; m < Mt; ++m) fb_T[m] = FB.add_base(DI(o_pT + (size_t)m * nl * 4), nl, n + m);
  for (uint32_t r = 0; r < n; ++r) fb_h2[r] = FB.add_base(DI(o_h2 + (size_t)r * nl * 4), nl, r);
  struct FbAdd {
    uint32_t base;
    uint64_t exp;
    uint32_t elen, ebits;
    uint64_t out;
  };
  std::vector<FbAdd> fb_later;   // the h2 instances, added after the T instances
  fb_later.reserve(2 * (size_t)P);
  std::vector<uint32_t> j9_index(P, 0xFFFFFFFFu);
  for (int which = 0; which < 2; ++which)
    for (uint32_t p = 0; p < P; ++p) {
      const uint32_t r = recv_of_pair[p];
      const uint64_t Ni = DI(o_rn + (size_t)r * nl * 4);
      // J1: s2^N (PDL, zk_pdl_with_slack.rs:129-135) | s^N (Alice, range_proofs.rs:148)
      if (!pl.ga_hit)
        J1.add(which == 0 ? DI(o_ps2 + (size_t)p * nl * 4) : DI(o_as + (size_t)p * nl * 4), nl, Ni, nl, recvn_max, r);
      // J2: c^e (PDL :136-142 via the cross-multiplied check) | c^e (Alice :142)
      const uint64_t cp = DI(o_enc + (size_t)p * nn * 4);
      if (which == 0) J2.add(cp, nn, DI(o_epdl + (size_t)p * 32), 8, 256, r);
      else J2.add(cp, nn, DI(o_ae + (size_t)p * el * 4), el, mx.ae, r);
      // fixed bases (FB): h1^s1 -> J3 slot | h2^s3 (s2 for Alice) -> J4 slot;  J5: z^e
      const size_t slot = (size_t)which * P + p;
      if (which == 0) {
        FB.add(fb_h1[r], DI(o_ps1 + (size_t)p * s1l * 4), s1l, mx.s1, DX(x_J3 + slot * nl * 4));
        fb_later.push_back({fb_h2[r], DI(o_ps3 + (size_t)p * s3l * 4), s3l, mx.s3, DX(x_J4 + slot * nl * 4)});
        J5.add(DI(o_pz + (size_t)p * nl * 4), nl, DI(o_epdl + (size_t)p * 32), 8, 256, r);
      } else {
        const bool use = alice_pre[p];
        FB.add(fb_h1[r], DI(o_as1 + (size_t)p * s1l * 4), use ? s1l : 0, mx.as1, DX(x_J3 + slot * nl * 4));
        fb_later.push_back({fb_h2[r], DI(o_as2 + (size_t)p * s3l * 4), use ? s3l : 0, mx.as2,
                            DX(x_J4 + slot * nl * 4)});
        J5.add(DI(o_az + (size_t)p * nl * 4), nl, DI(o_ae + (size_t)p * el * 4), use ? el : 0, mx.ae, r);
      }
    }
  for (uint32_t p = 0; p < P; ++p)
    if (!pdl_small[p]) {
      const uint32_t r = recv_of_pair[p];
      j9_index[p] = (uint32_t)J9.size();
      J9.add(DI(o_NP1 + (size_t)r * nn * 4), nn, DI(o_ps1 + (size_t)p * s1l * 4), s1l, mx.s1, r);
    }
  clk.lap("desc pairs");
  {  // ring-Pedersen T^Z_k mod N (ring_pedersen_proof.rs:144): Mt*M instances, filled in parallel
    const size_t o = FB.grow((size_t)Mt * M);
    for (uint32_t m = 0; m < Mt; ++m) FB.b_bits[fb_T[m]] = std::max(FB.b_bits[fb_T[m]], std::max(z_max, 1u));
    parallel_for(Mt, 16, [&](size_t m0, size_t m1) {
      for (size_t m = m0; m < m1; ++m) {
        const uint32_t b = fb_T[m], md = FB.b_mod[b];
        for (uint32_t k = 0; k < M; ++k) {
          const size_t i = o + m * M + k, z = m * M + k;
          FB.e_ptr[i] = DI(o_pZ + z * zl * 4);
          FB.e_len[i] = zl;
          FB.e_base[i] = b;
          FB.e_mod[i] = md;
          FB.o_ptr[i] = DX(x_RP + z * nl * 4);
        }
      }
    });
  }
  clk.lap("desc rp");
  for (const FbAdd& a : fb_later) FB.add(a.base, a.exp, a.elen, a.ebits, a.out);
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < CK_M2; ++k)  // correct-key sigma_k^n mod n
      GC.add(DI(o_cks + ((size_t)m * CK_M2 + k) * ckl * 4), ckl, DI(o_ckn + (size_t)m * ckl * 4), ckl,
             pl.ck_pre[m] ? ckn_max : 0u, m);
  for (uint32_t j = 0; j < J; ++j) {
    const uint32_t mi = n + Mt + j;
    J7.add(DI(o_dg + (size_t)j * nl * 4), nl, DI(o_dy1 + (size_t)j * yl * 4), yl, y_max, mi);
    J7.add(DI(o_dni + (size_t)j * nl * 4), nl, DI(o_dy2 + (size_t)j * yl * 4), yl, y_max, mi);
    J8.add(DI(o_dni + (size_t)j * nl * 4), nl, DI(o_de + (size_t)(2 * j) * 32), 8, 256, mi);
    J8.add(DI(o_dg + (size_t)j * nl * 4), nl, DI(o_de + (size_t)(2 * j + 1) * 32), 8, 256, mi);
  }
  // descriptor image, placed right after the inputs (desc_base is 256-aligned, so
  // alignment inside `desc` carries over to device addresses)
  std::vector<uint8_t> desc;
  const size_t desc_base = in_bytes_pre;
  auto D_al = [&]() {
    desc.resize(Img::al(desc.size()), 0);
    return desc_base + desc.size();
  };
  auto pack_job = [&](const ModexpJob& j) {
    const size_t o = D_al();
    j.pack(desc);
    return o;
  };
  auto put = [&](const void* src, size_t bytes) {
    const size_t o = D_al();
    const size_t at = desc.size();
    desc.resize(at + bytes);
    if (bytes) memcpy(desc.data() + at, src, bytes);
    return o;
  };
  ModexpJob GA = J1, GD = J7;
  GA.append(J9);
  GD.append(J8);
  const size_t d_GA = pack_job(GA), d_J2 = pack_job(J2), d_J5 = pack_job(J5), d_GD = pack_job(GD),
               d_GC = pack_job(GC);
  // the h1_i / h2_i tables of a prestart: sized for the prestart's exponent bounds
  // (taller tables only add unused entries), used if the layout then agrees
  const GaPre* gp = reinterpret_cast<const GaPre*>(c->ga_pre);
  const bool fb_cand = count == 1 && gp && gp->fb_valid && gp->nl == nl && gp->n == n && gp->Mt == Mt &&
                       memcmp(gp->ntilde.data(), bs->recv_ntilde, (size_t)n * nl * 4) == 0 &&
                       memcmp(gp->h1.data(), bs->recv_h1, (size_t)n * nl * 4) == 0 &&
                       memcmp(gp->h2.data(), bs->recv_h2, (size_t)n * nl * 4) == 0 &&
                       memcmp(gp->T.data(), bs->ped_T, (size_t)Mt * nl * 4) == 0 &&
                       memcmp(gp->pedmod.data(), PEDN.data(), (size_t)Mt * nl * 4) == 0 &&
                       std::max(mx.s1, mx.as1) <= gp->bits_h1 && std::max(mx.s3, mx.as2) <= gp->bits_h2 &&
                       z_max <= gp->bits_z;
  if (fb_cand) {
    for (uint32_t r = 0; r < n; ++r) {
      FB.b_bits[fb_h1[r]] = gp->bits_h1;
      FB.b_bits[fb_h2[r]] = gp->bits_h2;
    }
    for (uint32_t m = 0; m < Mt; ++m) FB.b_bits[fb_T[m]] = gp->bits_z;
  }
  FB.finalize();
  if (fb_cand && FB.w == gp->fb_w && FB.bases() == 2 * (size_t)n + Mt) {
    const FbLayout L = fb_layout(n, Mt, FB.w, gp->bits_h1, gp->bits_h2, gp->bits_z);
    bool same = L.entries == gp->fb_entries;
    for (uint32_t k = 0; k < FB.bases() && same; ++k)
      same = FB.b_h[k] == L.h[k] && FB.b_toff[k] == L.toff[k] && FB.b_mod[k] == L.mod[k];
    if (same) {
      pl.fb_hit = true;
      pl.fb_pre.table = gp->fb_table;
      pl.fb_pre.entries = gp->fb_entries;
      pl.fb_pre.ready = gp->fb_done;
      reinterpret_cast<GaPre*>(c->ga_pre)->fb_valid = false;   // consumed
    }
  }
  clk.lap("desc fb finalize");
  FB.pack(desc);   // FbJob offsets are positions in `desc`, i.e. relative to desc_base
  // binom descriptors: PDL B = 1 + s1*N (small s1) | Alice gs1 = 1 + s1A*N
  std::vector<uint64_t> bs_ptr(2 * (size_t)P), bn_ptr(2 * (size_t)P);
  for (uint32_t p = 0; p < P; ++p) {
    bs_ptr[p] = DI(o_ps1 + (size_t)p * s1l * 4);
    bs_ptr[P + p] = DI(o_as1 + (size_t)p * s1l * 4);
    bn_ptr[p] = bn_ptr[P + p] = DI(o_rn + (size_t)recv_of_pair[p] * nl * 4);
  }
  const size_t d_bs = put(bs_ptr.data(), bs_ptr.size() * 8), d_bn = put(bn_ptr.data(), bn_ptr.size() * 8);
  // inverse descriptors: nn: c^eA (Alice; also the PDL unit test of c when eA != 0) + c^e_pdl (eA == 0)
  std::vector<uint64_t> inv_y_nn, inv_m_nn, inv_y_nl(2 * (size_t)P), inv_m_nl(2 * (size_t)P);
  std::vector<uint32_t>& cpdl_extra = pl.cpdl_extra;
  cpdl_extra.clear();
  inv_y_nn.reserve(2 * (size_t)P);
  inv_m_nn.reserve(2 * (size_t)P);
  for (uint32_t p = 0; p < P; ++p) {
    inv_y_nn.push_back(DX(x_J2 + ((size_t)P + p) * nn * 4));
    inv_m_nn.push_back(DI(o_NN + (size_t)recv_of_pair[p] * nn * 4));
  }
  for (uint32_t p = 0; p < P; ++p)
    if (ae_bits[p] == 0 || !alice_pre[p]) {  // c^eA does not witness c's unit-ness
      inv_y_nn.push_back(DX(x_J2 + (size_t)p * nn * 4));
      inv_m_nn.push_back(DI(o_NN + (size_t)recv_of_pair[p] * nn * 4));
      cpdl_extra.push_back(p);
    }
  for (uint32_t p = 0; p < P; ++p) {  // zA^eA (value) then z^e_pdl (unit test)
    const uint64_t mt = DI(o_rt + (size_t)recv_of_pair[p] * nl * 4);
    inv_y_nl[p] = DX(x_J5 + ((size_t)P + p) * nl * 4);
    inv_m_nl[p] = mt;
    inv_y_nl[P + p] = DX(x_J5 + (size_t)p * nl * 4);
    inv_m_nl[P + p] = mt;
  }
  const size_t d_iynn = put(inv_y_nn.data(), inv_y_nn.size() * 8), d_imnn = put(inv_m_nn.data(), inv_m_nn.size() * 8);
  const size_t d_iynl = put(inv_y_nl.data(), inv_y_nl.size() * 8), d_imnl = put(inv_m_nl.data(), inv_m_nl.size() * 8);
  // eq_check descriptors
  clk.lap("desc fb/binom/inv");
  std::vector<EqOperand> eq_nn(P), eq_nl, eq_ck;
  std::vector<uint32_t> eq_nn_mod(P), eq_nl_mod, eq_ck_mod;
  for (uint32_t p = 0; p < P; ++p) {  // PDL u2: (N+1)^s1 * s2^N == u2 * c^e  (mod N^2), u2 < N^2
    EqOperand& e = eq_nn[p];
    e.a = pdl_small[p] ? DX(x_Bpdl + (size_t)p * nn * 4) : DX(x_J9 + (size_t)j9_index[p] * nn * 4);
    e.b = pl.ga_hit ? J1_at(p) : DX(x_J1 + (size_t)p * nn * 4);
    e.c = DI(o_pu2 + (size_t)p * nn * 4);
    e.d = DX(x_J2 + (size_t)p * nn * 4);
    e.a_len = e.b_len = e.c_len = e.d_len = nn;
    e.sel = 0xFFFFFFFFu;
    e.flags = 1;
    eq_nn_mod[p] = recv_of_pair[p];
  }
  eq_nl.reserve(n_eqnl);
  eq_nl_mod.reserve(n_eqnl);
  for (uint32_t p = 0; p < P; ++p) {  // PDL u3: h1^s1 * h2^s3 == u3 * z^e  (mod N~), u3 < N~
    EqOperand e;
    e.a = DX(x_J3 + (size_t)p * nl * 4);
    e.b = DX(x_J4 + (size_t)p * nl * 4);
    e.c = DI(o_pu3 + (size_t)p * nl * 4);
    e.d = DX(x_J5 + (size_t)p * nl * 4);
    e.a_len = e.b_len = e.c_len = e.d_len = nl;
    e.sel = 0xFFFFFFFFu;
    e.flags = 1;
    eq_nl.push_back(e);
    eq_nl_mod.push_back(recv_of_pair[p]);
  }
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < M; ++k) {  // RP: T^Z_k == A_k * S^(e_k)  (mod N; the odd part here)
      EqOperand e;
      e.a = DX(x_RP + ((size_t)m * M + k) * nl * 4);
      e.b = DI(o_one);
      e.c = DI(o_pA + ((size_t)m * M + k) * nl * 4);
      e.d = DI(o_pS + (size_t)m * nl * 4);
      e.a_len = e.b_len = e.c_len = e.d_len = nl;
      e.sel = m * MW * 32 + k;
      e.flags = 0;
      eq_nl.push_back(e);
      eq_nl_mod.push_back(n + m);
    }
  for (uint32_t j = 0; j < J; ++j)
    for (int which = 0; which < 2; ++which) {  // DLog: g^y * ni^e == x (mod N; x < N checked on the host)
      EqOperand e;
      e.a = DX(x_J7 + ((size_t)2 * j + which) * nl * 4);
      e.b = DX(x_J8 + ((size_t)2 * j + which) * nl * 4);
      e.c = DI((which == 0 ? o_dx1 : o_dx2) + (size_t)j * nl * 4);
      e.d = DI(o_one);
      e.a_len = e.b_len = e.c_len = e.d_len = nl;
      e.sel = 0xFFFFFFFFu;
      e.flags = 0;
      eq_nl.push_back(e);
      eq_nl_mod.push_back(n + Mt + j);
    }
  for (uint32_t m = 0; m < Mt; ++m)
    for (uint32_t k = 0; k < CK_M2; ++k) {  // correct key: sigma^n == rho (mod n)
      EqOperand e;
      e.a = DX(x_GC + ((size_t)m * CK_M2 + k) * ckl * 4);
      e.b = DI(o_one);
      e.c = DI(o_rho + ((size_t)m * CK_M2 + k) * ckl * 4);
      e.d = DI(o_one);
      e.a_len = e.b_len = e.c_len = e.d_len = ckl;
      e.sel = 0xFFFFFFFFu;
      e.flags = 0;
      eq_ck.push_back(e);
      eq_ck_mod.push_back(m);
    }
  clk.lap("desc eq build");
  const size_t d_eqnn = put(eq_nn.data(), eq_nn.size() * sizeof(EqOperand)),
               d_eqnnm = put(eq_nn_mod.data(), eq_nn_mod.size() * 4);
  const size_t d_eqnl = put(eq_nl.data(), eq_nl.size() * sizeof(EqOperand)),
               d_eqnlm = put(eq_nl_mod.data(), eq_nl_mod.size() * 4);
  const size_t d_eqck = put(eq_ck.data(), eq_ck.size() * sizeof(EqOperand)),
               d_eqckm = put(eq_ck_mod.data(), eq_ck_mod.size() * 4);
  // prod3 descriptors: u = gs1 * s^N * (c^e)^-1  (mod N^2) | w = h1^s1 * h2^s2 * (z^e)^-1 (mod N~)
  std::vector<Prod3Operand> p3_nn(P), p3_nl(P);
  for (uint32_t p = 0; p < P; ++p) {
    p3_nn[p] = {DX(x_gs1 + (size_t)p * nn * 4), pl.ga_hit ? J1_at((size_t)P + p) : DX(x_J1 + ((size_t)P + p) * nn * 4),
                DX(x_invc + (size_t)p * nn * 4),
                nn, nn, nn, 0};
    p3_nl[p] = {DX(x_J3 + ((size_t)P + p) * nl * 4), DX(x_J4 + ((size_t)P + p) * nl * 4),
                DX(x_invz + (size_t)p * nl * 4), nl, nl, nl, 0};
  }
  const size_t d_p3nn = put(p3_nn.data(), p3_nn.size() * sizeof(Prod3Operand)),
               d_p3nl = put(p3_nl.data(), p3_nl.size() * sizeof(Prod3Operand)),
               d_p3m = put(recv_of_pair.data(), recv_of_pair.size() * 4);
  // alice hash descriptors + pre-verdicts
  std::vector<uint64_t> ah_n(P), ah_c(P);
  for (uint32_t p = 0; p < P; ++p) {
    ah_n[p] = DI(o_rn + (size_t)recv_of_pair[p] * nl * 4);
    ah_c[p] = DI(o_enc + (size_t)p * nn * 4);
  }
  const size_t d_ahn = put(ah_n.data(), ah_n.size() * 8), d_ahc = put(ah_c.data(), ah_c.size() * 8);
  const size_t d_alpre = put(alice_pre.data(), alice_pre.size());
  // 2-adic halves (even ring-Pedersen / DLog moduli): a^ea * b^eb == c * d^[bit] (mod 2^k)
  std::vector<Pow2Op> p2(n_p2);
  for (uint32_t m = 0; m < Mt; ++m) {
    if (pl.ped_p2_first[m] == ~0u) continue;
    for (uint32_t k = 0; k < M; ++k) {   // T^Z_k == A_k * S^e_k  (S unreduced: pow2 reduces mod 2^k)
      Pow2Op& o = p2[pl.ped_p2_first[m] + k];
      o = Pow2Op{};
      o.a = DI(o_pT + (size_t)m * nl * 4);
      o.a_len = nl;
      o.ea = DI(o_pZ + ((size_t)m * M + k) * zl * 4);
      o.ea_len = zl;
      o.c = DI(o_pA + ((size_t)m * M + k) * nl * 4);
      o.c_len = nl;
      o.d = DI(o_pSraw + (size_t)m * nl * 4);
      o.d_len = nl;
      o.sel = m * MW * 32 + k;
      o.kbits = ped_tz[m];
    }
  }
  for (uint32_t j = 0; j < J; ++j) {
    if (pl.dlog_p2_first[j] == ~0u) continue;
    for (int which = 0; which < 2; ++which) {   // g^y * ni^e == x
      Pow2Op& o = p2[pl.dlog_p2_first[j] + which];
      o = Pow2Op{};
      o.a = DI((which == 0 ? o_dg : o_dni) + (size_t)j * nl * 4);
      o.a_len = nl;
      o.ea = DI((which == 0 ? o_dy1 : o_dy2) + (size_t)j * yl * 4);
      o.ea_len = yl;
      o.b = DI((which == 0 ? o_dni : o_dg) + (size_t)j * nl * 4);
      o.b_len = nl;
      o.eb = DI(o_de + (size_t)(2 * j + which) * 32);
      o.eb_len = 8;
      o.c = DI((which == 0 ? o_dx1 : o_dx2) + (size_t)j * nl * 4);
      o.c_len = nl;
      o.sel = 0xFFFFFFFFu;
      o.kbits = dlog_tz[j];
    }
  }
  const size_t d_p2 = put(p2.data(), p2.size() * sizeof(Pow2Op));
  if (desc_base + desc.size() > out_off) {
    c->fail("internal: descriptor bound exceeded (%zu > %zu)", desc.size(), desc_bound);
    return FSDKR_E_ARG;
  }
  // fixed-base scratch (power tables, schedules, step counts): its own context buffer
  {
    const int KD = shape_digits(nl);
    const size_t tb = Img::al(FB.table_bytes(KD)), sb = Img::al(FB.sched_bytes());
    uint8_t* fbs = (uint8_t*)c->buf("collect_fb", tb + sb + FB.nsteps_bytes() + 256);
    if (!fbs) {
      c->fail("fsdkr_verify_collect: fixed-base scratch allocation failed");
      return FSDKR_E_OOM;
    }
    pl.fb_table = (uint32_t*)fbs;
    pl.fb_sched = (uint16_t*)(fbs + tb);
    pl.fb_nsteps = (uint32_t*)(fbs + tb + sb);
  }
  pl.d_FB = desc_base;
  clk.lap("descriptors");

  // ---------------- materialise the image in the pinned arena; ONE host->device copy
  const size_t up_bytes = desc_base + desc.size();
  uint8_t* host = c->host_arena(up_bytes);
  if (!host) {
    c->fail("fsdkr_verify_collect: pinned host allocation of %zu bytes failed", up_bytes);
    return FSDKR_E_OOM;
  }
  I.materialize(host);
  memcpy(host + desc_base, desc.data(), desc.size());
  clk.lap("materialize");
  int rc = c->hip_check(hipMemcpyAsync(dev, host, up_bytes, hipMemcpyHostToDevice, c->stream), "H2D batch");
  if (!rc) rc = c->hip_check(hipStreamSynchronize(c->stream), "sync H2D");
  clk.lap("H2D");
  if (rc) return rc;

  // ---------------- record the plan
  pl.out_off = out_off;
  pl.total = total;
  pl.dev = dev;
  pl.o_Q = o_Q; pl.o_enc = o_enc; pl.o_pz = o_pz; pl.o_pu1 = o_pu1; pl.o_pu2 = o_pu2; pl.o_pu3 = o_pu3;
  pl.o_ps1 = o_ps1; pl.o_pA = o_pA; pl.o_az = o_az; pl.o_ae = o_ae; pl.o_vss = o_vss; pl.o_NN = o_NN;
  pl.o_mods = o_mods; pl.o_ckmods = o_ckmods; pl.o_one = o_one;
  pl.d_finfo = o_finfo;
  pl.d_p2 = d_p2;
  pl.n_p2 = n_p2;
  pl.n_mods_nl = n_mods_nl;
  pl.o_epdl = o_epdl; pl.x_pbits = x_pbits; pl.x_ppanic = x_ppanic; pl.x_Bpdl = x_Bpdl; pl.x_gs1 = x_gs1;
  // with a prestarted J1 the GA job is J9 alone, written where J9's rows live
  const size_t xs[CollectPlan::NJOB] = {pl.ga_hit ? x_J9 : x_GA, x_GD, x_J2, x_J5, x_GC};
  const size_t ds[CollectPlan::NJOB] = {d_GA, d_GD, d_J2, d_J5, d_GC};
  const ModexpJob* js[CollectPlan::NJOB] = {&GA, &GD, &J2, &J5, &GC};
  for (int k = 0; k < CollectPlan::NJOB; ++k) {
    pl.x_J[k] = xs[k];
    pl.d_J[k] = ds[k];
    pl.jk32[k] = js[k]->k32;
    pl.jcount[k] = (uint32_t)js[k]->size();
    pl.jbits[k] = js[k]->exp_bits;
  }
  pl.x_invc = x_invc; pl.x_invz = x_invz; pl.x_unn = x_unn; pl.x_uzA = x_uzA; pl.x_uzp = x_uzp;
  pl.x_eq2 = x_eq2; pl.x_eq3 = x_eq3; pl.x_eqck = x_eqck; pl.x_u = x_u; pl.x_w = x_w; pl.x_fel = x_fel;
  pl.x_pdlv = x_pdlv; pl.x_rng = x_rng; pl.x_p2 = x_p2;
  pl.d_bs = d_bs; pl.d_bn = d_bn; pl.d_iynn = d_iynn; pl.d_imnn = d_imnn; pl.d_iynl = d_iynl; pl.d_imnl = d_imnl;
  pl.d_eqnn = d_eqnn; pl.d_eqnnm = d_eqnnm; pl.d_eqnl = d_eqnl; pl.d_eqnlm = d_eqnlm; pl.d_eqck = d_eqck;
  pl.d_eqckm = d_eqckm; pl.d_p3nn = d_p3nn; pl.d_p3nl = d_p3nl; pl.d_p3m = d_p3m; pl.d_ahn = d_ahn; pl.d_ahc = d_ahc;
  pl.d_alpre = d_alpre;
  pl.n_inv_nn = (uint32_t)inv_y_nn.size();
  pl.n_eq_nn = (uint32_t)eq_nn.size();
  pl.n_eq_nl = (uint32_t)eq_nl.size();
  pl.n_eq_ck = (uint32_t)eq_ck.size();
  for (Sess& x : pl.ss) x.b = nullptr;   // the caller's buffers are not used after prepare
  c->plan = plan.release();
  return FSDKR_OK;
}

// Enqueue the kernel pipeline on the prepared (device-resident) batch.
static int collect_launch_impl(Ctx* c) {
  CollectPlan* plan = reinterpret_cast<CollectPlan*>(c->plan);
  if (!plan) {
    c->fail("fsdkr_collect_launch: no prepared batch");
    return FSDKR_E_ARG;
  }
  CollectPlan& pl = *plan;
  if (pl.launched) {
    c->fail("fsdkr_collect_launch: the batch is already in flight (call finish first)");
    return FSDKR_E_ARG;
  }
  const uint32_t nl = pl.nl, nn = pl.nn, P = pl.P, n = pl.n, Mt = pl.Mt, M = pl.M;
  uint8_t* dev = pl.dev;
  uint8_t* const out_base = dev + pl.out_off;
  auto DI = [&](size_t o) { return (uint64_t)(uintptr_t)(dev + o); };
  auto PX = [&](size_t o) { return (uint32_t*)(out_base + o); };
  auto PI = [&](size_t o) { return (const uint32_t*)(dev + o); };
  int rc;
  hipStream_t st = c->stream;
  // the alice pre-verdicts become the initial range verdicts
  if ((rc = c->hip_check(hipMemcpyAsync(out_base + pl.x_rng, dev + pl.d_alpre, P, hipMemcpyDeviceToDevice, st), "D2D")))
    return rc;
  // moduli constants
  uint32_t *cons_nn = nullptr, *cons_nl = nullptr, *cons_ck = nullptr;
  if ((rc = setup_moduli(c, nn, PI(pl.o_NN), n, &cons_nn, "collect_nn"))) return rc;
  if ((rc = setup_moduli(c, nl, PI(pl.o_mods), pl.n_mods_nl, &cons_nl, "collect_nl"))) return rc;
  if ((rc = setup_moduli(c, pl.ckl, PI(pl.o_ckmods), Mt, &cons_ck, "collect_ck"))) return rc;
  // J2 / J5 (256-bit challenge exponents): 8 lanes per instance
  const uint32_t j2_group = 8, j5_group = 8;
  const uint32_t ga_group = ga_lanes(pl.jcount[0], nn);
  uint32_t* cons_nn_w = nullptr;
  if (ga_group == kWideGroup && pl.jcount[0] &&
      (rc = setup_moduli(c, nn, PI(pl.o_NN), n, &cons_nn_w, "collect_nn_w", kWideGroup)))
    return rc;
  // ---- stream plan (up to thirteen concurrent lanes of work: give HIP >= 12 hardware
  //      queues, GPU_MAX_HW_QUEUES, or streams share queues and serialise):
  //   side 0  : GA (nn, long exponents, priority)               | start after mod_setup
  //   side 8  : FB table chains (h1, h2, T: the longest dependent chain), top priority
  //   side 1  : FB schedules, then (after the tables) fixed-base exponents
  //   side 3  : ped_hash (serial SHA-256 chains, priority) -> 2-adic checks of even moduli
  //   side 4  : GD (DLog), GC (correct key) -> correct-key equalities
  //   side 6  : Feldman (secp256k1 Horner per pair)
  //   st      : binom x2 | fork | J5, nl inverses | join | eq, prod3, alice  (the PDL
  //             challenges come from prepare's host pass)
  //   side 2  :                    J2 (nn, 256-bit challenges) -> nn inverses
  //   side 5  :                    pdl_u1 (secp256k1)
  std::vector<hipEvent_t> done;
  // issue-priority levels of the serial chains: GA, FB tables, GD/GC, J5 (measured)
  uint32_t prio[4] = {3, 3, 2, 1};
  pl.fb.table_prio = prio[1];
  auto fork = [&](hipStream_t from, hipEvent_t* ev) -> int {
    int r = c->hip_check(hipEventCreateWithFlags(ev, hipEventDisableTiming), "event");
    if (!r) (void)hipEventRecord(*ev, from);
    return r;
  };
  auto join_later = [&](hipStream_t ss) -> int {
    hipEvent_t ev;
    int r = c->hip_check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "event");
    if (r) return r;
    (void)hipEventRecord(ev, ss);
    done.push_back(ev);
    return FSDKR_OK;
  };
  static const char* tags[CollectPlan::NJOB] = {"mxt_GA", "mxt_GD", "mxt_J2", "mxt_J5", "mxt_GC"};
  auto launch_group = [&](int k, hipStream_t ss, uint32_t pr, uint32_t group, const uint32_t* cons) -> int {
    if (!pl.jcount[k]) return FSDKR_OK;
    return launch_modexp_desc(c, pl.jk32[k], pl.jcount[k], pl.jbits[k], dev + pl.d_J[k], cons, PX(pl.x_J[k]), ss,
                              tags[k], pr, group);
  };
  // (1) chains that need only the inputs and the moduli constants start at once
  hipEvent_t consts_ready;
  if ((rc = fork(st, &consts_ready))) return rc;
  {  // GA: s2^N, s^N mod N^2 (4096-bit, 2048-bit exponents): the longest chains
    hipStream_t ss = c->side_stream(0);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    // small batches (multi-GPU shards): the h2 fixed-base table chain (2816
    // dependent squarings) is the critical path, so GA steps down one issue
    // priority level below it (8-way shard: 33.4 -> 31.7 ms, tools/ab_hwq.sh)
    if (ga_group >= 16) prio[0] = 2;
    const uint32_t* cga = (ga_group == kWideGroup) ? cons_nn_w : cons_nn;
    if ((rc = launch_group(0, ss, prio[0], ga_group, cga)) || (rc = join_later(ss))) return rc;
  }
  {  // FB: h1, h2, T fixed-base tables -> schedules -> exponents
    hipStream_t ss = c->side_stream(1);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    FbDev fd{dev + pl.d_FB, pl.fb_table, pl.fb_sched, pl.fb_nsteps};
    hipStream_t ts = c->side_stream(8);   // own stream: the chain starts beside fb_sched
    (void)hipStreamWaitEvent(ts, consts_ready, 0);
    if ((rc = fb_launch(c, pl.fb, fd, cons_nl, ss, "fb collect", ts, pl.fb_hit ? &pl.fb_pre : nullptr)) ||
        (rc = join_later(ss)))
      return rc;
  }
  {  // ring-Pedersen challenges (one serial SHA-256 chain per message), then the
     // 2-adic halves of even-modulus checks (they read the challenge bits)
    hipStream_t ss = c->side_stream(3);
    PedHashArgs h{PI(pl.o_pA), M, nl, PX(pl.x_pbits), PX(pl.x_ppanic), Mt};
    c->mark("ped_hash", true, ss);
    rc = c->hip_check(launch_ped_hash(h, ss), "ped_hash");
    c->mark("ped_hash", false, ss);
    if (rc) return rc;
    if (pl.n_p2) {
      Pow2Args a{(const Pow2Op*)(dev + pl.d_p2), PX(pl.x_pbits), PX(pl.x_p2), pl.n_p2};
      if ((rc = c->hip_check(launch_pow2_check(a, ss), "pow2_check"))) return rc;
    }
    if ((rc = join_later(ss))) return rc;
  }
  {  // Feldman share checks (inputs only; one Horner chain per pair)
    hipStream_t ss = c->side_stream(6);
    FeldmanArgs f{PI(pl.o_vss), PI(pl.o_Q), (const FeldmanInfo*)(dev + pl.d_finfo), (uint8_t*)(out_base + pl.x_fel),
                  P};
    c->mark("ec", true, ss);
    rc = c->hip_check(launch_feldman(f, ss), "feldman");
    c->mark("ec", false, ss);
    if (rc || (rc = join_later(ss))) return rc;
  }
  {  // GD: DLog g^y / ni^e (few long chains); GC: correct-key sigma^n (2048-bit
     // exponents, Mt*11 instances) on a stream of its own, so the two latency-bound
     // jobs run side by side
    hipStream_t ss = c->side_stream(4);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    if ((rc = launch_group(1, ss, prio[2], 0, cons_nl)) || (rc = join_later(ss))) return rc;
    ss = c->side_stream(9);
    (void)hipStreamWaitEvent(ss, consts_ready, 0);
    if ((rc = launch_group(4, ss, prio[2], 0, cons_ck))) return rc;
    EqCheckArgs a{(const EqOperand*)(dev + pl.d_eqck), PI(pl.d_eqckm), cons_ck, PX(pl.x_pbits), DI(pl.o_one),
                  PX(pl.x_eqck), pl.n_eq_ck};
    c->mark("eq_check", true, ss);
    rc = c->hip_check(launch_eq_check(pl.ckl, a, ss), "eq_check ck");
    c->mark("eq_check", false, ss);
    if (rc || (rc = join_later(ss))) return rc;
  }
  // (2) the jobs that exponentiate by the PDL challenges (hashed on the host by prepare)
  {
    BinomArgs a{(const uint64_t*)(dev + pl.d_bs), (const uint64_t*)(dev + pl.d_bn), pl.s1l, nl, nn, PX(pl.x_Bpdl), P};
    if ((rc = c->hip_check(launch_binom(a, st), "binom"))) return rc;
    BinomArgs a2{(const uint64_t*)(dev + pl.d_bs) + P, (const uint64_t*)(dev + pl.d_bn) + P, pl.s1l, nl, nn,
                 PX(pl.x_gs1), P};
    if ((rc = c->hip_check(launch_binom(a2, st), "binom"))) return rc;
  }
  hipEvent_t ready;
  if ((rc = fork(st, &ready))) return rc;
  {  // J2: c^e (4096-bit, 256-bit challenges) -> nn inverses
    hipStream_t ss = c->side_stream(2);
    (void)hipStreamWaitEvent(ss, ready, 0);
    if ((rc = launch_group(2, ss, 0, j2_group, cons_nn))) return rc;
    InverseArgs a{(const uint64_t*)(dev + pl.d_iynn), (const uint64_t*)(dev + pl.d_imnn), PX(pl.x_invc),
                  PX(pl.x_unn), nullptr, pl.n_inv_nn};
    c->mark("inverse", true, ss);
    rc = c->hip_check(launch_inverse(nn, a, ss), "inverse nn");
    c->mark("inverse", false, ss);
    if (rc || (rc = join_later(ss))) return rc;
  }
  {  // PDL u1 on secp256k1 (one Shamir ladder per pair, latency-bound) off the main chain
    hipStream_t ss = c->side_stream(5);
    (void)hipStreamWaitEvent(ss, ready, 0);
    PdlU1Args u{PI(pl.o_ps1), PI(pl.o_epdl), PI(pl.o_Q), PI(pl.o_pu1), pl.s1l, (uint8_t*)(out_base + pl.x_pdlv), P};
    c->mark("ec", true, ss);
    rc = c->hip_check(launch_pdl_u1(u, ss), "pdl_u1");
    c->mark("ec", false, ss);
    if (rc) return rc;
    if ((rc = join_later(ss))) return rc;
  }
  (void)hipEventDestroy(consts_ready);
  (void)hipEventDestroy(ready);
  {  // J5: z^e (2048-bit, 256-bit challenges) -> nl inverses
    hipStream_t js = st;
    if ((rc = launch_group(3, js, prio[3], j5_group, cons_nl))) return rc;
    InverseArgs b1{(const uint64_t*)(dev + pl.d_iynl), (const uint64_t*)(dev + pl.d_imnl), PX(pl.x_invz),
                   PX(pl.x_uzA), nullptr, P};
    c->mark("inverse", true, js);
    rc = c->hip_check(launch_inverse(nl, b1, js), "inverse nl");
    c->mark("inverse", false, js);
    if (rc) return rc;
    InverseArgs b2{(const uint64_t*)(dev + pl.d_iynl) + P, (const uint64_t*)(dev + pl.d_imnl) + P, nullptr,
                   PX(pl.x_uzp), nullptr, P};
    if ((rc = c->hip_check(launch_inverse(nl, b2, js), "inverse nl 2"))) return rc;
  }
  for (hipEvent_t ev : done) {
    (void)hipStreamWaitEvent(st, ev, 0);
    (void)hipEventDestroy(ev);
  }
  if (pl.ga_hit) (void)hipStreamWaitEvent(st, pl.ga_done, 0);   // the prestarted s^N rows
  // equality checks and exact products
  {
    EqCheckArgs a{(const EqOperand*)(dev + pl.d_eqnn), PI(pl.d_eqnnm), cons_nn, PX(pl.x_pbits), DI(pl.o_one),
                  PX(pl.x_eq2), pl.n_eq_nn};
    c->mark("eq_check", true);
    rc = c->hip_check(launch_eq_check(nn, a, st), "eq_check nn");
    c->mark("eq_check", false);
    if (rc) return rc;
    // eq_nl outputs: [u3 P | RP Mt*M | DLog 2J] contiguous from x_eq3
    EqCheckArgs b1{(const EqOperand*)(dev + pl.d_eqnl), PI(pl.d_eqnlm), cons_nl, PX(pl.x_pbits), DI(pl.o_one),
                   PX(pl.x_eq3), pl.n_eq_nl};
    c->mark("eq_check", true);
    rc = c->hip_check(launch_eq_check(nl, b1, st), "eq_check nl");
    c->mark("eq_check", false);
    if (rc) return rc;
    Prod3Args pa{(const Prod3Operand*)(dev + pl.d_p3nn), PI(pl.d_p3m), cons_nn, PX(pl.x_u), P};
    if ((rc = c->hip_check(launch_prod3(nn, pa, st), "prod3 nn"))) return rc;
    Prod3Args pb{(const Prod3Operand*)(dev + pl.d_p3nl), PI(pl.d_p3m), cons_nl, PX(pl.x_w), P};
    if ((rc = c->hip_check(launch_prod3(nl, pb, st), "prod3 nl"))) return rc;
  }
  {
    AliceHashArgs a{(const uint64_t*)(dev + pl.d_ahn), (const uint64_t*)(dev + pl.d_ahc), PI(pl.o_az), PX(pl.x_u),
                    PX(pl.x_w), PI(pl.o_ae), nl, nn, nl, pl.el, (uint8_t*)(out_base + pl.x_rng), P};
    c->mark("alice_hash", true);
    rc = c->hip_check(launch_alice_hash(a, st), "alice_hash");
    c->mark("alice_hash", false);
    if (rc) return rc;
  }
  pl.launched = true;
  return FSDKR_OK;
}

static bool caps_ok(const fsdkr_verdicts& v, const Sess& x) {
  return v.feldman && v.pdl && v.range && v.ped && v.ck && (x.J == 0 || v.dlog) && v.cap_pairs >= x.P &&
         v.cap_msgs >= x.Mt && v.cap_joins >= x.J;
}

// Wait for the launched pipeline, read the verdict words back, assemble per session.
static int collect_finish_impl(Ctx* c, fsdkr_verdicts* out, uint32_t count) {
  CollectPlan* plan = reinterpret_cast<CollectPlan*>(c->plan);
  if (!plan || !plan->launched) {
    c->fail("fsdkr_collect_finish: no launched batch");
    return FSDKR_E_ARG;
  }
  CollectPlan& pl = *plan;
  if (!out || count != pl.S) {
    c->fail("fsdkr_collect_finish: %u verdict blocks for %u sessions", count, pl.S);
    return FSDKR_E_ARG;
  }
  for (uint32_t s = 0; s < count; ++s)
    if (!caps_ok(out[s], pl.ss[s])) {
      c->fail("fsdkr_collect_finish: session %u: verdict arrays missing or too small", s);
      return FSDKR_E_ARG;
    }
  pl.launched = false;
  const uint32_t P = pl.P, Mt = pl.Mt, M = pl.M;
  uint8_t* const out_base = pl.dev + pl.out_off;
  hipStream_t st = c->stream;
  const std::vector<uint32_t>& e_pdl = pl.e_pdl;
  std::vector<uint32_t> ppanic(Mt), unn(pl.n_inv_nn), uzA(P), uzp(P), eq2(P), eq3(pl.n_eq_nl),
      eqck(pl.n_eq_ck), p2(pl.n_p2);
  std::vector<uint8_t> fel(P), pdlv(P), rng(P);
  int rc;
  auto D2H = [&](void* dst, size_t off, size_t bytes) {
    if (!bytes) return (int)FSDKR_OK;
    return c->hip_check(hipMemcpyAsync(dst, out_base + off, bytes, hipMemcpyDeviceToHost, st), "D2H verdicts");
  };
  if ((rc = D2H(ppanic.data(), pl.x_ppanic, Mt * 4)) ||
      (rc = D2H(unn.data(), pl.x_unn, unn.size() * 4)) || (rc = D2H(uzA.data(), pl.x_uzA, P * 4)) ||
      (rc = D2H(uzp.data(), pl.x_uzp, P * 4)) || (rc = D2H(eq2.data(), pl.x_eq2, P * 4)) ||
      (rc = D2H(eq3.data(), pl.x_eq3, eq3.size() * 4)) || (rc = D2H(eqck.data(), pl.x_eqck, eqck.size() * 4)) ||
      (rc = D2H(p2.data(), pl.x_p2, p2.size() * 4)) || (rc = D2H(fel.data(), pl.x_fel, P)) ||
      (rc = D2H(pdlv.data(), pl.x_pdlv, P)) || (rc = D2H(rng.data(), pl.x_rng, P)))
    return rc;
  if ((rc = c->sync())) return rc;
  // PDL unit test of c: c^eA witnesses it unless eA == 0 / the Alice proof was rejected early
  std::vector<uint32_t> unit_c_pdl(unn.begin(), unn.begin() + P);
  for (size_t k = 0; k < pl.cpdl_extra.size(); ++k) unit_c_pdl[pl.cpdl_extra[k]] = unn[P + k];
  for (uint32_t s = 0; s < count; ++s) {
    const Sess& x = pl.ss[s];
    fsdkr_verdicts& v = out[s];
    for (uint32_t lp = 0; lp < x.P; ++lp) {
      const uint32_t p = x.pbase + lp;
      bool ez = true;
      for (int k = 0; k < 8; ++k) ez = ez && e_pdl[(size_t)p * 8 + k] == 0;
      // reference panics (mod_inv(..).unwrap(), zk_pdl_with_slack.rs:180) when e != 0 and c or z is not a unit
      const bool panic = !ez && (!unit_c_pdl[p] || !uzp[p]);
      uint8_t bits = (uint8_t)(pdlv[p] & 1u);
      if (eq2[p]) bits |= 2;
      if (eq3[p]) bits |= 4;
      if (panic) bits |= 8;
      v.pdl[lp] = bits;
      v.feldman[lp] = fel[p];
      // Alice: pre-checks, invertibility of z^e and c^e, transcript hash (range_proofs.rs:125-163)
      v.range[lp] = (rng[p] && unn[p] && uzA[p]) ? 1 : 0;
    }
    for (uint32_t lm = 0; lm < x.Mt; ++lm) {
      const uint32_t m = x.mbase + lm;
      uint32_t* eqm = &eq3[P + (size_t)m * M];
      if (pl.ped_mode[m] == 1)
        for (uint32_t k = 0; k < M; ++k) eqm[k] = 1;   // odd part 1
      if (pl.ped_p2_first[m] != ~0u)
        for (uint32_t k = 0; k < M; ++k) eqm[k] = eqm[k] && p2[pl.ped_p2_first[m] + k];
      // panic index: challenge shorter than M bits (BitVec) or Z shorter than M, whichever first
      uint32_t pw = ppanic[m];
      if (pl.ped_zlen[m] < M) pw = pw ? std::min(pw, pl.ped_zlen[m] + 1) : pl.ped_zlen[m] + 1;
      v.ped[lm] = pl.ped_mode[m] == 2 ? 2 : ped_verdict(eqm, M, pw);   // A short / modulus 0: panic
      bool ck = pl.ck_pre[m];
      for (uint32_t k = 0; k < CK_M2; ++k) ck = ck && eqck[(size_t)m * CK_M2 + k];
      v.ck[lm] = pl.ck_short[m] ? 2 : ((ck || pl.ck_one[m]) ? 1 : 0);
    }
    for (uint32_t lj = 0; lj < x.J; ++lj) {
      const uint32_t j = x.jbase + lj;
      const size_t base = P + (size_t)Mt * M + 2 * (size_t)j;
      uint8_t d = 0;
      for (int which = 0; which < 2; ++which) {
        bool ok = (pl.dlog_pre[j] >> which) & 1u;
        ok = ok && (pl.dlog_trivial[j] || eq3[base + which]);
        if (pl.dlog_p2_first[j] != ~0u) ok = ok && p2[pl.dlog_p2_first[j] + which];
        if (ok) d |= (uint8_t)(1u << which);
      }
      v.dlog[lj] = d;
    }
  }
  return FSDKR_OK;
}

int first_error_impl(const fsdkr_collect_batch* b, const fsdkr_verdicts* v, fsdkr_error* e) {
  memset(e, 0, sizeof *e);
  const uint32_t R = b->n_refresh, J = b->n_join, n = R + J;
  // validate_collect (refresh_message.rs:147-191)
  if (R <= b->t) {
    e->variant = FSDKR_ERR_PARTIES_THRESHOLD_VIOLATION;
    e->f[0] = b->t;
    e->f[1] = R;
    return FSDKR_OK;
  }
  if (b->msg_lens) {
    const uint32_t ref = b->msg_lens[0];
    for (uint32_t k = 0; k < R; ++k) {
      const uint32_t* l = b->msg_lens + 3 * (size_t)k;
      if (!(l[0] == ref && l[1] == ref && l[2] == ref)) {
        e->variant = FSDKR_ERR_SIZE_MISMATCH;
        e->f[0] = k;
        e->f[1] = l[0];
        e->f[2] = l[1];
        e->f[3] = l[2];
        return FSDKR_OK;
      }
    }
    if (ref < n) {  // points_committed_vec[i] indexed past its end (:182); the host
                    // layer checks message 0's first `ref` shares before this panic
      e->panic = 1;
      e->variant = FSDKR_ERR_PUBLIC_SHARE_VALIDATION;
      return FSDKR_OK;
    }
  }
  if (!v) return FSDKR_E_ARG;
  if (v->cap_pairs < R * n || v->cap_msgs < R + J || (J && (!v->dlog || v->cap_joins < J))) return FSDKR_E_ARG;
  for (uint32_t k = 0; k < R; ++k)
    for (uint32_t i = 0; i < n; ++i) {
      const uint8_t f = v->feldman[(size_t)k * n + i];
      if (f & 2) {   // empty commitment vector: curv's unwrap panics
        e->panic = 1;
        e->variant = FSDKR_ERR_PUBLIC_SHARE_VALIDATION;
        return FSDKR_OK;
      }
      if (!(f & 1)) {
        e->variant = FSDKR_ERR_PUBLIC_SHARE_VALIDATION;
        return FSDKR_OK;
      }
    }
  // PDL then range, per (k, i)  (:330-350)
  for (uint32_t k = 0; k < R; ++k)
    for (uint32_t i = 0; i < n; ++i) {
      if (b->recv_avail && i >= b->recv_avail) {   // local_key.paillier_key_vec[i] out of bounds (:334)
        e->panic = 1;
        e->variant = FSDKR_ERR_PDL_W_SLACK_PROOF;
        return FSDKR_OK;
      }
      const uint8_t d = v->pdl[(size_t)k * n + i];
      if (d & 8) {
        e->panic = 1;
        e->variant = FSDKR_ERR_PDL_W_SLACK_PROOF;
        return FSDKR_OK;
      }
      if ((d & 7) != 7) {
        e->variant = FSDKR_ERR_PDL_W_SLACK_PROOF;
        e->f[0] = d & 1;
        e->f[1] = (d >> 1) & 1;
        e->f[2] = (d >> 2) & 1;
        return FSDKR_OK;
      }
      if (b->range_lens && i >= b->range_lens[k]) {   // range_proofs[i] out of bounds (:342)
        e->panic = 1;
        e->variant = FSDKR_ERR_RANGE_PROOF;
        e->f[0] = i;
        return FSDKR_OK;
      }
      if (!v->range[(size_t)k * n + i]) {
        e->variant = FSDKR_ERR_RANGE_PROOF;
        e->f[0] = i;
        return FSDKR_OK;
      }
    }
  // ring-Pedersen: refresh then join (:353-365)
  for (uint32_t m = 0; m < R + J; ++m) {
    if (v->ped[m] & 2) {
      e->panic = 1;
      e->variant = FSDKR_ERR_RING_PEDERSEN_PROOF;
      return FSDKR_OK;
    }
    if (!(v->ped[m] & 1)) {
      e->variant = FSDKR_ERR_RING_PEDERSEN_PROOF;
      return FSDKR_OK;
    }
  }
  const uint32_t ckl = b->ckl ? b->ckl : b->nl;
  // correct key + modulus size per refresh message (:375-396)
  for (uint32_t m = 0; m < R; ++m) {
    const uint32_t pi = b->party_index[m];
    if (v->ck[m] & 2) {   // sigma_vec[i] out of bounds in zk-paillier's verify
      e->panic = 1;
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    if (!(v->ck[m] & 1)) {
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    const uint32_t bits = hbn::bitlen(b->ck_n + (size_t)m * ckl, ckl);
    if (bits > b->key_bits || bits < b->key_bits - 1) {
      e->variant = FSDKR_ERR_MODULI_TOO_SMALL;
      e->f[0] = pi;
      e->f[1] = bits;
      return FSDKR_OK;
    }
    e->keys_applied = m + 1;
  }
  // joins (:398-437)
  for (uint32_t j = 0; j < J; ++j) {
    const uint32_t pi = b->party_index[R + j];
    if (pi == 0) {
      e->variant = FSDKR_ERR_NEW_PARTY_UNASSIGNED_INDEX;
      return FSDKR_OK;
    }
    if (v->ck[R + j] & 2) {
      e->panic = 1;
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    if (!(v->ck[R + j] & 1)) {
      e->variant = FSDKR_ERR_PAILLIER_VERIFICATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    if ((v->dlog[j] & 3) != 3) {
      e->variant = FSDKR_ERR_DLOG_PROOF_VALIDATION;
      e->f[0] = pi;
      return FSDKR_OK;
    }
    const uint32_t bits = hbn::bitlen(b->ck_n + (size_t)(R + j) * ckl, ckl);
    if (bits > b->key_bits || bits < b->key_bits - 1) {
      e->variant = FSDKR_ERR_MODULI_TOO_SMALL;
      e->f[0] = pi;
      e->f[1] = bits;
      return FSDKR_OK;
    }
    e->keys_applied = R + j + 1;
  }
  e->variant = FSDKR_ERR_NONE;
  return FSDKR_OK;
}

}  // namespace fsdkr

extern "C" {

int fsdkr_collect_prepare_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_prepare_impl(c, batches, count);
}

int fsdkr_collect_prepare(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch) {
  return fsdkr_collect_prepare_multi(ctx, batch, 1);
}

int fsdkr_collect_prestart(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_prestart_impl(c, batch);
}

int fsdkr_collect_prestart_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  uint32_t n = 0, P = 0;
  return fsdkr::prestart_ga(c, batches, count, &n, &P);
}

int fsdkr_collect_launch(fsdkr_ctx* ctx) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_launch_impl(c);
}

int fsdkr_collect_finish_multi(fsdkr_ctx* ctx, fsdkr_verdicts* out, uint32_t count) {
  fsdkr::Ctx* c = reinterpret_cast<fsdkr::Ctx*>(ctx);
  if (!c) return FSDKR_E_ARG;
  return fsdkr::collect_finish_impl(c, out, count);
}

int fsdkr_collect_finish(fsdkr_ctx* ctx, fsdkr_verdicts* out) { return fsdkr_collect_finish_multi(ctx, out, 1); }

int fsdkr_collect_run(fsdkr_ctx* ctx, fsdkr_verdicts* out) {
  int rc = fsdkr_collect_launch(ctx);
  return rc ? rc : fsdkr_collect_finish(ctx, out);
}

int fsdkr_verify_collect_multi(fsdkr_ctx* ctx, const fsdkr_collect_batch* batches, uint32_t count,
                               fsdkr_verdicts* out) {
  if (!ctx || !batches || !out || count == 0) return FSDKR_E_ARG;
  int rc = fsdkr_collect_prepare_multi(ctx, batches, count);
  if (!rc) rc = fsdkr_collect_launch(ctx);
  if (!rc) rc = fsdkr_collect_finish_multi(ctx, out, count);
  return rc;
}

int fsdkr_verify_collect(fsdkr_ctx* ctx, const fsdkr_collect_batch* batch, fsdkr_verdicts* out) {
  return fsdkr_verify_collect_multi(ctx, batch, 1, out);
}

int fsdkr_collect_first_error(const fsdkr_collect_batch* batch, const fsdkr_verdicts* verdicts, fsdkr_error* out) {
  if (!batch || !out) return FSDKR_E_ARG;
  return fsdkr::first_error_impl(batch, verdicts, out);
}

}  // extern "C"
