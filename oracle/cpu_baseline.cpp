// C++ restatement of RefreshMessage::collect()'s verification over GMP -- TEST
// INFRASTRUCTURE ONLY (the CPU baseline leg of bench.py and a second checker of
// the GPU verdicts).  Never linked into or called by the product.
//
// It reads the same packed batch the product's C ABI takes (struct
// fsdkr_collect_batch, include/fsdkr/fsdkr.h) and verifies every instance the
// way the reference does, with GMP -- the bignum engine curv-kzen 0.10 uses by
// default (Cargo.toml:41-44) -- loaded with dlopen("libgmp.so.10") because the
// image has the library but no headers:
//   PDLwSlackProof::verify   zk_pdl_with_slack.rs:113-188 (no binomial shortcut:
//                            mod_pow(N+1, s1, N^2) as commitment_unknown_order does)
//   AliceProof::verify       range_proofs.rs:112-164
//   RingPedersenProof::verify ring_pedersen_proof.rs:126-157
//   NiCorrectKeyProof::verify zk-paillier 0.4.4 [dep, restated]
//   CompositeDLogProof::verify zk-paillier 0.4.4 [dep, restated]
//   validate_share_public    curv feldman_vss (Horner) [dep, restated]
// secp256k1 arithmetic is plain Jacobian formulas over GMP (the reference links
// libsecp256k1, which is faster: the EC share of this baseline is pessimistic;
// it is < 5 % of a pair's time).  Instances are spread over std::threads.
#include <dlfcn.h>
#include <stdint.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "fsdkr/fsdkr.h"

namespace {

// ---------------------------------------------------------------- GMP --------
struct mpz_s {
  int alloc, size;
  void* d;
};
typedef mpz_s mpz_t[1];
typedef unsigned long ulong_t;

struct Gmp {
  void (*init)(mpz_s*);
  void (*clear)(mpz_s*);
  void (*import_)(mpz_s*, size_t, int, size_t, int, size_t, const void*);
  void* (*export_)(void*, size_t*, int, size_t, int, size_t, const mpz_s*);
  void (*powm)(mpz_s*, const mpz_s*, const mpz_s*, const mpz_s*);
  int (*invert)(mpz_s*, const mpz_s*, const mpz_s*);
  void (*mul)(mpz_s*, const mpz_s*, const mpz_s*);
  void (*mod)(mpz_s*, const mpz_s*, const mpz_s*);
  void (*add)(mpz_s*, const mpz_s*, const mpz_s*);
  void (*add_ui)(mpz_s*, const mpz_s*, ulong_t);
  void (*sub)(mpz_s*, const mpz_s*, const mpz_s*);
  int (*cmp)(const mpz_s*, const mpz_s*);
  void (*set)(mpz_s*, const mpz_s*);
  void (*set_ui)(mpz_s*, ulong_t);
  size_t (*sizeinbase)(const mpz_s*, int);
  void (*gcd)(mpz_s*, const mpz_s*, const mpz_s*);
  void (*mul_2exp)(mpz_s*, const mpz_s*, ulong_t);
  void (*mul_ui)(mpz_s*, const mpz_s*, ulong_t);
  bool ok = false;
};

Gmp G;

template <class T>
bool sym(void* h, const char* name, T& f) {
  f = reinterpret_cast<T>(dlsym(h, name));
  return f != nullptr;
}

bool load_gmp() {
  if (G.ok) return true;
  void* h = dlopen("libgmp.so.10", RTLD_NOW | RTLD_LOCAL);
  if (!h) return false;
  G.ok = sym(h, "__gmpz_init", G.init) && sym(h, "__gmpz_clear", G.clear) && sym(h, "__gmpz_import", G.import_) &&
         sym(h, "__gmpz_export", G.export_) && sym(h, "__gmpz_powm", G.powm) && sym(h, "__gmpz_invert", G.invert) &&
         sym(h, "__gmpz_mul", G.mul) && sym(h, "__gmpz_mod", G.mod) && sym(h, "__gmpz_add", G.add) &&
         sym(h, "__gmpz_add_ui", G.add_ui) && sym(h, "__gmpz_sub", G.sub) && sym(h, "__gmpz_cmp", G.cmp) &&
         sym(h, "__gmpz_set", G.set) && sym(h, "__gmpz_set_ui", G.set_ui) &&
         sym(h, "__gmpz_sizeinbase", G.sizeinbase) && sym(h, "__gmpz_gcd", G.gcd) &&
         sym(h, "__gmpz_mul_2exp", G.mul_2exp) && sym(h, "__gmpz_mul_ui", G.mul_ui);
  return G.ok;
}

// RAII big integer
struct Z {
  mpz_t v;
  Z() { G.init(v); }
  explicit Z(ulong_t x) {
    G.init(v);
    G.set_ui(v, x);
  }
  Z(const uint32_t* limbs, size_t n) {
    G.init(v);
    G.import_(v, n, -1, 4, 0, 0, limbs);
  }
  Z(const Z& o) {
    G.init(v);
    G.set(v, o.v);
  }
  Z& operator=(const Z& o) {
    G.set(v, o.v);
    return *this;
  }
  ~Z() { G.clear(v); }
  mpz_s* p() { return v; }
  const mpz_s* p() const { return v; }
  bool is_zero() const { return v->size == 0; }
  size_t bits() const { return is_zero() ? 0 : G.sizeinbase(v, 2); }
  // curv to_bytes: minimal big-endian magnitude, zero -> one 0x00 byte
  std::vector<uint8_t> bytes() const {
    if (is_zero()) return {0};
    std::vector<uint8_t> out((bits() + 7) / 8 + 1);
    size_t cnt = 0;
    G.export_(out.data(), &cnt, 1, 1, 1, 0, v);
    out.resize(cnt);
    return out;
  }
};
int cmp(const Z& a, const Z& b) { return G.cmp(a.p(), b.p()); }
Z powm(const Z& b, const Z& e, const Z& m) {
  Z r;
  G.powm(r.p(), b.p(), e.p(), m.p());
  return r;
}
Z mulm(const Z& a, const Z& b, const Z& m) {
  Z r;
  G.mul(r.p(), a.p(), b.p());
  G.mod(r.p(), r.p(), m.p());
  return r;
}
bool invert(Z& r, const Z& a, const Z& m) { return G.invert(r.p(), a.p(), m.p()) != 0; }

// ---------------------------------------------------------------- SHA-256 ----
struct Sha {
  uint32_t h[8];
  uint8_t buf[64];
  uint64_t len = 0;
  Sha() {
    const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                            0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    memcpy(h, iv, 32);
  }
  static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
        0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
        0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
        0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
        0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
        0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
        0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; ++i) w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; ++i) {
      const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
      const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
      w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
      const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
  void update(const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      buf[len % 64] = p[i];
      ++len;
      if (len % 64 == 0) block(buf);
    }
  }
  void big(const Z& z) {   // curv DigestExt::chain_bigint
    const std::vector<uint8_t> b = z.bytes();
    update(b.data(), b.size());
  }
  Z finish() {   // result_bigint: BigInt::from_bytes(digest)
    const uint64_t bits = len * 8;
    const uint8_t one = 0x80, zero = 0;
    update(&one, 1);
    while (len % 64 != 56) update(&zero, 1);
    uint8_t L[8];
    for (int i = 0; i < 8; ++i) L[i] = (uint8_t)(bits >> (56 - 8 * i));
    update(L, 8);
    uint8_t dig[32];
    for (int i = 0; i < 8; ++i)
      for (int k = 0; k < 4; ++k) dig[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
    Z r;
    G.import_(r.p(), 32, 1, 1, 1, 0, dig);
    return r;
  }
};

// ---------------------------------------------------------------- secp256k1 --
struct Curve {
  Z p, q, gx, gy;
  Curve() {
    const uint32_t P[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    const uint32_t Qo[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    const uint32_t GX[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu, 0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
    const uint32_t GY[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u, 0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};
    p = Z(P, 8);
    q = Z(Qo, 8);
    gx = Z(GX, 8);
    gy = Z(GY, 8);
  }
};
const Curve& C() {
  static Curve c;
  return c;
}

struct Pt {   // Jacobian; Z = 0 is infinity
  Z X, Y, Zc;
  bool inf() const { return Zc.is_zero(); }
};
Pt infinity() {
  Pt r;
  G.set_ui(r.X.p(), 1);
  G.set_ui(r.Y.p(), 1);
  return r;
}
Pt affine(const uint32_t* p16) {   // (0,0) = infinity
  bool zero = true;
  for (int i = 0; i < 16; ++i) zero = zero && p16[i] == 0;
  if (zero) return infinity();
  Pt r;
  r.X = Z(p16, 8);
  r.Y = Z(p16 + 8, 8);
  G.set_ui(r.Zc.p(), 1);
  return r;
}
Z fm(const Z& a, const Z& b) { return mulm(a, b, C().p); }
Z fs(const Z& a, const Z& b) {
  Z r;
  G.sub(r.p(), a.p(), b.p());
  G.mod(r.p(), r.p(), C().p.p());
  return r;
}
Z fa(const Z& a, const Z& b) {
  Z r;
  G.add(r.p(), a.p(), b.p());
  G.mod(r.p(), r.p(), C().p.p());
  return r;
}
Z fk(const Z& a, ulong_t k) {
  Z r;
  G.mul_ui(r.p(), a.p(), k);
  G.mod(r.p(), r.p(), C().p.p());
  return r;
}
Pt dbl(const Pt& a) {
  if (a.inf() || a.Y.is_zero()) return infinity();
  const Z XX = fm(a.X, a.X), YY = fm(a.Y, a.Y), YYYY = fm(YY, YY);
  const Z S = fk(fm(a.X, YY), 4), Mm = fk(XX, 3);
  Pt r;
  r.X = fs(fm(Mm, Mm), fk(S, 2));
  r.Y = fs(fm(Mm, fs(S, r.X)), fk(YYYY, 8));
  r.Zc = fk(fm(a.Y, a.Zc), 2);
  return r;
}
Pt add(const Pt& a, const Pt& b) {
  if (a.inf()) return b;
  if (b.inf()) return a;
  const Z Z1Z1 = fm(a.Zc, a.Zc), Z2Z2 = fm(b.Zc, b.Zc);
  const Z U1 = fm(a.X, Z2Z2), U2 = fm(b.X, Z1Z1);
  const Z S1 = fm(fm(a.Y, b.Zc), Z2Z2), S2 = fm(fm(b.Y, a.Zc), Z1Z1);
  if (cmp(U1, U2) == 0) return cmp(S1, S2) == 0 ? dbl(a) : infinity();
  const Z H = fs(U2, U1), Rr = fs(S2, S1);
  const Z HH = fm(H, H), HHH = fm(HH, H), V = fm(U1, HH);
  Pt r;
  r.X = fs(fs(fm(Rr, Rr), HHH), fk(V, 2));
  r.Y = fs(fm(Rr, fs(V, r.X)), fm(S1, HHH));
  r.Zc = fm(fm(a.Zc, b.Zc), H);
  return r;
}
Pt mul(const Pt& a, const Z& k) {
  Pt r = infinity();
  for (long b = (long)k.bits() - 1; b >= 0; --b) {
    r = dbl(r);
    const size_t limb = (size_t)b / 64;
    const unsigned long* d = reinterpret_cast<const unsigned long*>(k.p()->d);
    if (limb < (size_t)k.p()->size && ((d[limb] >> (b % 64)) & 1ul)) r = add(r, a);
  }
  return r;
}
bool eq_affine(const Pt& a, const uint32_t* p16) {   // a == the affine point p16
  Pt b = affine(p16);
  if (a.inf() || b.inf()) return a.inf() && b.inf();
  const Z z2 = fm(a.Zc, a.Zc), z3 = fm(z2, a.Zc);
  return cmp(a.X, fm(b.X, z2)) == 0 && cmp(a.Y, fm(b.Y, z3)) == 0;
}
// BigInt::from_bytes(P.to_bytes(true)): 33 bytes, or one 0x00 for infinity
void absorb_point(Sha& h, const uint32_t* p16) {
  bool zero = true;
  for (int i = 0; i < 16; ++i) zero = zero && p16[i] == 0;
  if (zero) {
    const uint8_t z = 0;
    h.update(&z, 1);
    return;
  }
  uint8_t b[33];
  b[0] = (uint8_t)(2 + (p16[8] & 1u));
  for (int i = 0; i < 8; ++i)
    for (int k = 0; k < 4; ++k) b[1 + 4 * i + k] = (uint8_t)(p16[7 - i] >> (24 - 8 * k));
  h.update(b, 33);
}

// ---------------------------------------------------------------- verifiers --
struct View {
  const fsdkr_collect_batch* b;
  uint32_t R, J, n, nl, nn, ckl;
  const uint32_t* row(const uint32_t* base, size_t idx, uint32_t w) const { return base + idx * w; }
};

// PDLwSlackProof::verify -> bits (u1 | u2 << 1 | u3 << 2), 8 = the reference panics
uint8_t pdl_verify(const View& v, uint32_t p) {
  const fsdkr_collect_batch* b = v.b;
  const uint32_t i = p % v.n;
  const Z N(v.row(b->recv_n, i, v.nl), v.nl), Nt(v.row(b->recv_ntilde, i, v.nl), v.nl);
  const Z h1(v.row(b->recv_h1, i, v.nl), v.nl), h2(v.row(b->recv_h2, i, v.nl), v.nl);
  Z NN;
  G.mul(NN.p(), N.p(), N.p());
  const Z c(v.row(b->enc, p, v.nn), v.nn), z(v.row(b->pdl_z, p, v.nl), v.nl);
  const Z u2(v.row(b->pdl_u2, p, v.nn), v.nn), u3(v.row(b->pdl_u3, p, v.nl), v.nl);
  const Z s1(v.row(b->pdl_s1, p, b->s1l), b->s1l), s2(v.row(b->pdl_s2, p, v.nl), v.nl);
  const Z s3(v.row(b->pdl_s3, p, b->s3l), b->s3l);
  const uint32_t* Q = b->commit + (size_t)p * 16;
  const uint32_t* u1 = b->pdl_u1 + (size_t)p * 16;
  Sha h;
  static const uint8_t GC[33] = {0x02, 0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62, 0x95, 0xCE, 0x87, 0x0B, 0x07,
                                 0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE, 0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98};
  h.update(GC, 33);
  absorb_point(h, Q);
  h.big(c);
  h.big(z);
  absorb_point(h, u1);
  h.big(u2);
  h.big(u3);
  const Z e = h.finish();
  // u1: G*(s1 mod q) + Q*((q - e) mod q)
  Z k1, k2, em;
  G.mod(k1.p(), s1.p(), C().q.p());
  G.mod(em.p(), e.p(), C().q.p());
  G.sub(k2.p(), C().q.p(), em.p());
  G.mod(k2.p(), k2.p(), C().q.p());
  Pt g;
  g.X = C().gx;
  g.Y = C().gy;
  G.set_ui(g.Zc.p(), 1);
  const Pt u1t = add(mul(g, k1), mul(affine(Q), k2));
  uint8_t bits = eq_affine(u1t, u1) ? 1 : 0;
  // u2 = commitment_unknown_order(N+1, c, N^2, s1, N) then (., c, N^2, 1, -e)
  Z N1;
  G.add_ui(N1.p(), N.p(), 1);
  const Z t2 = mulm(powm(N1, s1, NN), powm(s2, N, NN), NN);
  Z cinv;
  const bool e_nonzero = !e.is_zero();
  if (e_nonzero && !invert(cinv, c, NN)) return 8;   // mod_inv(..).unwrap() (:180)
  const Z u2t = e_nonzero ? mulm(t2, powm(cinv, e, NN), NN) : mulm(t2, Z(1), NN);
  if (cmp(u2t, u2) == 0) bits |= 2;
  const Z t3 = mulm(powm(h1, s1, Nt), powm(h2, s3, Nt), Nt);
  Z zinv;
  if (e_nonzero && !invert(zinv, z, Nt)) return 8;
  const Z u3t = e_nonzero ? mulm(t3, powm(zinv, e, Nt), Nt) : mulm(t3, Z(1), Nt);
  if (cmp(u3t, u3) == 0) bits |= 4;
  return bits;
}

// AliceProof::verify
uint8_t alice_verify(const View& v, uint32_t p) {
  const fsdkr_collect_batch* b = v.b;
  const uint32_t i = p % v.n;
  const Z N(v.row(b->recv_n, i, v.nl), v.nl), Nt(v.row(b->recv_ntilde, i, v.nl), v.nl);
  const Z h1(v.row(b->recv_h1, i, v.nl), v.nl), h2(v.row(b->recv_h2, i, v.nl), v.nl);
  Z NN;
  G.mul(NN.p(), N.p(), N.p());
  const Z c(v.row(b->enc, p, v.nn), v.nn), z(v.row(b->rp_z, p, v.nl), v.nl), e(v.row(b->rp_e, p, b->el), b->el);
  const Z s(v.row(b->rp_s, p, v.nl), v.nl), s1(v.row(b->rp_s1, p, b->s1l), b->s1l);
  const Z s2(v.row(b->rp_s2, p, b->s3l), b->s3l);
  Z q3;
  G.mul(q3.p(), C().q.p(), C().q.p());
  G.mul(q3.p(), q3.p(), C().q.p());
  if (cmp(s1, q3) > 0) return 0;
  Z zinv;
  if (!invert(zinv, powm(z, e, Nt), Nt)) return 0;
  const Z w = mulm(mulm(powm(h1, s1, Nt), powm(h2, s2, Nt), Nt), zinv, Nt);
  Z gs1;
  G.mul(gs1.p(), s1.p(), N.p());
  G.add_ui(gs1.p(), gs1.p(), 1);
  G.mod(gs1.p(), gs1.p(), NN.p());
  Z cinv;
  if (!invert(cinv, powm(c, e, NN), NN)) return 0;
  const Z u = mulm(mulm(gs1, powm(s, N, NN), NN), cinv, NN);
  Z N1;
  G.add_ui(N1.p(), N.p(), 1);
  Sha h;
  h.big(N);
  h.big(N1);
  h.big(c);
  h.big(z);
  h.big(u);
  h.big(w);
  return cmp(h.finish(), e) == 0 ? 1 : 0;
}

// RingPedersenProof::verify -> 1 ok, 0 error, 2 panic
uint8_t ped_verify(const View& v, uint32_t m) {
  const fsdkr_collect_batch* b = v.b;
  const uint32_t M = b->m_security;
  const Z S(v.row(b->ped_S, m, v.nl), v.nl), T(v.row(b->ped_T, m, v.nl), v.nl), N(v.row(b->ped_N, m, v.nl), v.nl);
  Sha h;
  std::vector<Z> A;
  A.reserve(M);
  for (uint32_t k = 0; k < M; ++k) {
    A.emplace_back(b->ped_A + ((size_t)m * M + k) * v.nl, v.nl);
    h.big(A.back());
  }
  const std::vector<uint8_t> eb = h.finish().bytes();
  if (N.is_zero()) return 2;
  for (uint32_t k = 0; k < M; ++k) {
    if (k >= 8 * eb.size()) return 2;   // BitVec index
    const bool bit = (eb[k >> 3] >> (k & 7)) & 1;
    const Z Zk(b->ped_Z + ((size_t)m * M + k) * b->zl, b->zl);
    const Z lhs = powm(T, Zk, N);
    Z Am;
    G.mod(Am.p(), A[k].p(), N.p());
    Z Se;
    G.mod(Se.p(), S.p(), N.p());
    const Z rhs = bit ? mulm(Am, Se, N) : Am;
    if (cmp(lhs, rhs) != 0) return 0;
  }
  return 1;
}

// NiCorrectKeyProof::verify (zk-paillier 0.4.4 [dep, restated])
uint8_t ck_verify(const View& v, uint32_t m) {
  const fsdkr_collect_batch* b = v.b;
  const Z n(v.row(b->ck_n, m, v.ckl), v.ckl);
  if (n.is_zero()) return 2;
  static const Z primorial = [] {
    Z p(1);
    std::vector<bool> comp(6370, false);
    for (uint32_t i = 2; i < 6370; ++i) {
      if (comp[i]) continue;
      G.mul_ui(p.p(), p.p(), i);
      for (uint32_t j = i * i; j < 6370; j += i) comp[j] = true;
    }
    return p;
  }();
  Z g;
  G.gcd(g.p(), primorial.p(), n.p());
  bool ok = cmp(g, Z(1)) == 0;
  const uint32_t key_len = (uint32_t)n.bits(), msklen = key_len / 256 + 1;
  for (uint32_t j = 0; j < 11; ++j) {
    Sha h;
    h.big(n);
    h.big(Z(0x4B5A656Eul));   // SALT_STRING "KZen"
    h.big(Z(j));
    const Z seed = h.finish();
    Z mask(0ul);
    for (uint32_t k = 0; k < msklen; ++k) {
      Sha hk;
      hk.big(seed);
      hk.big(Z(k));
      Z part = hk.finish();
      G.mul_2exp(part.p(), part.p(), 256ul * k);
      G.add(mask.p(), mask.p(), part.p());
    }
    Z rho;
    G.mod(rho.p(), mask.p(), n.p());
    const Z sig(b->ck_sigma + ((size_t)m * 11 + j) * v.ckl, v.ckl);
    ok = ok && cmp(powm(sig, n, n), rho) == 0;
  }
  return ok ? 1 : 0;
}

// CompositeDLogProof::verify x2 (zk-paillier 0.4.4 [dep, restated])
uint8_t dlog_verify(const View& v, uint32_t j) {
  const fsdkr_collect_batch* b = v.b;
  const Z N(v.row(b->dlog_N, j, v.nl), v.nl), g(v.row(b->dlog_g, j, v.nl), v.nl), ni(v.row(b->dlog_ni, j, v.nl), v.nl);
  uint8_t out = 0;
  for (int which = 0; which < 2; ++which) {
    const Z& gg = which == 0 ? g : ni;
    const Z& nn = which == 0 ? ni : g;
    const Z x(v.row(which == 0 ? b->dlog_x1 : b->dlog_x2, j, v.nl), v.nl);
    const Z y(v.row(which == 0 ? b->dlog_y1 : b->dlog_y2, j, b->yl), b->yl);
    Z two128(1);
    G.mul_2exp(two128.p(), two128.p(), 128);
    if (cmp(N, two128) <= 0) continue;
    Z d1, d2;
    G.gcd(d1.p(), gg.p(), N.p());
    G.gcd(d2.p(), nn.p(), N.p());
    if (cmp(d1, Z(1)) != 0 || cmp(d2, Z(1)) != 0) continue;
    Sha h;
    h.big(x);
    h.big(gg);
    h.big(N);
    h.big(nn);
    const Z e = h.finish();
    if (cmp(x, mulm(powm(gg, y, N), powm(nn, e, N), N)) == 0) out |= (uint8_t)(1 << which);
  }
  return out;
}

// validate_share_public: Horner over the message's commitments
uint8_t feldman_verify(const View& v, uint32_t p) {
  const fsdkr_collect_batch* b = v.b;
  const uint32_t k = p / v.n, i = p % v.n;
  size_t off = 0;
  for (uint32_t q = 0; q < k; ++q) off += b->vss_len ? b->vss_len[q] : b->t + 1;
  const uint32_t nc = b->vss_len ? b->vss_len[k] : b->t + 1;
  if (nc == 0) return 2;
  const uint32_t* A = b->vss + off * 16;
  Pt acc = affine(A + (size_t)(nc - 1) * 16);
  const Z idx((ulong_t)(i + 1));
  for (int j = (int)nc - 2; j >= 0; --j) acc = add(mul(acc, idx), affine(A + (size_t)j * 16));
  return eq_affine(acc, b->commit + (size_t)p * 16) ? 1 : 0;
}

template <class F>
double run_threads(uint32_t count, uint32_t threads, F&& f) {
  const auto t0 = std::chrono::steady_clock::now();
  std::atomic<uint32_t> next{0};
  auto work = [&] {
    for (;;) {
      const uint32_t k = next++;
      if (k >= count) return;
      f(k);
    }
  };
  std::vector<std::thread> th;
  for (uint32_t t = 1; t < threads; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

extern "C" {

int cpubase_available(void) { return load_gmp() ? 1 : 0; }

// Verify pairs [0, n_pairs), ring-Pedersen + correct-key proofs [0, n_msgs),
// DLog proofs [0, n_joins), Feldman checks [0, n_fel) of the batch on `threads`
// threads.  Outputs as struct fsdkr_verdicts (pdl bits, range, ped, ck, dlog,
// feldman); secs[5] = wall seconds of the pairs, ped, ck, dlog, feldman phases.
int cpubase_verify(const fsdkr_collect_batch* b, uint32_t n_pairs, uint32_t n_msgs, uint32_t n_joins,
                   uint32_t n_fel, uint32_t threads, uint8_t* pdl, uint8_t* range, uint8_t* ped, uint8_t* ck,
                   uint8_t* dlog, uint8_t* fel, double* secs) {
  if (!load_gmp() || !b) return -1;
  (void)C();
  View v;
  v.b = b;
  v.R = b->n_refresh;
  v.J = b->n_join;
  v.n = b->n_recv ? b->n_recv : v.R + v.J;
  v.nl = b->nl;
  v.nn = 2 * b->nl;
  v.ckl = b->ckl ? b->ckl : b->nl;
  if (threads == 0) threads = 1;
  secs[0] = run_threads(n_pairs, threads, [&](uint32_t p) {
    pdl[p] = pdl_verify(v, p);
    range[p] = alice_verify(v, p);
  });
  secs[1] = run_threads(n_msgs, threads, [&](uint32_t m) { ped[m] = ped_verify(v, m); });
  secs[2] = run_threads(n_msgs, threads, [&](uint32_t m) { ck[m] = ck_verify(v, m); });
  secs[3] = run_threads(n_joins, threads, [&](uint32_t j) { dlog[j] = dlog_verify(v, j); });
  secs[4] = run_threads(n_fel, threads, [&](uint32_t p) { fel[p] = feldman_verify(v, p); });
  return 0;
}

}  // extern "C"
