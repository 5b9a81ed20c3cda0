// secp256k1 field / group arithmetic, one point operation per lane (gfx950).
//
// Replaces libsecp256k1 behind curv Point<Secp256k1> on the collect() path:
//   PDL u1 check  G*s1 + Q*(q-e) == u1      (zk_pdl_with_slack.rs:124-127,158)
//   Feldman check S_i == sum_k A_k (i+1)^k  (refresh_message.rs:177-188 via
//                 curv VerifiableSS::validate_share_public, Horner form)
//   pk_vec / y    sum_j P_j * lambda_j, G*x (refresh_message.rs:451-464)
// Field elements: 8 little-endian u32 limbs, fully reduced mod p.
// Points: Jacobian (X, Y, Z), Z == 0 is the point at infinity.  Affine inputs
// use (0, 0) for infinity ((0,0) is not on the curve).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fsdkr {
namespace ec {

#define EC_D __device__ __forceinline__

struct Fe {
  uint32_t v[8];
};

// p = 2^256 - 2^32 - 977
__constant__ const uint32_t P_LIMBS[8] = {0xFFFFFC2Fu, 0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                          0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
// q = group order
__constant__ const uint32_t Q_LIMBS[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                                          0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
__constant__ const uint32_t GX_LIMBS[8] = {0x16F81798u, 0x59F2815Bu, 0x2DCE28D9u, 0x029BFCDBu,
                                           0xCE870B07u, 0x55A06295u, 0xF9DCBBACu, 0x79BE667Eu};
__constant__ const uint32_t GY_LIMBS[8] = {0xFB10D4B8u, 0x9C47D08Fu, 0xA6855419u, 0xFD17B448u,
                                           0x0E1108A8u, 0x5DA4FBFCu, 0x26A3C465u, 0x483ADA77u};

EC_D bool fe_is_zero(const Fe& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i];
  return o == 0;
}
EC_D bool fe_eq(const Fe& a, const Fe& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.v[i] ^ b.v[i];
  return o == 0;
}
// a >= p ?
EC_D bool fe_ge_p(const Fe& a) {
  // p has limbs 1..7 = ff..fe/ff; a >= p  <=>  a[2..7] all ones and (a[1] > fffffffe or (== and a[0] >= fffffc2f))
  uint32_t hi = 0xFFFFFFFFu;
#pragma unroll
  for (int i = 2; i < 8; ++i) hi &= a.v[i];
  if (hi != 0xFFFFFFFFu) return false;
  if (a.v[1] != 0xFFFFFFFEu) return a.v[1] == 0xFFFFFFFFu;
  return a.v[0] >= 0xFFFFFC2Fu;
}
// a - p (only valid when a >= p) == a + 2^32 + 977 mod 2^256
EC_D void fe_sub_p(Fe& a) {
  uint64_t c = (uint64_t)a.v[0] + 977u;
  a.v[0] = (uint32_t)c;
  c = (c >> 32) + (uint64_t)a.v[1] + 1u;
  a.v[1] = (uint32_t)c;
  c >>= 32;
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    c += a.v[i];
    a.v[i] = (uint32_t)c;
    c >>= 32;
  }
}

EC_D void fe_add(Fe& r, const Fe& a, const Fe& b) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.v[i] + b.v[i];
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
  // overflow (2^256) == 2^32 + 977 mod p
  if (c) {
    uint64_t d = (uint64_t)r.v[0] + 977u;
    r.v[0] = (uint32_t)d;
    d = (d >> 32) + (uint64_t)r.v[1] + 1u;
    r.v[1] = (uint32_t)d;
    d >>= 32;
#pragma unroll
    for (int i = 2; i < 8; ++i) {
      d += r.v[i];
      r.v[i] = (uint32_t)d;
      d >>= 32;
    }
  }
  if (fe_ge_p(r)) fe_sub_p(r);
}

EC_D void fe_sub(Fe& r, const Fe& a, const Fe& b) {
  int64_t br = 0;
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    int64_t d = (int64_t)a.v[i] - b.v[i] + br;
    t[i] = (uint32_t)d;
    br = d >> 32;
  }
  if (br) {  // add p back
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      c += (uint64_t)t[i] + P_LIMBS[i];
      t[i] = (uint32_t)c;
      c >>= 32;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = t[i];
}

// r = a*b mod p
EC_D void fe_mul(Fe& r, const Fe& a, const Fe& b) {
  uint32_t t[16];
  // product scanning with a 96-bit column accumulator
  uint64_t acc = 0;
  uint32_t acc_hi = 0;
#pragma unroll
  for (int col = 0; col < 15; ++col) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = col - i;
      if (j < 0 || j > 7) continue;
      const uint64_t p = (uint64_t)a.v[i] * b.v[j];
      const uint64_t s = acc + p;
      acc_hi += (s < acc);
      acc = s;
    }
    t[col] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)acc_hi << 32);
    acc_hi = 0;
  }
  t[15] = (uint32_t)acc;
  // fold: T = L + H*2^256 ; 2^256 == 2^32 + 977 (mod p)
  uint32_t u[10];
  uint64_t c = 0;
  // u = L + H*977 + (H << 32)
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint64_t s = c;
    if (i < 8) s += t[i];
    if (i < 8) s += (uint64_t)t[8 + i] * 977u;
    if (i >= 1 && i <= 8) s += t[8 + i - 1];
    u[i] = (uint32_t)s;
    c = s >> 32;
  }
  // second fold of u[8..9] (< 2^34)
  const uint64_t h = ((uint64_t)u[9] << 32) | u[8];
  uint64_t s0 = (uint64_t)u[0] + (h & 0xFFFFFFFFu) * 977u;
  r.v[0] = (uint32_t)s0;
  uint64_t s1 = (s0 >> 32) + (uint64_t)u[1] + (h >> 32) * 977u + (h & 0xFFFFFFFFu);
  r.v[1] = (uint32_t)s1;
  uint64_t s2 = (s1 >> 32) + (uint64_t)u[2] + (h >> 32);
  r.v[2] = (uint32_t)s2;
  uint64_t cc = s2 >> 32;
#pragma unroll
  for (int i = 3; i < 8; ++i) {
    cc += u[i];
    r.v[i] = (uint32_t)cc;
    cc >>= 32;
  }
  if (cc) {  // one more 2^256 wrap (rare)
    uint64_t d = (uint64_t)r.v[0] + 977u;
    r.v[0] = (uint32_t)d;
    d = (d >> 32) + (uint64_t)r.v[1] + 1u;
    r.v[1] = (uint32_t)d;
    d >>= 32;
#pragma unroll
    for (int i = 2; i < 8; ++i) {
      d += r.v[i];
      r.v[i] = (uint32_t)d;
      d >>= 32;
    }
  }
  if (fe_ge_p(r)) fe_sub_p(r);
}

EC_D void fe_sqr(Fe& r, const Fe& a) { fe_mul(r, a, a); }

EC_D void fe_load(Fe& r, const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = p[i];
}
EC_D void fe_set_u32(Fe& r, uint32_t x) {
  r.v[0] = x;
#pragma unroll
  for (int i = 1; i < 8; ++i) r.v[i] = 0;
}

// a^(p-2)
EC_D void fe_inv(Fe& r, const Fe& a) {
  // p-2 = ff..fe ffffffff fffffc2d : plain left-to-right square and multiply
  Fe x;
  fe_set_u32(x, 1);
  for (int i = 7; i >= 0; --i) {
    uint32_t e = (i == 0) ? 0xFFFFFC2Du : (i == 1 ? 0xFFFFFFFEu : 0xFFFFFFFFu);
    for (int b = 31; b >= 0; --b) {
      fe_sqr(x, x);
      if ((e >> b) & 1u) fe_mul(x, x, a);
    }
  }
  r = x;
}

struct Jac {
  Fe X, Y, Z;
};

EC_D void jac_set_inf(Jac& p) {
  fe_set_u32(p.X, 1);
  fe_set_u32(p.Y, 1);
  fe_set_u32(p.Z, 0);
}
EC_D bool jac_is_inf(const Jac& p) { return fe_is_zero(p.Z); }

// affine loader: (0,0) = infinity
EC_D bool aff_load(Fe& x, Fe& y, const uint32_t* p16) {
  fe_load(x, p16);
  fe_load(y, p16 + 8);
  return fe_is_zero(x) && fe_is_zero(y);
}

EC_D void jac_dbl(Jac& r, const Jac& p) {
  if (jac_is_inf(p) || fe_is_zero(p.Y)) {
    jac_set_inf(r);
    return;
  }
  Fe A, B, C, D, E, F, t;
  fe_sqr(A, p.X);
  fe_sqr(B, p.Y);
  fe_sqr(C, B);
  fe_add(t, p.X, B);
  fe_sqr(t, t);
  fe_sub(t, t, A);
  fe_sub(t, t, C);
  fe_add(D, t, t);
  fe_add(E, A, A);
  fe_add(E, E, A);
  fe_sqr(F, E);
  Fe X3, Y3, Z3;
  fe_add(t, D, D);
  fe_sub(X3, F, t);
  fe_sub(t, D, X3);
  fe_mul(Y3, E, t);
  fe_add(C, C, C);
  fe_add(C, C, C);
  fe_add(C, C, C);
  fe_sub(Y3, Y3, C);
  fe_mul(Z3, p.Y, p.Z);
  fe_add(Z3, Z3, Z3);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// r = p + (x2, y2) affine (not infinity)
EC_D void jac_add_aff(Jac& r, const Jac& p, const Fe& x2, const Fe& y2) {
  if (jac_is_inf(p)) {
    r.X = x2;
    r.Y = y2;
    fe_set_u32(r.Z, 1);
    return;
  }
  Fe Z1Z1, U2, S2, H, Rr, t;
  fe_sqr(Z1Z1, p.Z);
  fe_mul(U2, x2, Z1Z1);
  fe_mul(t, p.Z, Z1Z1);
  fe_mul(S2, y2, t);
  fe_sub(H, U2, p.X);
  fe_sub(Rr, S2, p.Y);
  if (fe_is_zero(H)) {
    if (fe_is_zero(Rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  Fe HH, HHH, V, X3, Y3, Z3;
  fe_sqr(HH, H);
  fe_mul(HHH, H, HH);
  fe_mul(V, p.X, HH);
  fe_sqr(X3, Rr);
  fe_sub(X3, X3, HHH);
  fe_sub(X3, X3, V);
  fe_sub(X3, X3, V);
  fe_sub(t, V, X3);
  fe_mul(Y3, Rr, t);
  fe_mul(t, p.Y, HHH);
  fe_sub(Y3, Y3, t);
  fe_mul(Z3, p.Z, H);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// general Jacobian addition
EC_D void jac_add(Jac& r, const Jac& p, const Jac& q) {
  if (jac_is_inf(p)) {
    r = q;
    return;
  }
  if (jac_is_inf(q)) {
    r = p;
    return;
  }
  Fe Z1Z1, Z2Z2, U1, U2, S1, S2, H, Rr, t;
  fe_sqr(Z1Z1, p.Z);
  fe_sqr(Z2Z2, q.Z);
  fe_mul(U1, p.X, Z2Z2);
  fe_mul(U2, q.X, Z1Z1);
  fe_mul(t, q.Z, Z2Z2);
  fe_mul(S1, p.Y, t);
  fe_mul(t, p.Z, Z1Z1);
  fe_mul(S2, q.Y, t);
  fe_sub(H, U2, U1);
  fe_sub(Rr, S2, S1);
  if (fe_is_zero(H)) {
    if (fe_is_zero(Rr)) {
      jac_dbl(r, p);
    } else {
      jac_set_inf(r);
    }
    return;
  }
  Fe HH, HHH, V, X3, Y3, Z3;
  fe_sqr(HH, H);
  fe_mul(HHH, H, HH);
  fe_mul(V, U1, HH);
  fe_sqr(X3, Rr);
  fe_sub(X3, X3, HHH);
  fe_sub(X3, X3, V);
  fe_sub(X3, X3, V);
  fe_sub(t, V, X3);
  fe_mul(Y3, Rr, t);
  fe_mul(t, S1, HHH);
  fe_sub(Y3, Y3, t);
  fe_mul(t, p.Z, q.Z);
  fe_mul(Z3, t, H);
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// Jacobian point == affine point (inf encoded by aff_inf)
EC_D bool jac_eq_aff(const Jac& p, const Fe& x, const Fe& y, bool aff_inf) {
  if (jac_is_inf(p)) return aff_inf;
  if (aff_inf) return false;
  Fe Z2, Z3, t;
  fe_sqr(Z2, p.Z);
  fe_mul(t, x, Z2);
  if (!fe_eq(t, p.X)) return false;
  fe_mul(Z3, Z2, p.Z);
  fe_mul(t, y, Z3);
  return fe_eq(t, p.Y);
}

EC_D void jac_to_aff(uint32_t* out16, const Jac& p) {
  if (jac_is_inf(p)) {
#pragma unroll
    for (int i = 0; i < 16; ++i) out16[i] = 0;
    return;
  }
  Fe zi, zi2, zi3, x, y;
  fe_inv(zi, p.Z);
  fe_sqr(zi2, zi);
  fe_mul(zi3, zi2, zi);
  fe_mul(x, p.X, zi2);
  fe_mul(y, p.Y, zi3);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out16[i] = x.v[i];
    out16[8 + i] = y.v[i];
  }
}

// k (8 limbs, any value < 2^256) reduced mod q, in place
EC_D void scalar_reduce(uint32_t* k) {
  // k < 2^256 < 2q: one conditional subtraction
  int64_t br = 0;
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    int64_t d = (int64_t)k[i] - Q_LIMBS[i] + br;
    t[i] = (uint32_t)d;
    br = d >> 32;
  }
  if (br == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = t[i];
  }
}

}  // namespace ec
}  // namespace fsdkr
