// secp256k1 kernels of the batched collect() job (gfx950, secp256k1.hpp):
//   pdl_u1          G*s1 + Q*(q-e) == u1                       zk_pdl_with_slack.rs:124-127
//   feldman         S_i == sum_k A_k (i+1)^k                   refresh_message.rs:177-188
//   ec_msm          sum_j s_j P_j (pk_vec, G*x)                refresh_message.rs:446-464
#include "secp256k1.hpp"
#include "verify.h"
#include <cstdlib>

namespace fsdkr {

__device__ __forceinline__ const uint32_t* P32(uint64_t a) { return reinterpret_cast<const uint32_t*>(a); }
static inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

// ------------------------------------------------------------- secp256k1 ------
// scalar (len limbs, any size) mod q
__device__ __forceinline__ void bigint_mod_q(uint32_t* r, const uint32_t* x, uint32_t len) {
  // Horner over 32-bit limbs from the top: r = r*2^32 + limb (mod q)
  // q = 2^256 - c, c = 0x14551231950b75fc4402da1732fc9bebf (129 bits)
  const uint32_t C5[5] = {0x2FC9BEBFu, 0x402DA173u, 0x50B75FC4u, 0x45512319u, 0x1u};
  for (int i = 0; i < 8; ++i) r[i] = 0;
  for (int k = (int)len - 1; k >= 0; --k) {
    // t = r * 2^32 + x[k]  (288 bits): hi = top limb of r
    const uint32_t hi = r[7];
    for (int i = 7; i > 0; --i) r[i] = r[i - 1];
    r[0] = x[k];
    // r += hi * c   (hi*c < 2^161)
    uint64_t cc = 0;
    for (int i = 0; i < 8; ++i) {
      cc += (uint64_t)r[i] + (i < 5 ? (uint64_t)hi * C5[i] : 0ull);
      r[i] = (uint32_t)cc;
      cc >>= 32;
    }
    // overflow (2^256) == c mod q
    while (cc) {
      const uint64_t ov = cc;
      cc = 0;
      for (int i = 0; i < 8; ++i) {
        cc += (uint64_t)r[i] + (i < 5 ? ov * C5[i] : 0ull);
        r[i] = (uint32_t)cc;
        cc >>= 32;
      }
    }
    ec::scalar_reduce(r);
  }
  ec::scalar_reduce(r);
}

// ---- GLV endomorphism of secp256k1 (lambda P = (beta x, y), lambda^3 = 1 mod q) ----
// k = r1 + r2 lambda (mod q) with |r1|, |r2| < 2^128 (the lattice split of
// libsecp256k1's secp256k1_scalar_split_lambda, restated; constants and the
// 128-bit bound checked against the oracle's secp256k1 in
// tests/test_ec_glv.py), so k P = r1 P + r2 (lambda P) runs 128 doublings
// instead of 256.
__constant__ const uint32_t GLV_LAMBDA[8] = {0x1B23BD72u, 0xDF02967Cu, 0x20816678u, 0x122E22EAu,
                                             0x8812645Au, 0xA5261C02u, 0xC05C30E0u, 0x5363AD4Cu};
__constant__ const uint32_t GLV_BETA[8] = {0x719501EEu, 0xC1396C28u, 0x12F58995u, 0x9CF04975u,
                                           0xAC3434E9u, 0x6E64479Eu, 0x657C0710u, 0x7AE96A2Bu};
__constant__ const uint32_t GLV_MB1[4] = {0x0ABFE4C3u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};   // -b1
__constant__ const uint32_t GLV_MB2[8] = {0x3DB1562Cu, 0xD765CDA8u, 0x0774346Du, 0x8A280AC5u,
                                          0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};   // -b2 mod q
__constant__ const uint32_t GLV_G1[8] = {0x45DBB031u, 0xE893209Au, 0x71E8CA7Fu, 0x3DAA8A14u,
                                         0x9284EB15u, 0xE86C90E4u, 0xA7D46BCDu, 0x3086D221u};   // round(2^384 b2 / q)
__constant__ const uint32_t GLV_G2[8] = {0x8AC47F71u, 0x1571B4AEu, 0x9DF506C6u, 0x221208ACu,
                                         0x0ABFE4C4u, 0x6F547FA9u, 0x010E8828u, 0xE4437ED6u};   // round(2^384 (-b1) / q)
__constant__ const uint32_t Q_HALF[8] = {0x681B20A0u, 0xDFE92F46u, 0x57A4501Du, 0x5D576E73u,
                                         0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};   // (q - 1) / 2

// t[0 .. na + nb) = a * b (schoolbook, exact)
__device__ __forceinline__ void mul_limbs(uint32_t* t, const uint32_t* a, int na, const uint32_t* b, int nb) {
  for (int i = 0; i < na + nb; ++i) t[i] = 0;
  for (int i = 0; i < na; ++i) {
    uint64_t c = 0;
    for (int j = 0; j < nb; ++j) {
      c += (uint64_t)a[i] * b[j] + t[i + j];
      t[i + j] = (uint32_t)c;
      c >>= 32;
    }
    t[i + nb] = (uint32_t)c;
  }
}
// r = (a + b) mod q, a, b < q
__device__ __forceinline__ void scalar_add_mod(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint64_t c = 0;
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a[i] + b[i];
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  // >= q or a carry out: subtract q (2^256 - q fits the carry)
  int64_t br = 0;
  uint32_t t[8];
  for (int i = 0; i < 8; ++i) {
    const int64_t d = (int64_t)r[i] - ec::Q_LIMBS[i] + br;
    t[i] = (uint32_t)d;
    br = d >> 32;
  }
  if (c || br == 0)
    for (int i = 0; i < 8; ++i) r[i] = t[i];
}
// r = (a - b) mod q, a, b < q
__device__ __forceinline__ void scalar_sub_mod(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  int64_t br = 0;
  for (int i = 0; i < 8; ++i) {
    const int64_t d = (int64_t)a[i] - b[i] + br;
    r[i] = (uint32_t)d;
    br = d >> 32;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 8; ++i) {
      c += (uint64_t)r[i] + ec::Q_LIMBS[i];
      r[i] = (uint32_t)c;
      c >>= 32;
    }
  }
}
// c = round(k g / 2^384): 5 limbs (< 2^129)
__device__ __forceinline__ void mul_shift_384(uint32_t* c, const uint32_t* k, const uint32_t* g) {
  uint32_t t[16];
  mul_limbs(t, k, 8, g, 8);
  uint64_t x = (uint64_t)t[12] + (t[11] >> 31);
  for (int i = 0; i < 4; ++i) {
    c[i] = (uint32_t)x;
    x = (x >> 32) + (i + 13 < 16 ? t[i + 13] : 0u);
  }
  c[4] = (uint32_t)x;
}
// k (< q) = s1 + s2 lambda (mod q), |s1|, |s2| < 2^128: magnitudes m1, m2 (4 limbs) and signs
__device__ __forceinline__ void scalar_split_lambda(const uint32_t* k, uint32_t* m1, bool* neg1, uint32_t* m2,
                                                    bool* neg2) {
  uint32_t c1[5], c2[5], a[8], b[8], r2[8], u[8], r1[8], t[16];
  mul_shift_384(c1, k, GLV_G1);
  mul_shift_384(c2, k, GLV_G2);
  mul_limbs(t, c1, 5, GLV_MB1, 4);
  bigint_mod_q(a, t, 9);
  mul_limbs(t, c2, 5, GLV_MB2, 8);
  bigint_mod_q(b, t, 13);
  scalar_add_mod(r2, a, b);
  mul_limbs(t, r2, 8, GLV_LAMBDA, 8);
  bigint_mod_q(u, t, 16);
  scalar_sub_mod(r1, k, u);
  // signed: r > (q - 1) / 2 stands for r - q
  auto signed_mag = [](const uint32_t* r, uint32_t* m, bool* neg) {
    int64_t br = 0;
    for (int i = 0; i < 8; ++i) {   // Q_HALF - r: borrow iff r > (q - 1) / 2
      const int64_t d = (int64_t)Q_HALF[i] - r[i] + br;
      br = d >> 32;
    }
    *neg = br != 0;
    if (*neg) {   // q - r
      int64_t b2 = 0;
      for (int i = 0; i < 4; ++i) {
        const int64_t d = (int64_t)ec::Q_LIMBS[i] - r[i] + b2;
        m[i] = (uint32_t)d;
        b2 = d >> 32;
      }
    } else {
      for (int i = 0; i < 4; ++i) m[i] = r[i];
    }
  };
  signed_mag(r1, m1, neg1);
  signed_mag(r2, m2, neg2);
}

// r = m P (P affine (x, y), m < 2^128 in 4 limbs): 4-bit fixed windows, a
// 15-entry Jacobian table (scratch) built by mixed additions
__device__ __forceinline__ void mul_aff_128(ec::Jac& r, const uint32_t* m, const ec::Fe& x, const ec::Fe& y, bool inf) {
  using namespace ec;
  if (inf) {
    jac_set_inf(r);
    return;
  }
  Jac T[16];
  jac_set_inf(T[0]);
  T[1].X = x;
  T[1].Y = y;
  fe_set_u32(T[1].Z, 1);
  for (int d = 2; d < 16; ++d) jac_add_aff(T[d], T[d - 1], x, y);
  Jac acc;
  jac_set_inf(acc);
  for (int nib = 31; nib >= 0; --nib) {
    if (nib != 31) {
      jac_dbl(acc, acc);
      jac_dbl(acc, acc);
      jac_dbl(acc, acc);
      jac_dbl(acc, acc);
    }
    const uint32_t d = (m[nib >> 3] >> (4 * (nib & 7))) & 15u;
    if (d) jac_add(acc, acc, T[d]);
  }
  r = acc;
}

// r = k P (P affine, k < q) in one thread: the GLV split and Shamir's trick over
// the two 128-bit halves (128 shared doublings; the lambda table is the first
// one's X times beta, with Y negated where the halves' signs differ)
__device__ __forceinline__ void glv_mul_aff(ec::Jac& r, const uint32_t* k, const ec::Fe& x, const ec::Fe& y) {
  using namespace ec;
  uint32_t m1[4], m2[4];
  bool n1, n2;
  scalar_split_lambda(k, m1, &n1, m2, &n2);
  Fe x1 = x, y1 = y;
  if (n1 && !fe_is_zero(y1)) {
    Fe pp;
    fe_load(pp, P_LIMBS);
    fe_sub(y1, pp, y1);
  }
  Jac T1[16], T2[16];
  jac_set_inf(T1[0]);
  T1[1].X = x1;
  T1[1].Y = y1;
  fe_set_u32(T1[1].Z, 1);
  for (int d = 2; d < 16; ++d) jac_add_aff(T1[d], T1[d - 1], x1, y1);
  Fe bt, pp;
  fe_load(bt, GLV_BETA);
  fe_load(pp, P_LIMBS);
  const bool flip = n1 != n2;
  T2[0] = T1[0];
  for (int d = 1; d < 16; ++d) {   // lambda (±T1[d]) = (beta X, ±Y, Z) in Jacobian coordinates
    fe_mul(T2[d].X, T1[d].X, bt);
    if (flip && !fe_is_zero(T1[d].Y)) fe_sub(T2[d].Y, pp, T1[d].Y);
    else T2[d].Y = T1[d].Y;
    T2[d].Z = T1[d].Z;
  }
  Jac acc;
  jac_set_inf(acc);
  for (int nib = 31; nib >= 0; --nib) {
    if (nib != 31) {
      jac_dbl(acc, acc);
      jac_dbl(acc, acc);
      jac_dbl(acc, acc);
      jac_dbl(acc, acc);
    }
    const uint32_t d1 = (m1[nib >> 3] >> (4 * (nib & 7))) & 15u;
    const uint32_t d2 = (m2[nib >> 3] >> (4 * (nib & 7))) & 15u;
    if (d1) jac_add(acc, acc, T1[d1]);
    if (d2) jac_add(acc, acc, T2[d2]);
  }
  r = acc;
}

// lambda-image and sign of an affine point: (beta x, y) when lam, y -> p - y when neg
__device__ __forceinline__ void glv_point(ec::Fe& x, ec::Fe& y, bool lam, bool neg) {
  using namespace ec;
  if (lam) {
    Fe bt;
    fe_load(bt, GLV_BETA);
    fe_mul(x, x, bt);
  }
  if (neg && !fe_is_zero(y)) {
    Fe pp;
    fe_load(pp, P_LIMBS);
    fe_sub(y, pp, y);
  }
}

// G*s1 + Q*(q-e) == u1 (zk_pdl_with_slack.rs:124-127): four lanes per pair, each
// one 128-bit scalar multiplication of the GLV split -- lane 0: s1_a G, lane 1:
// s1_b (lambda G), lane 2: k2_a Q, lane 3: k2_b (lambda Q) -- then two rounds of
// Jacobian additions across the quad.  The round-5 kernel ran one thread per pair
// (a 256-bit Shamir ladder, 60 waves at n = 64: 19-23 ms, the pipeline's longest
// latency chain after GA); this one issues 128 doublings per lane on 4x the waves.
__global__ void pdl_u1_kernel(const PdlU1Args a) {
  using namespace ec;
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t p = tid >> 2, j = tid & 3u;
  if (p >= a.count) return;   // whole quads (count pairs x 4 lanes)
  __builtin_amdgcn_s_setprio(3);   // a long serial EC chain per lane on few waves: wins issue arbitration
  uint32_t k[8];
  if (j < 2) {
    bigint_mod_q(k, a.s1 + (size_t)p * a.s1_len, a.s1_len);
  } else {   // (q - (e mod q)) mod q
    const uint32_t* e = a.e + (size_t)p * 8;
    uint32_t em[8];
    for (int i = 0; i < 8; ++i) em[i] = e[i];
    scalar_reduce(em);
    bool ez = true;
    for (int i = 0; i < 8; ++i) ez = ez && em[i] == 0;
    int64_t br = 0;
    for (int i = 0; i < 8; ++i) {
      const int64_t d = (int64_t)Q_LIMBS[i] - em[i] + br;
      k[i] = ez ? 0u : (uint32_t)d;
      br = d >> 32;
    }
  }
  uint32_t m1[4], m2[4];
  bool n1, n2;
  scalar_split_lambda(k, m1, &n1, m2, &n2);
  const bool second = (j & 1u) != 0;
  Fe x, y;
  bool inf;
  if (j < 2) {
    fe_load(x, GX_LIMBS);
    fe_load(y, GY_LIMBS);
    inf = false;
  } else {
    inf = aff_load(x, y, a.Q + (size_t)p * 16);
  }
  glv_point(x, y, second, second ? n2 : n1);
  Jac r;
  mul_aff_128(r, second ? m2 : m1, x, y, inf);
  // quad sum: lanes (0,1) and (2,3), then the two halves
  for (int step = 1; step <= 2; step <<= 1) {
    Jac o;
    for (int i = 0; i < 8; ++i) {
      o.X.v[i] = (uint32_t)__shfl_xor((int)r.X.v[i], step);
      o.Y.v[i] = (uint32_t)__shfl_xor((int)r.Y.v[i], step);
      o.Z.v[i] = (uint32_t)__shfl_xor((int)r.Z.v[i], step);
    }
    jac_add(r, r, o);
  }
  if (j == 0) {
    Fe ux, uy;
    const bool uinf = aff_load(ux, uy, a.u1 + (size_t)p * 16);
    const bool eq = jac_eq_aff(r, ux, uy, uinf);
    a.verdict[p] = (uint8_t)((a.verdict[p] & ~1u) | (eq ? 1u : 0u));
  }
}

// S_{k,i} == Horner(A_k, i+1) over the message's own commitment vector
// (curv get_point_commitment: fold from the top coefficient; empty -> unwrap panic)
__global__ void feldman_kernel(const FeldmanArgs a) {
  using namespace ec;
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.count) return;
  if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  const FeldmanInfo in = a.info[p];
  if (in.ncoef == 0) {
    a.verdict[p] = 2u;
    return;
  }
  const uint32_t* A = a.vss + (size_t)in.off * 16;
  const uint32_t idx = in.idx;
  Jac acc;
  Fe x, y;
  if (aff_load(x, y, A + (size_t)(in.ncoef - 1) * 16)) {
    jac_set_inf(acc);
  } else {
    acc.X = x;
    acc.Y = y;
    fe_set_u32(acc.Z, 1);
  }
  for (int j = (int)in.ncoef - 2; j >= 0; --j) {
    // acc = acc * idx
    Jac r;
    jac_set_inf(r);
    for (int b = 31 - __builtin_clz(idx); b >= 0; --b) {
      jac_dbl(r, r);
      if ((idx >> b) & 1u) jac_add(r, r, acc);
    }
    acc = r;
    if (!aff_load(x, y, A + (size_t)j * 16)) jac_add_aff(acc, acc, x, y);
  }
  const bool sinf = aff_load(x, y, a.S + (size_t)p * 16);
  a.verdict[p] = jac_eq_aff(acc, x, y, sinf) ? 1u : 0u;
}

// out[o] = sum_j s[o][j] * P[o][j]: one thread per term (a full 256-bit scalar
// multiplication each), then one thread per output sums its terms.  The terms
// of one output are independent, so spreading them over threads turns the
// pk_vec rebuild (n outputs x (t+1) terms, refresh_message.rs:455-464) from
// t+1 serial ladders per thread into one ladder per thread.
__global__ void ec_msm_term_kernel(const EcMsmArgs a) {
  using namespace ec;
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= a.count * a.terms) return;
  if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  else if (a.prio == 2) __builtin_amdgcn_s_setprio(2);
  else if (a.prio == 1) __builtin_amdgcn_s_setprio(1);
  uint32_t* J = a.scratch + (size_t)q * 24;
  const uint32_t* pt = P32(a.pt_ptr[q]);
  const uint32_t* sc = a.scalars + (size_t)q * 8;
  Fe x, y;
  Jac r;
  if (aff_load(x, y, pt)) {
    jac_set_inf(r);
  } else {
    uint32_t k[8];
    for (int i = 0; i < 8; ++i) k[i] = sc[i];
    scalar_reduce(k);
    glv_mul_aff(r, k, x, y);   // 128 shared doublings instead of a 256-bit double-and-add ladder
  }
  for (int i = 0; i < 8; ++i) {
    J[i] = r.X.v[i];
    J[8 + i] = r.Y.v[i];
    J[16 + i] = r.Z.v[i];
  }
}

__global__ void ec_msm_sum_kernel(const EcMsmArgs a) {
  using namespace ec;
  const uint32_t o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= a.count) return;
  if (a.prio >= 3) __builtin_amdgcn_s_setprio(3);
  Jac acc;
  jac_set_inf(acc);
  for (uint32_t j = 0; j < a.terms; ++j) {
    const uint32_t* J = a.scratch + ((size_t)o * a.terms + j) * 24;
    Jac t;
    for (int i = 0; i < 8; ++i) {
      t.X.v[i] = J[i];
      t.Y.v[i] = J[8 + i];
      t.Z.v[i] = J[16 + i];
    }
    jac_add(acc, acc, t);
  }
  jac_to_aff(a.out + (size_t)o * 16, acc);
}

// ------------------------------------------------------------- launchers -------
hipError_t launch_pdl_u1(const PdlU1Args& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  hipLaunchKernelGGL(pdl_u1_kernel, dim3(blocks_for(a.count * 4, 64)), dim3(64), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_feldman(const FeldmanArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  hipLaunchKernelGGL(feldman_kernel, dim3(blocks_for(a.count, 64)), dim3(64), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_ec_msm(const EcMsmArgs& a, hipStream_t st) {
  if (!a.count || !a.terms) return hipSuccess;
  hipLaunchKernelGGL(ec_msm_term_kernel, dim3(blocks_for(a.count * a.terms, 64)), dim3(64), 0, st, a);
  hipLaunchKernelGGL(ec_msm_sum_kernel, dim3(blocks_for(a.count, 64)), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace fsdkr
