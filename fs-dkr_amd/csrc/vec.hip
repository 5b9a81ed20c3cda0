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

__global__ void pdl_u1_kernel(const PdlU1Args a) {
  using namespace ec;
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.count) return;
  __builtin_amdgcn_s_setprio(1);   // one long serial EC chain per thread
  uint32_t k1[8], k2[8];
  bigint_mod_q(k1, a.s1 + (size_t)p * a.s1_len, a.s1_len);
  // k2 = (q - (e mod q)) mod q
  const uint32_t* e = a.e + (size_t)p * 8;
  uint32_t em[8];
  for (int i = 0; i < 8; ++i) em[i] = e[i];
  scalar_reduce(em);
  bool ez = true;
  for (int i = 0; i < 8; ++i) ez = ez && em[i] == 0;
  int64_t br = 0;
  for (int i = 0; i < 8; ++i) {
    const int64_t d = (int64_t)Q_LIMBS[i] - em[i] + br;
    k2[i] = ez ? 0u : (uint32_t)d;
    br = d >> 32;
  }
  Fe gx, gy, qx, qy, ux, uy;
  fe_load(gx, GX_LIMBS);
  fe_load(gy, GY_LIMBS);
  const bool qinf = aff_load(qx, qy, a.Q + (size_t)p * 16);
  const bool uinf = aff_load(ux, uy, a.u1 + (size_t)p * 16);
  Jac r;
  shamir_mul2_aff(r, k1, gx, gy, k2, qx, qy, qinf);
  const bool eq = jac_eq_aff(r, ux, uy, uinf);
  a.verdict[p] = (uint8_t)((a.verdict[p] & ~1u) | (eq ? 1u : 0u));
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
    scalar_mul_aff(r, k, x, y);
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
  hipLaunchKernelGGL(pdl_u1_kernel, dim3(blocks_for(a.count, 64)), dim3(64), 0, st, a);
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
