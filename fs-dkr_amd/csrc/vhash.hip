// Hashing and small-arithmetic kernels of the batched collect() job (gfx950).
// Fiat-Shamir transcripts restated from curv DigestExt::chain_bigint (SHA-256
// over BigInt::to_bytes):
//   pdl_hash        e = H(G,Q,c,z,u1,u2,u3)                    zk_pdl_with_slack.rs:114-122
//   alice_hash      e' = H(N,N+1,c,z,u,w) == e                 range_proofs.rs:150-163
//   ped_hash        e = H(A_0..A_M-1), Lsb0 bits              ring_pedersen_proof.rs:130-142
//   binom           (N+1)^s1 = 1 + s1*N  (s1 < N)              zk_pdl_with_slack.rs:129-135
#include "mont29.hpp"
#include "sha256.hpp"
#include "verify.h"
#include <cstdlib>

namespace fsdkr {

__device__ __forceinline__ const uint32_t* P32(uint64_t a) { return reinterpret_cast<const uint32_t*>(a); }
static inline uint32_t blocks_for(uint32_t n, uint32_t per) { return (n + per - 1) / per; }

// ---------------------------------------------------------------- binom --------
// out[p] (out_limbs) = 1 + s[p] * n[p]   (caller guarantees no overflow of out_limbs)
__global__ void binom_kernel(const BinomArgs a) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.count) return;
  const uint32_t* s = P32(a.s_ptr[p]);
  const uint32_t* n = P32(a.n_ptr[p]);
  uint32_t* o = a.out + (size_t)p * a.out_limbs;
  for (uint32_t k = 0; k < a.out_limbs; ++k) o[k] = 0;
  for (uint32_t i = 0; i < a.s_len; ++i) {
    const uint32_t si = s[i];
    if (!si) continue;
    uint64_t c = 0;
    for (uint32_t j = 0; j < a.n_len && i + j < a.out_limbs; ++j) {
      c += (uint64_t)si * n[j] + o[i + j];
      o[i + j] = (uint32_t)c;
      c >>= 32;
    }
    for (uint32_t k = i + a.n_len; c && k < a.out_limbs; ++k) {
      c += o[k];
      o[k] = (uint32_t)c;
      c >>= 32;
    }
  }
  uint64_t c = 1;
  for (uint32_t k = 0; c && k < a.out_limbs; ++k) {
    c += o[k];
    o[k] = (uint32_t)c;
    c >>= 32;
  }
}

// ------------------------------------------------------------- hashing --------
__constant__ const uint8_t G_COMPRESSED[33] = {
    0x02, 0x79, 0xBE, 0x66, 0x7E, 0xF9, 0xDC, 0xBB, 0xAC, 0x55, 0xA0, 0x62, 0x95, 0xCE, 0x87, 0x0B, 0x07,
    0x02, 0x9B, 0xFC, 0xDB, 0x2D, 0xCE, 0x28, 0xD9, 0x59, 0xF2, 0x81, 0x5B, 0x16, 0xF8, 0x17, 0x98};

// BigInt::from_bytes(P.to_bytes(true)) re-encoded by to_bytes: 33 bytes for a
// finite point (prefix 2/3 is nonzero), a single 0x00 for infinity.
__device__ __forceinline__ void absorb_point(Sha256& h, const uint32_t* p16) {
  bool inf = true;
#pragma unroll
  for (int i = 0; i < 16; ++i) inf = inf && (p16[i] == 0);
  if (inf) {
    h.byte(0);
    return;
  }
  h.byte((uint8_t)(2 + (p16[8] & 1u)));
  for (int i = 7; i >= 0; --i) {
    const uint32_t x = p16[i];
    h.byte((uint8_t)(x >> 24));
    h.byte((uint8_t)(x >> 16));
    h.byte((uint8_t)(x >> 8));
    h.byte((uint8_t)x);
  }
}

__global__ void pdl_hash_kernel(const PdlHashArgs a) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.count) return;
  __shared__ uint32_t sha_w[64 * 16];  // launch blocks are 64 threads
  Sha256 h;
  h.init(sha_w + threadIdx.x * 16);
  for (int i = 0; i < 33; ++i) h.byte(G_COMPRESSED[i]);
  absorb_point(h, a.Q + (size_t)p * 16);
  h.bigint(a.c + (size_t)p * a.c_len, a.c_len);
  h.bigint(a.z + (size_t)p * a.z_len, a.z_len);
  absorb_point(h, a.u1 + (size_t)p * 16);
  h.bigint(a.u2 + (size_t)p * a.c_len, a.c_len);
  h.bigint(a.u3 + (size_t)p * a.z_len, a.z_len);
  h.finish_le(a.e_out + (size_t)p * 8);
}

// e = H(A_0 .. A_{M-1}); bits[m][i/32] bit i%32 = Lsb0 bit i of e.to_bytes();
// panic[m] != 0 if e.to_bytes() is shorter than M bits (BitVec index panic at bit
// panic[m]-1; checks before that index still run and may fail first).
__global__ void ped_hash_kernel(const PedHashArgs a) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= a.count) return;
  __builtin_amdgcn_s_setprio(3);   // a long serial chain sharing SIMDs with exponentiation waves
  __shared__ uint32_t sha_w[64 * 16];  // launch blocks are 64 threads
  Sha256 h;
  h.init(sha_w + threadIdx.x * 16);
  const uint32_t* A = a.A + (size_t)m * a.M * a.a_len;
  for (uint32_t i = 0; i < a.M; ++i) h.bigint(A + (size_t)i * a.a_len, a.a_len);
  uint32_t e[8];
  h.finish_le(e);
  // big-endian minimal bytes of e
  uint8_t be[32];
  int nb = 0;
  bool lead = true;
  for (int i = 7; i >= 0; --i)
    for (int sh = 24; sh >= 0; sh -= 8) {
      const uint8_t b = (uint8_t)(e[i] >> sh);
      if (lead && b == 0) continue;
      lead = false;
      be[nb++] = b;
    }
  if (nb == 0) be[nb++] = 0;
  uint32_t* bits = a.bits + (size_t)m * ((a.M + 31) / 32);
  for (uint32_t w = 0; w < (a.M + 31) / 32; ++w) bits[w] = 0;
  // short challenge: 1 + the number of bits the reference reads before its index panic
  a.panic[m] = (8u * (uint32_t)nb < a.M) ? 1u + 8u * (uint32_t)nb : 0u;
  for (uint32_t i = 0; i < a.M && (i >> 3) < (uint32_t)nb; ++i)
    if ((be[i >> 3] >> (i & 7)) & 1u) bits[i >> 5] |= 1u << (i & 31);
}

// e' = H(N, N+1, c, z, u, w) == e  ->  verdict bit (AND-ed with the host's pre-checks)
__global__ void alice_hash_kernel(const AliceHashArgs a) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.count) return;
  const uint32_t* N = P32(a.n_ptr[p]);
  __shared__ uint32_t sha_w[64 * 16];  // launch blocks are 64 threads
  Sha256 h;
  h.init(sha_w + threadIdx.x * 16);
  h.bigint(N, a.n_len);
  // N + 1, streamed limb by limb from the top: compute the carry chain first
  {
    uint32_t np1[128];
    uint64_t c = 1;
    for (uint32_t k = 0; k < a.n_len; ++k) {
      c += N[k];
      np1[k] = (uint32_t)c;
      c >>= 32;
    }
    if (c) {  // N + 1 == 2^(32 n_len): needs one more limb
      np1[a.n_len] = 1;
      h.bigint(np1, a.n_len + 1);
    } else {
      h.bigint(np1, a.n_len);
    }
  }
  h.bigint(P32(a.c_ptr[p]), a.c_len);
  h.bigint(a.z + (size_t)p * a.z_len, a.z_len);
  h.bigint(a.u + (size_t)p * a.c_len, a.c_len);
  h.bigint(a.w + (size_t)p * a.z_len, a.z_len);
  uint32_t d[8];
  h.finish_le(d);
  const uint32_t* e = a.e + (size_t)p * a.e_len;
  bool eq = true;
  for (uint32_t k = 0; k < a.e_len; ++k) eq = eq && (e[k] == (k < 8 ? d[k] : 0u));
  for (uint32_t k = a.e_len; k < 8; ++k) eq = eq && (d[k] == 0u);
  a.verdict[p] = (a.verdict[p] && eq) ? 1 : 0;
}

// ------------------------------------------------------------- launchers -------
hipError_t launch_binom(const BinomArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  hipLaunchKernelGGL(binom_kernel, dim3(blocks_for(a.count, 128)), dim3(128), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_pdl_hash(const PdlHashArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  hipLaunchKernelGGL(pdl_hash_kernel, dim3(blocks_for(a.count, 64)), dim3(64), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_ped_hash(const PedHashArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  hipLaunchKernelGGL(ped_hash_kernel, dim3(blocks_for(a.count, 64)), dim3(64), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_alice_hash(const AliceHashArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  hipLaunchKernelGGL(alice_hash_kernel, dim3(blocks_for(a.count, 64)), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace fsdkr
