// Hashing and small-arithmetic kernels of the batched collect() job (gfx950).
// Fiat-Shamir transcripts restated from curv DigestExt::chain_bigint (SHA-256
// over BigInt::to_bytes):
//   (the PDL challenge e = H(G,Q,c,z,u1,u2,u3), zk_pdl_with_slack.rs:114-122, is
//    hashed on the host by fsdkr_collect_prepare: collect.cpp)
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
  __builtin_amdgcn_s_setprio(3);   // on the main chain ahead of J5: short, latency-critical
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
// e = H(A_0 .. A_{M-1}); bits[m][i/32] bit i%32 = Lsb0 bit i of e.to_bytes();
// panic[m] != 0 if e.to_bytes() is shorter than M bits (BitVec index panic at bit
// panic[m]-1; checks before that index still run and may fail first).
//
// One wave per message.  The M values are absorbed PED_CHUNK at a time: the 64
// lanes load the chunk's limbs (coalesced) into LDS, lanes 0..PED_CHUNK-1 find
// each value's minimal big-endian length, and all lanes scatter the bytes of
// the chunk's to_bytes() encodings into one contiguous LDS byte stream behind
// the previous chunk's unconsumed tail; lane 0 then runs the serial SHA-256
// compressions straight from LDS.  (One thread per message reading limbs from
// global memory word by word exposed the load latency on every 4 bytes.)
constexpr int PED_CHUNK = 16;
constexpr int PED_MAX_LIMBS = 96;   // 3072-bit moduli
__global__ __launch_bounds__(64) void ped_hash_kernel(const PedHashArgs a) {
  const uint32_t m = blockIdx.x;
  if (m >= a.count) return;
  __builtin_amdgcn_s_setprio(2);   // a serial chain sharing SIMDs with exponentiation waves
  const int lane = threadIdx.x;
  __shared__ uint32_t lim[PED_CHUNK * PED_MAX_LIMBS];
  __shared__ uint8_t stream[64 + PED_CHUNK * PED_MAX_LIMBS * 4 + 64];
  __shared__ uint32_t len[PED_CHUNK], off[PED_CHUNK + 1];
  __shared__ uint32_t sha_w[16];
  const uint32_t nl = a.a_len;
  const uint32_t* A = a.A + (size_t)m * a.M * nl;
  Sha256 h;
  if (lane == 0) h.init(sha_w);
  uint32_t have = 0;          // unconsumed stream bytes at the front of `stream` (< 64)
  uint64_t consumed = 0;      // bytes compressed so far
  for (uint32_t c0 = 0; c0 < a.M; c0 += PED_CHUNK) {
    const uint32_t cnt = min((uint32_t)PED_CHUNK, a.M - c0);
    for (uint32_t k = lane; k < cnt * nl; k += 64) lim[k] = A[(size_t)c0 * nl + k];
    __syncthreads();
    if (lane < (int)cnt) {     // BigInt::to_bytes length: minimal magnitude, 0 -> one 0x00 byte
      const uint32_t* x = lim + lane * nl;
      int top = (int)nl - 1;
      while (top >= 0 && x[top] == 0) --top;
      uint32_t bytes = 1;
      if (top >= 0) bytes = 4u * (uint32_t)top + (32u - (uint32_t)__builtin_clz(x[top]) + 7u) / 8u;
      len[lane] = bytes;
    }
    __syncthreads();
    if (lane == 0) {
      uint32_t o = have;
      for (uint32_t i = 0; i < cnt; ++i) {
        off[i] = o;
        o += len[i];
      }
      off[cnt] = o;
    }
    __syncthreads();
    // big-endian bytes: byte j (from the least significant end) of value i at off[i] + len[i] - 1 - j
    for (uint32_t k = lane; k < cnt * nl; k += 64) {
      const uint32_t i = k / nl, limb = k % nl, v = lim[k];
      const uint32_t L = len[i], base = off[i] + L - 1;
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t j = 4 * limb + b;
        if (j < L) stream[base - j] = (uint8_t)(v >> (8 * b));
      }
    }
    __syncthreads();
    const uint32_t total = off[cnt];
    const uint32_t blocks = total / 64;
    if (lane == 0) {
      for (uint32_t blk = 0; blk < blocks; ++blk) {
        const uint8_t* s = stream + blk * 64;
#pragma unroll
        for (int q = 0; q < 16; ++q)
          sha_w[q] = ((uint32_t)s[4 * q] << 24) | ((uint32_t)s[4 * q + 1] << 16) | ((uint32_t)s[4 * q + 2] << 8) |
                     (uint32_t)s[4 * q + 3];
        h.compress();
      }
    }
    consumed += 64ull * blocks;
    have = total - 64 * blocks;
    __syncthreads();
    // move the tail (< 64 bytes) to the front for the next chunk
    uint8_t t = 0;
    if (lane < (int)have) t = stream[64 * blocks + lane];
    __syncthreads();
    if (lane < (int)have) stream[lane] = t;
    __syncthreads();
  }
  if (lane != 0) return;
  for (int q = 0; q < 16; ++q) sha_w[q] = 0;
  h.nbuf = 0;
  h.total = consumed;
  for (uint32_t k = 0; k < have; ++k) h.byte(stream[k]);
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

// the inputs-only prefix of Alice's hash: N, N + 1, c, z (range_proofs.rs:150-154)
__device__ __forceinline__ void alice_absorb_prefix(Sha256& h, const AliceHashArgs& a, uint32_t p) {
  const uint32_t* N = P32(a.n_ptr[p]);
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
}

// The SHA-256 state after the prefix, per proof: launched early beside the
// exponentiations, so the pipeline's last kernel (alice_hash) absorbs only u and
// w (12 of ~32 blocks at 2048-bit keys).  [h0..h7 | nbuf | total lo, hi | w0..w15]
__global__ void alice_prefix_kernel(const AliceHashArgs a) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.count) return;
  __shared__ uint32_t sha_w[64 * 16];  // launch blocks are 64 threads
  Sha256 h;
  h.init(sha_w + threadIdx.x * 16);
  alice_absorb_prefix(h, a, p);
  uint32_t* s = a.state + (size_t)p * 32;
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = h.h[i];
  s[8] = h.nbuf;
  s[9] = (uint32_t)h.total;
  s[10] = (uint32_t)(h.total >> 32);
#pragma unroll
  for (int i = 0; i < 16; ++i) s[11 + i] = h.w[i];
}

// e' = H(N, N+1, c, z, u, w) == e  ->  verdict bit (AND-ed with the host's pre-checks);
// with a.state the prefix comes from alice_prefix_kernel
__global__ void alice_hash_kernel(const AliceHashArgs a) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.count) return;
  __shared__ uint32_t sha_w[64 * 16];  // launch blocks are 64 threads
  Sha256 h;
  h.init(sha_w + threadIdx.x * 16);
  if (a.state) {
    const uint32_t* s = a.state + (size_t)p * 32;
#pragma unroll
    for (int i = 0; i < 8; ++i) h.h[i] = s[i];
    h.nbuf = s[8];
    h.total = (uint64_t)s[9] | ((uint64_t)s[10] << 32);
#pragma unroll
    for (int i = 0; i < 16; ++i) h.w[i] = s[11 + i];
  } else {
    alice_absorb_prefix(h, a, p);
  }
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
hipError_t launch_ped_hash(const PedHashArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  if (a.a_len > (uint32_t)PED_MAX_LIMBS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ped_hash_kernel, dim3(a.count), dim3(64), 0, st, a);   // one wave per message
  return hipGetLastError();
}
hipError_t launch_alice_hash(const AliceHashArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  hipLaunchKernelGGL(alice_hash_kernel, dim3(blocks_for(a.count, 64)), dim3(64), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_alice_prefix(const AliceHashArgs& a, hipStream_t st) {
  if (!a.count) return hipSuccess;
  if (!a.state) return hipErrorInvalidValue;
  hipLaunchKernelGGL(alice_prefix_kernel, dim3(blocks_for(a.count, 64)), dim3(64), 0, st, a);
  return hipGetLastError();
}

}  // namespace fsdkr
