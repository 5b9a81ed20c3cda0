// SHA-256 (FIPS 180-4), host + device, streaming.  Used for the Fiat–Shamir
// challenges of the collect() path: curv DigestExt::chain_bigint over
// BigInt::to_bytes (minimal big-endian magnitude, zero -> one 0x00 byte)
// at zk_pdl_with_slack.rs:114-122, range_proofs.rs:150-157,
// ring_pedersen_proof.rs:130-135 and zk-paillier compute_digest.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fsdkr {

#define FSDKR_HD __host__ __device__ __forceinline__

struct Sha256 {
  uint32_t h[8];
  uint32_t* w;      // pending block as big-endian words (device: a per-thread LDS slot, see init)
  uint32_t nbuf;    // bytes in pending block
  uint64_t total;   // bytes absorbed
  uint32_t own[16]; // host storage (device code passes LDS: a dynamically indexed private array is scratch)

  FSDKR_HD static uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

  FSDKR_HD void init(uint32_t* buf = nullptr) {
    w = buf ? buf : own;
    h[0] = 0x6a09e667u; h[1] = 0xbb67ae85u; h[2] = 0x3c6ef372u; h[3] = 0xa54ff53au;
    h[4] = 0x510e527fu; h[5] = 0x9b05688cu; h[6] = 0x1f83d9abu; h[7] = 0x5be0cd19u;
    nbuf = 0;
    total = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = 0;
  }

  FSDKR_HD void compress() {
    const uint32_t K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
        0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
        0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
        0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
        0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
        0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
        0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = w[i];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      uint32_t wi;
      if (i < 16) {
        wi = W[i];
      } else {
        const uint32_t w15 = W[(i - 15) & 15], w2 = W[(i - 2) & 15];
        const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
        wi = W[i & 15] = W[i & 15] + s0 + W[(i - 7) & 15] + s1;
      }
      const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = hh + S1 + ch + K[i] + wi;
      const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
      const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }

  FSDKR_HD void byte(uint8_t v) {
    const uint32_t idx = nbuf >> 2, sh = 24 - 8 * (nbuf & 3);
    w[idx] |= (uint32_t)v << sh;
    ++nbuf;
    ++total;
    if (nbuf == 64) {
      compress();
      nbuf = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = 0;
    }
  }

  // four bytes x>>24, x>>16, x>>8, x (big-endian word) at any alignment
  FSDKR_HD void word(uint32_t x) {
    const uint32_t off = nbuf & 3, idx = nbuf >> 2;
    if (off == 0) w[idx] = x;
    else w[idx] |= x >> (8 * off);
    nbuf += 4;
    total += 4;
    if (nbuf >= 64) {
      compress();
      nbuf -= 64;
#pragma unroll
      for (int i = 0; i < 16; ++i) w[i] = 0;
      if (off) w[0] = x << (32 - 8 * off);
    } else if (off) {
      w[idx + 1] = x << (32 - 8 * off);
    }
  }

  FSDKR_HD void bytes(const uint8_t* p, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) byte(p[i]);
  }

  // BigInt::to_bytes of a little-endian limb array: minimal big-endian bytes,
  // zero encodes as a single 0x00 byte.
  FSDKR_HD void bigint(const uint32_t* limbs, uint32_t nlimbs) {
    int top = (int)nlimbs - 1;
    while (top >= 0 && limbs[top] == 0) --top;
    if (top < 0) {
      byte(0);
      return;
    }
    uint32_t v = limbs[top];
    int sh = 24;
    while (sh > 0 && ((v >> sh) & 0xffu) == 0) sh -= 8;
    for (; sh >= 0; sh -= 8) byte((uint8_t)(v >> sh));
    for (int k = top - 1; k >= 0; --k) word(limbs[k]);
  }

  // finalize; digest as a 256-bit little-endian limb array (= BigInt::from_bytes(digest))
  FSDKR_HD void finish_le(uint32_t* out8) {
    const uint64_t bits = total * 8;
    byte(0x80);
    while (nbuf != 56) byte(0);
    for (int i = 7; i >= 0; --i) byte((uint8_t)(bits >> (8 * i)));
#pragma unroll
    for (int i = 0; i < 8; ++i) out8[i] = h[7 - i];
  }
};

}  // namespace fsdkr
