// Integer / f64 VALU issue-rate microbenchmark for gfx950 (MI355X).
// Measures the chip-wide throughput of the instructions a multi-limb
// Montgomery multiply can be built from; the v_mad_u64_u32 rate is the
// roofline denominator quoted in DESIGN.md and bench.py ("peak").
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 32768;

// 8 independent dependency chains per lane; each asm block issues one instruction per chain.
template <int OP>
__global__ __launch_bounds__(256) void bench_kernel(uint32_t* out, uint32_t seed) {
  uint32_t a = seed ^ threadIdx.x, b = seed * 3u + blockIdx.x;
  uint64_t acc[8];
  uint32_t acc32[8];
  double accf[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { acc[k] = a + k; acc32[k] = b + k; accf[k] = (double)(a + k); }
  double fb = (double)b * 1e-9;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (OP == 0) {  // v_mad_u64_u32
        uint64_t carry;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(carry) : "v"(a), "v"(b));
      } else if constexpr (OP == 1) {  // v_mul_lo_u32
        asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
      } else if constexpr (OP == 2) {  // v_mul_hi_u32
        asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
      } else if constexpr (OP == 3) {  // v_mad_u32_u24
        asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(acc32[k]) : "v"(a), "v"(b));
      } else if constexpr (OP == 4) {  // v_mul_hi_u32_u24
        asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
      } else if constexpr (OP == 5) {  // v_add_co_u32 + v_addc_co_u32 pair (counts 2)
        asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc32[k]) : "v"(b) : "vcc");
      } else if constexpr (OP == 6) {  // v_add3_u32
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(acc32[k]) : "v"(a), "v"(b));
      } else if constexpr (OP == 7) {  // v_fma_f64
        asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(accf[k]) : "v"(fb));
      } else if constexpr (OP == 8) {  // v_dot2_u32_u16
        asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(acc32[k]) : "v"(a), "v"(b));
      } else if constexpr (OP == 9) {  // v_dot4_u32_u8
        asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(acc32[k]) : "v"(a), "v"(b));
      } else if constexpr (OP == 10) {  // v_lshl_add_u64
        asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"(acc[(k + 1) & 7]));
      } else if constexpr (OP == 11) {  // v_mad_u64_u32 with SGPR multiplicand
        uint64_t carry;
        uint32_t s = __builtin_amdgcn_readfirstlane(b);
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(carry) : "s"(s), "v"(a));
      } else if constexpr (OP == 12) {  // v_add_u32 (full-rate reference)
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
      } else if constexpr (OP == 14) {  // v_add_co_u32_e32 alone (VCC out)
        asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(acc32[k]) : "v"(b) : "vcc");
      } else if constexpr (OP == 15) {  // v_addc_co_u32_e32 (VCC in/out)
        asm volatile("v_addc_co_u32 %0, vcc, 0, %0, vcc" : "+v"(acc32[k]) :: "vcc");
      } else if constexpr (OP == 16) {  // mad_u64 (carry->vcc) + addc into a third word: 2 insts
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc" : "+v"(acc[k]), "+v"(acc32[k]) : "v"(a), "v"(b) : "vcc");
      } else if constexpr (OP == 17) {  // v_add_u32_e64 (VOP3 encoding)
        asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
      } else if constexpr (OP == 18) {  // v_and_b32
        asm volatile("v_and_b32 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
      } else if constexpr (OP == 19) {  // v_alignbit_b32
        asm volatile("v_alignbit_b32 %0, %0, %1, 29" : "+v"(acc32[k]) : "v"(b));
      } else if constexpr (OP == 20) {  // v_lshrrev_b64
        asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc[k]));
      } else if constexpr (OP == 21) {  // v_cndmask_b32 with vcc
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(acc32[k]) : "v"(b) : "vcc");
      } else if constexpr (OP == 22) {  // v_addc_co_u32_e64 with SGPR-pair carries
        uint64_t cc;
        asm volatile("v_add_co_u32_e64 %0, %1, %0, %2\n\tv_addc_co_u32_e64 %0, %1, %0, %2, %1" : "+v"(acc32[k]), "=&s"(cc) : "v"(b));
      } else if constexpr (OP == 23) {  // v_mad_u64_u32 only, 1 dependency chain (latency)
        if (k == 0) { uint64_t carry; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[0]), "=s"(carry) : "v"(a), "v"(b)); }
      } else if constexpr (OP == 24) {  // v_mul_lo_u32 + v_and_b32 (m mod 2^r)
        asm volatile("v_mul_lo_u32 %0, %0, %1\n\tv_and_b32 %0, 0x1fffffff, %0" : "+v"(acc32[k]) : "v"(b));
      } else if constexpr (OP == 25) {  // v_mov_b32
        asm volatile("v_mov_b32 %0, %1" : "=v"(acc32[k]) : "v"(acc32[(k+1)&7]));
      } else if constexpr (OP == 13) {  // v_mov_b32 dpp wave_shr:1
        asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %0 wave_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(acc32[k]));
      }
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) r += acc[k] + acc32[k] + (uint64_t)accf[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)r ^ (uint32_t)(r >> 32);
}

template <int OP>
int run(const char* name, double insts_per_chain_step, uint32_t* d_out, int blocks, int waves_per_block) {
  int threads = waves_per_block * 64;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(bench_kernel<OP>, dim3(blocks), dim3(threads), 0, 0, d_out, 7u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(bench_kernel<OP>, dim3(blocks), dim3(threads), 0, 0, d_out, 7u + r);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double lane_insts = (double)blocks * threads * ITERS * 8 * insts_per_chain_step;
  double rate = lane_insts / (best * 1e-3);
  // full-rate reference: 256 CU * 4 SIMD * 32 lanes * clock
  printf("{\"op\": \"%s\", \"blocks\": %d, \"threads\": %d, \"ms\": %.4f, \"lane_ops_per_s\": %.4e}\n",
         name, blocks, threads, best, rate);
  CHECK(hipEventDestroy(e0)); CHECK(hipEventDestroy(e1));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  uint32_t* d_out;
  int blocks = p.multiProcessorCount * 8;
  CHECK(hipMalloc(&d_out, sizeof(uint32_t) * blocks * 1024));
  for (int wpb : {4, 2, 1}) {
    int b = (wpb == 4) ? blocks : p.multiProcessorCount * 4;  // wpb<4: few waves per SIMD
    if (wpb == 2) b = p.multiProcessorCount * 8;
    run<0>("v_mad_u64_u32", 1, d_out, b, wpb);
    run<11>("v_mad_u64_u32_sgpr", 1, d_out, b, wpb);
    run<16>("mad_u64+addc_e32 (2 insts)", 2, d_out, b, wpb);
    run<1>("v_mul_lo_u32", 1, d_out, b, wpb);
    run<2>("v_mul_hi_u32", 1, d_out, b, wpb);
    run<3>("v_mad_u32_u24", 1, d_out, b, wpb);
    run<14>("v_add_co_u32_e32", 1, d_out, b, wpb);
    run<15>("v_addc_co_u32_e32", 1, d_out, b, wpb);
    run<22>("add_co+addc_e64 sgpr carry (2)", 2, d_out, b, wpb);
    run<5>("v_add_co+addc_e32 (2)", 2, d_out, b, wpb);
    run<6>("v_add3_u32", 1, d_out, b, wpb);
    run<12>("v_add_u32_e32", 1, d_out, b, wpb);
    run<17>("v_add_u32_e64", 1, d_out, b, wpb);
    run<18>("v_and_b32", 1, d_out, b, wpb);
    run<19>("v_alignbit_b32", 1, d_out, b, wpb);
    run<20>("v_lshrrev_b64", 1, d_out, b, wpb);
    run<21>("v_cndmask_b32_vcc", 1, d_out, b, wpb);
    run<25>("v_mov_b32", 1, d_out, b, wpb);
    run<24>("mul_lo+and (2)", 2, d_out, b, wpb);
    run<7>("v_fma_f64", 1, d_out, b, wpb);
    run<10>("v_lshl_add_u64", 1, d_out, b, wpb);
    run<13>("v_mov_dpp_wave_shr(+s_nop1) (2)", 2, d_out, b, wpb);
    run<23>("v_mad_u64_u32 1-chain (x1/8)", 0.125, d_out, b, wpb);
  }
  CHECK(hipFree(d_out));
  return 0;
}
