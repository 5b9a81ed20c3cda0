// Dependent-issue latency of the instructions on a Montgomery row's critical
// path (gfx950): one wave, one dependency chain, cycles per link from
// s_memtime.  The row chain of Mont29::row (mont29.hpp) is
//   m = bcast(col0) & M29  ->  col0 += m * n0  ->  col1 += col0 >> 29  ->  next m
// and variants that take the 64-bit carry off that path.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(64) void lat_kernel(uint64_t* out, uint32_t seed) {
  uint32_t x = seed ^ threadIdx.x, n0 = seed * 7u + 1u, m29 = (1u << 29) - 1;
  uint64_t acc = x, acc1 = x + 3u;
  asm volatile("" : "+v"(x), "+v"(n0), "+v"(m29), "+v"(acc), "+v"(acc1));
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0) {   // v_mad_u64_u32 -> itself
      uint64_t c;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(n0), "v"(m29));
    } else if constexpr (OP == 1) {   // v_lshrrev_b64 -> itself
      asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(acc));
    } else if constexpr (OP == 2) {   // v_lshl_add_u64 -> itself
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc) : "v"(acc1));
    } else if constexpr (OP == 3) {   // v_add_u32 -> itself
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(n0));
    } else if constexpr (OP == 4) {   // v_and_b32_dpp row_newbcast:0 -> itself (+ the s_nop 1 DPP hazard)
      asm volatile("s_nop 1\n\tv_and_b32_dpp %0, %0, %1 row_newbcast:0 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                   : "+v"(x) : "v"(m29));
    } else if constexpr (OP == 5) {   // v_alignbit_b32 -> itself
      asm volatile("v_alignbit_b32 %0, %0, %1, 29" : "+v"(x) : "v"(n0));
    } else if constexpr (OP == 6) {   // the row chain today: dpp-and -> mad -> lshr64 -> lshl_add64
      uint64_t c;
      uint32_t m;
      asm volatile(
          "s_nop 1\n\t"
          "v_and_b32_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf bound_ctrl:1"
          : "=&v"(m) : "v"((uint32_t)acc), "v"(m29));
      asm volatile(
          "v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
          "v_lshrrev_b64 %0, 29, %0\n\t"
          "v_lshl_add_u64 %0, %1, 0, %0"
          : "+v"(acc), "+v"(acc1), "=s"(c) : "v"(m), "v"(n0));
    } else if constexpr (OP == 7) {   // carry off the path: dpp-and -> mad -> alignbit -> add_u32
      uint64_t c;
      uint32_t m;
      asm volatile(
          "s_nop 1\n\t"
          "v_and_b32_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf bound_ctrl:1"
          : "=&v"(m) : "v"(x), "v"(m29));
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(m), "v"(n0));
      x = (uint32_t)(acc >> 29) + n0;   // v_alignbit_b32 + v_add_u32
    } else if constexpr (OP == 8) {   // dpp-and -> mad (the quotient's use)
      uint64_t c;
      uint32_t m;
      asm volatile(
          "s_nop 1\n\t"
          "v_and_b32_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf bound_ctrl:1"
          : "=&v"(m) : "v"((uint32_t)acc), "v"(m29));
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(c) : "v"(m), "v"(n0));
    } else if constexpr (OP == 9) {   // v_mov_b32_dpp row_ror:15 -> itself
      asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %0 row_ror:15 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x));
    } else if constexpr (OP == 10) {   // s_nop 1 alone (the DPP hazard padding)
      asm volatile("s_nop 1" ::: "memory");
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (threadIdx.x == 1) out[1] = acc + x + acc1;
}

int main() {
  uint64_t* d;
  CHECK(hipMalloc(&d, 64));
  const char* names[] = {"v_mad_u64_u32", "v_lshrrev_b64", "v_lshl_add_u64", "v_add_u32", "s_nop1+v_and_b32_dpp newbcast",
                         "v_alignbit_b32", "row chain today (nop,dpp,mad,lshr64,lshl_add64)",
                         "row chain 32-bit carry (nop,dpp,mad,alignbit)", "nop,dpp-and -> mad",
                         "s_nop1+v_mov_dpp row_ror", "s_nop 1"};
  // s_memtime counts at the shader clock on gfx9 (the reference clock on some parts): the
  // s_nop 1 line (2 cycles per link by definition) calibrates
  for (int op = 0; op <= 10; ++op) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (op) {
#define L(k) case k: hipLaunchKernelGGL(lat_kernel<k>, dim3(1), dim3(64), 0, 0, d, 12345u); break;
        L(0) L(1) L(2) L(3) L(4) L(5) L(6) L(7) L(8) L(9) L(10)
#undef L
      }
      CHECK(hipDeviceSynchronize());
    }
    uint64_t h[2];
    CHECK(hipMemcpy(h, d, 16, hipMemcpyDeviceToHost));
    printf("{\"op\": \"%s\", \"ticks_per_link\": %.2f}\n", names[op], (double)h[0] / ITERS);
  }
  return 0;
}
