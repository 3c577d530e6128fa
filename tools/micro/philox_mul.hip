// Micro-benchmark (development): cost of the Philox4x32 round's two 32x32->64
// products as v_mul_hi_u32 + v_mul_lo_u32 pairs vs one v_mad_u64_u32 each,
// 64 waves per CU, FP64-free.  hipcc --offload-arch=gfx950 -O3 philox_mul.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <bool kMad>
__global__ __launch_bounds__(64) void k(uint32_t* o, int iters) {
  uint32_t c0 = threadIdx.x + 7u * blockIdx.x, c1 = c0 ^ 0x1234u, c2 = c0 * 3u, c3 = c0 + 99u, k0 = 11u, k1 = 13u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      uint32_t hi0, lo0, hi1, lo1;
      if (kMad) {
        uint64_t p0, p1;
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p0) : "v"(c0), "s"(0xD2511F53u) : "vcc");
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p1) : "v"(c2), "s"(0xCD9E8D57u) : "vcc");
        hi0 = (uint32_t)(p0 >> 32); lo0 = (uint32_t)p0; hi1 = (uint32_t)(p1 >> 32); lo1 = (uint32_t)p1;
      } else {
        hi0 = __umulhi(0xD2511F53u, c0); lo0 = 0xD2511F53u * c0;
        hi1 = __umulhi(0xCD9E8D57u, c2); lo1 = 0xCD9E8D57u * c2;
        asm volatile("" : "+v"(hi0), "+v"(lo0), "+v"(hi1), "+v"(lo1));
      }
      const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
      c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
      k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
  }
  o[blockIdx.x * 64 + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3;
}

int main() {
  const int blocks = 256 * 16, iters = 2000;
  uint32_t* o;
  (void)hipMalloc(&o, blocks * 64 * 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < 2; ++v) {
      (void)hipEventRecord(a);
      if (v) k<true><<<blocks, 64>>>(o, iters);
      else k<false><<<blocks, 64>>>(o, iters);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, a, b);
      const double rounds = (double)blocks * 64 * iters * 10;
      printf("%s %.3f ms  %.3f ns per wave-round per CU\n", v ? "mad_u64" : "mul_hi+lo", ms, ms * 1e6 / (rounds / 64 / 256));
    }
  return 0;
}
