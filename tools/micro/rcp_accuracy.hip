// Accuracy of v_rcp_f64 (__builtin_amdgcn_rcp on double) with 0, 1, 2 Newton
// steps against the correctly rounded 1/x (IEEE division), in ulps of the
// result, over log-uniform x in [2^-20, 2^40] (development probe: how many
// Newton steps mdfit_special.h's rcp needs).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/rcp_accuracy.hip -o tools/micro/rcp_accuracy
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>

__device__ double ulps(double a, double b) {
  const double u = fabs(b) * 2.220446049250313e-16;
  return fabs(a - b) / u;
}

__global__ void probe(int64_t n, double* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double m0 = 0, m1 = 0, m2 = 0;
  for (int64_t k = i; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    // log-uniform x from a hash of k
    uint64_t h = (uint64_t)k * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    const double u = (double)(h >> 11) * 0x1.0p-53;
    const double x = exp2(-20.0 + 60.0 * u);
    const double ex = 1.0 / x;
    double r = __builtin_amdgcn_rcp(x);
    m0 = fmax(m0, ulps(r, ex));
    r = fma(fma(-x, r, 1.0), r, r);
    m1 = fmax(m1, ulps(r, ex));
    r = fma(fma(-x, r, 1.0), r, r);
    m2 = fmax(m2, ulps(r, ex));
  }
  out[3 * i + 0] = m0;
  out[3 * i + 1] = m1;
  out[3 * i + 2] = m2;
}

int main() {
  const int blocks = 1024, threads = 256;
  const int64_t n = 1ll << 28;
  double* d;
  hipMalloc(&d, sizeof(double) * 3 * blocks * threads);
  hipLaunchKernelGGL(probe, dim3(blocks), dim3(threads), 0, 0, n, d);
  static double h[3 * 1024 * 256];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  double m[3] = {0, 0, 0};
  for (int i = 0; i < blocks * threads; ++i)
    for (int j = 0; j < 3; ++j) m[j] = fmax(m[j], h[3 * i + j]);
  printf("{\"samples\": %lld, \"max_ulp_rcp\": %.4g, \"max_ulp_1_newton\": %.4g, \"max_ulp_2_newton\": %.4g}\n",
         (long long)n, m[0], m[1], m[2]);
  return 0;
}
