// Micro-benchmark (development): the latency of the fit kernel's per-trip
// pieces for ONE wave alone on its SIMD (the regime of C2's critical chain):
// cycles per iteration (s_memtime) of make_theta, the point evaluation
// (point_accum<true>: 5 lg3 + the contributions), one lg3, and newton_dir.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/fit_latency.hip -o tools/micro/fit_latency
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../metadamage_amd/csrc/mdfit_model.h"
using namespace mdfit;

template <int V>
__global__ __launch_bounds__(64) void k(double* o, unsigned long long* cyc, int iters, double y0, double N0, int rt_pmd, int rt_accf) {
  const int lane = threadIdx.x;
  double u[4] = {-1.0 + 1e-3 * lane, -2.0, 0.01, 5.0};
  PointData pd;
  pd.y = (lane & 15) < 15 ? y0 + lane : 0.0;
  pd.N = (lane & 15) < 15 ? N0 + 7 * lane : 0.0;
  pd.k = (lane & 15) < 15 ? (lane & 15) : 0;
  pd.valid = (lane & 15) < 15;
  pd.pmd = V >= 7 ? rt_pmd : 1;
  double sink = 0.0;
  Theta th = make_theta<16>(true, u);
  double H[10] = {4, 0.1, 0.2, 0.3, 5, 0.1, 0.2, 6, 0.3, 7};
  double g[4] = {0.1, -0.2, 0.3, -0.4};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (V == 0) {
      th = make_theta<16>(true, u);
      u[0] += th.q * 1e-300;
    } else if (V == 1) {
      double acc[kNAcc];
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) acc[j] = 0.0;
      point_accum<true>(pd, th, acc, 0);
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) s += acc[j];
      th.phi += s * 1e-300;
    } else if (V == 2) {
      th = make_theta<16>(true, u);
      double acc[kNAcc];
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) acc[j] = 0.0;
      point_accum<true>(pd, th, acc, 0);
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) s += acc[j];
      u[0] += s * 1e-300;
    } else if (V == 7) {
      th = make_theta<16>(pd.pmd, u);
      double acc[kNAcc];
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) acc[j] = 0.0;
      point_accum<true>(pd, th, acc, rt_accf);
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) s += acc[j];
      u[0] += s * 1e-300;
    } else if (V == 3) {
      const LG3 r = lg3<true, false>(pd.y + th.phi);
      th.phi += (r.l + r.p + r.q) * 1e-300;
    } else if (V == 4) {
      const LG3 r = lg3<true, false>(0.37 + th.phi * 1e-3);  // the shifted branch (x < 10)
      th.phi += (r.l + r.p + r.q) * 1e-300;
    } else if (V == 5) {
      double d[4];
      newton_dir<16>(true, u, g, H, 1.0, d, false);
      g[0] += d[0] * 1e-300;
    } else if (V == 6) {
      Eval e;
      double acc[kNAcc];
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) acc[j] = 1.0 + j + 1e-3 * lane;
      acc[6] = -50; acc[10] = -60; acc[13] = -70; acc[15] = -80;
      acc[0] += sink * 1e-300;
      finish_eval(true, th, acc, e);
      const double pg = pgnorm(u, e.g);
      double d[4];
      newton_dir<16>(true, u, e.g, e.H, pg, d, false);
      sink += d[0] + d[3];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  o[blockIdx.x * 64 + lane] = u[0] + th.phi + g[0] + sink;
  if (lane == 0) cyc[blockIdx.x] = (t1 - t0) / iters;
}

int main() {
  double* o;
  unsigned long long* c;
  (void)hipMalloc(&o, 1024 * 64 * 8);
  (void)hipMalloc(&c, 1024 * 8);
  const char* names[8] = {"make_theta", "point_accum (5 lg3 + contrib)", "make_theta + point_accum", "lg3 unshifted",
                          "lg3 shifted", "newton_dir (PD)", "finish_eval + pgnorm + newton_dir", "eval, runtime pmd / accf (0)"};
  for (int y0 = 0; y0 < 2; ++y0) {
    const double yy = y0 ? 500.0 : 3.0, NN = y0 ? 1e5 : 20.0;
    for (int v = 0; v < 8; ++v) {
      for (int blocks : {1, 1024}) {
        switch (v) {
          case 0: k<0><<<blocks, 64>>>(o, c, 200, yy, NN, 1, 0); break;
          case 1: k<1><<<blocks, 64>>>(o, c, 200, yy, NN, 1, 0); break;
          case 2: k<2><<<blocks, 64>>>(o, c, 200, yy, NN, 1, 0); break;
          case 3: k<3><<<blocks, 64>>>(o, c, 200, yy, NN, 1, 0); break;
          case 4: k<4><<<blocks, 64>>>(o, c, 200, yy, NN, 1, 0); break;
          case 5: k<5><<<blocks, 64>>>(o, c, 200, yy, NN, 1, 0); break;
          case 6: k<6><<<blocks, 64>>>(o, c, 200, yy, NN, 1, 0); break;
          case 7: k<7><<<blocks, 64>>>(o, c, 200, yy, NN, 1, 0); break;
        }
        unsigned long long h[1024];
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, c, blocks * 8, hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < blocks; ++i) m += (double)h[i];
        printf("%-36s y=%5.0f N=%7.0f blocks %4d: %8.0f cycles/iter\n", names[v], yy, NN, blocks, m / blocks);
      }
    }
  }
  return 0;
}
