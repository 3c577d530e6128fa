// Development check: newton_dir<G> (lane-parallel shift search) against the
// sequential form it replaced, bit for bit, on random (mostly indefinite)
// 4x4 systems replicated over G-lane groups.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/newton_check.hip -o tools/micro/newton_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../metadamage_amd/csrc/mdfit_model.h"
namespace mdfit {
#include "old_nd.h"
}
using namespace mdfit;

__device__ double rnd(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (double)(s >> 11) * 0x1.0p-53 * 2.0 - 1.0;
}

template <int G>
__global__ void k(int n, unsigned long long* bad, unsigned long long* tot) {
  const int grp = (blockIdx.x * 64 + threadIdx.x) / G;
  if (grp >= n) return;
  uint64_t s = 0x9E3779B97F4A7C15ull * (grp + 1);
  double H[10], g[4], u[4];
  for (int j = 0; j < 10; ++j) H[j] = rnd(s) * pow(10.0, 4.0 * rnd(s));
  for (int j = 0; j < 4; ++j) { g[j] = rnd(s) * 10.0; u[j] = rnd(s) * 3.0; }
  const bool pmd = rnd(s) > -0.8;
  const bool nc = rnd(s) > 0.7;
  double d1[4], d2[4];
  const bool i1 = newton_dir<G>(pmd, u, g, H, 1.0, d1, nc);
  const bool i2 = G == 16 ? newton_dir<8>(pmd, u, g, H, 1.0, d2, nc) : newton_dir_old(pmd, u, g, H, 1.0, d2, nc);
  bool same = i1 == i2;
  for (int j = 0; j < 4; ++j) same = same && (__double_as_longlong(d1[j]) == __double_as_longlong(d2[j]));
  int astar = -1;
  {
    bool fr[4]; double dbind[4], L[10], iL[4];
    free_set(pmd, u, g, H, 1.0, fr, dbind);
    if (chol4(fr, H, 0.0, L, iL) < 0) astar = 0;
    else {
      double sc = 0.0;
      for (int j = 0; j < 4; ++j) if (fr[j]) sc = fmax(sc, fabs(H[hidx(j, j)]));
      if (sc == 0.0) sc = 1.0;
      double mu = 1e-10 * sc;
      for (int a = 1; a < 40; ++a, mu *= 10.0) if (chol4(fr, H, opaque(mu), L, iL) < 0) { astar = a; break; }
    }
  }
  if (!same) atomicAdd(&bad[1 + (astar < 0 ? 0 : (astar > 30 ? 30 : astar))], 1ull);
  if (!same) {
    if (atomicAdd(bad, 1ull) == 0ull) {
      printf("G=%d grp %d lane %d pmd %d nc %d i1 %d i2 %d\n", G, grp, (int)threadIdx.x, (int)pmd, (int)nc, (int)i1, (int)i2);
      printf(" H %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", H[0],H[1],H[2],H[3],H[4],H[5],H[6],H[7],H[8],H[9]);
      printf(" g %.17g %.17g %.17g %.17g u %.17g %.17g %.17g %.17g\n", g[0],g[1],g[2],g[3],u[0],u[1],u[2],u[3]);
      printf(" d1 %.17g %.17g %.17g %.17g\n d2 %.17g %.17g %.17g %.17g\n", d1[0],d1[1],d1[2],d1[3],d2[0],d2[1],d2[2],d2[3]);
    }
  }
  atomicAdd(tot, 1ull);
}

int main() {
  unsigned long long *b, *t;
  (void)hipMalloc(&b, 8 * 32);
  (void)hipMalloc(&t, 8);
  for (int G : {8, 16}) {
    (void)hipMemset(b, 0, 8 * 32);
    (void)hipMemset(t, 0, 8);
    const int n = 1 << 16;
    if (G == 8) k<8><<<n * 8 / 64, 64>>>(n, b, t);
    else k<16><<<n * 16 / 64, 64>>>(n, b, t);
    unsigned long long hb, ht;
    (void)hipMemcpy(&hb, b, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&ht, t, 8, hipMemcpyDeviceToHost);
    printf("G=%d (%s): %llu of %llu lanes differ\n", G, G == 16 ? "vs newton_dir<8>" : "vs the sequential form", hb, ht);
    unsigned long long hh[32];
    (void)hipMemcpy(hh, b, 8 * 32, hipMemcpyDeviceToHost);
    printf("  by first successful attempt:");
    for (int a = 0; a < 31; ++a) if (hh[1 + a]) printf(" %d:%llu", a - 0, hh[1 + a]);
    printf("\n");
  }
  return 0;
}
