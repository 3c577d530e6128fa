// Development check: mdfit::xrow (v_permlane16_swap) returns the value of
// the lane 16 away in its 32-lane row pair (lane ^ 16), bit for bit.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/micro/xrow_check.hip -o tools/micro/xrow_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../metadamage_amd/csrc/mdfit_model.h"

__global__ void k(int* bad) {
  const int l = threadIdx.x;
  const double v = 1.0 / (3.0 + l) + 1e-300 * l;
  const double w = mdfit::xrow(v);
  const double want = 1.0 / (3.0 + (l ^ 16)) + 1e-300 * (l ^ 16);
  if (__double_as_longlong(w) != __double_as_longlong(want)) atomicAdd(bad, 1);
}

int main() {
  int* b;
  (void)hipMalloc(&b, 4);
  (void)hipMemset(b, 0, 4);
  k<<<4, 64>>>(b);
  int h = -1;
  (void)hipMemcpy(&h, b, 4, hipMemcpyDeviceToHost);
  printf("xrow: %d of 256 lanes wrong\n", h);
  return h != 0;
}
