// mdfit_host.h — host-side helpers shared by the translation units of
// libmdfit.so (mdfit.hip: C-ABI + MAP kernels, mdfit_nuts.hip: sampling mode).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/mdfit.h"

namespace mdfit {
constexpr int kWave = 64;
constexpr int kQueues = 8;  // one work queue per XCD (blockIdx % 8 share an XCD)
}  // namespace mdfit

namespace mdfit::host {
extern thread_local char g_err[512];
// record an argument / launch error for mdfit_last_error(); returns code
int set_err(int code, const char* msg);
// hipGetLastError after a launch -> 0 or the hipError_t (message recorded)
int check_launch(const char* what);

// optional HIP-event timing (mdfit_profile_enable): slot 1 / 2 bracket the
// dominant kernel of the call
void prof_mark(int slot, hipStream_t s);

// persistent grid: no more waves than can be resident at once (so every
// wave starts immediately and pulls work until its queue is drained), a
// multiple of the 8 queues
// (cap_per_cu > 0: at most that many waves per CU; force_per_cu > 0: exactly
// that many -- development A/B; MDFIT_DEV_GRID prints the sizing)
template <typename K>
int64_t fit_grid(K kernel, int64_t ntask, int fits_per_wave, int cap_per_cu = 0, int force_per_cu = 0) {
  int dev = 0, n_cu = 256, per_cu = 8;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0)
    n_cu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kWave, 0) != hipSuccess || per_cu <= 0)
    per_cu = 8;
  if (cap_per_cu > 0 && cap_per_cu < per_cu) per_cu = cap_per_cu;
  const int api = per_cu;
  if (force_per_cu > 0) per_cu = force_per_cu;
  const int64_t want = (ntask + fits_per_wave - 1) / fits_per_wave;
  const int64_t cap = (int64_t)n_cu * per_cu;
  int64_t g = want < cap ? want : cap;
  g = ((g + kQueues - 1) / kQueues) * kQueues;
  if (std::getenv("MDFIT_DEV_GRID")) {
    hipFuncAttributes fa{};
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kernel));
    int lds_cu = 0;
    (void)hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
    std::fprintf(stderr, "fit_grid: n_cu %d occupancy-api %d per_cu %d lds/block %zu regs %d lds/cu %d -> grid %lld\n",
                 n_cu, api, per_cu, fa.sharedSizeBytes, fa.numRegs, lds_cu, (long long)g);
  }
  return g < kQueues ? kQueues : g;
}
}  // namespace mdfit::host

namespace mdfit::host {
// MDFIT_DEBUG_POISON_LDS=1 (tests): NaN into every CU's LDS on stream s
// (mdfit_poison_lds) -- called before each LDS-using kernel of a call
void debug_poison(hipStream_t s);
}  // namespace mdfit::host

namespace mdfit::nuts {
// sampling mode (mdfit_nuts.hip): workspace = 256 B of queue counters, then
// the chains' samples double[T][6][num_samples][4] = (q, A, c, phi)
constexpr int64_t kSamplesOffset = 256;
int64_t workspace_bytes(int64_t n_taxa, int num_samples);
// register-only throughput probe of the chain kernel's potential evaluation
int peak_probe(int64_t n_waves, int iters, double* sink, hipStream_t s);
int potential(const int32_t* model, const int32_t* subset, const uint32_t* y, const uint32_t* N, const double* v,
              int64_t n, double* U, double* g, hipStream_t s);
// launches the chain and post-processing kernels (workspace already zeroed)
int fit_batch(const uint32_t* y, const uint32_t* N, const uint32_t* mm, int64_t n_taxa, const mdfit_opts& o,
              double* out, float* pred, int32_t* status, void* workspace, hipStream_t s);
}  // namespace mdfit::nuts
