// mdfit.hip — MI355X (gfx950) batched per-TaxID damage fit + C-ABI (include/mdfit.h).
//
// Replaces the per-taxon NUTS loop of /root/reference/metadamage/fits.py
// (compute_fits :709-730 -> fit_single_group_without_timeout :428-469) with
// four stream-ordered launches over a dense count tensor (MDFIT-MAP v1,
// DESIGN.md §3-4):
//
//   K0 init_kernel     the data-driven initial point of all 6T sub-fits
//   K1 fit_kernel      persistent: first the 2T all-position sub-fits
//                      (model_PMD / model_null, fits.py:438-439), then the 4T
//                      forward / reverse ones (fits.py:311-313, 333-335),
//                      warm-started at the all-position modes
//   K3 assemble_kernel one wave per taxon: pointwise log-likelihoods at
//                              the 6 modes, n_sigma x3, asymmetry, predictive
//                              medians, sums, noise (fits.py:230-376)
//   K4 hpdi_kernel     one lane per (taxon, position): the 68 % predictive
//                      HPDI of the PMD-all mode (MDFIT-HPDI v2, mdfit_hpdi.h;
//                      fits.py:112-120, 260-261)
//
// K1 work decomposition (details at fit_kernel): lane = position; a "slot"
// (32 lanes at 1 point per lane, 16 at 2) runs either one all-position
// sub-fit (both halves hold identical Newton state) or the forward / reverse
// pair of one model (each half its own Newton state machine).  Per trip every
// running fit evaluates value + gradient + Hessian at its trial point (then a
// DPP butterfly) and runs its Newton logic.  Free slots pull all-position
// tasks from 8 per-XCD queues (one atomic per wave-trip) and continue in
// place with the task's fwd/rev pair, warm-started at the all-position mode.
// (Claiming one task ahead to hide the atomic + load latency was measured
// slower: the last tasks then queue behind long fits while other slots sit
// idle.)  Everything is FP64 (the reference enables x64, fits.py:32).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "../../include/mdfit.h"
#include "mdfit_hpdi.h"
#include "mdfit_host.h"
#include "mdfit_model.h"
#include "mdfit_special.h"

#ifdef MDFIT_DEV_HPTIME
// development: clock stamps of the MAP call's HPDI hand-off (tools/_hptime.py):
// [0, T) PMD-all mode published, [T, 2T) the taxon's pair done, then per item
// taken and written (T * 30 each)
__device__ unsigned long long* g_dev_hpt = nullptr;
#define MDFIT_DEV_T(idx) \
  do {                     \
    if (g_dev_hpt != nullptr) g_dev_hpt[(idx)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#endif

namespace mdfit {

constexpr int kAll = 0, kFR = 1;

// diag slots of the out record (include/mdfit.h): during K1 slots 0..3 of a
// sub-fit hold its unconstrained mode u*, K3 turns them into (q, A, c, phi)
__device__ __forceinline__ double* diag(double* out, int64_t taxon, int sub) {
  return out + taxon * MDFIT_NOUT + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * sub;
}

// v[j] for a lane-varying j in 0..3 without dynamic register indexing
__device__ __forceinline__ double sel4(const double v[4], int j) {
  return j == 0 ? v[0] : (j == 1 ? v[1] : (j == 2 ? v[2] : v[3]));
}

#ifdef MDFIT_STAMP
// diagnostic build (-DMDFIT_STAMP): per-wave cycle split of the fit loop.
// Never quote this build's run time; read its shares (cdna_hip_programming.md §7).
__device__ unsigned long long* g_stamp = nullptr;
__device__ __forceinline__ unsigned long long stamp() {
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif

// MAP workspace, int32 words of the 256-byte header (zeroed by K0):
//   [0, 8) the per-XCD all-position task counters (fit_kernel)
//   [8]    ready-list length (fit_kernel appends a PMD-all mode per taxon)
//   [9]    hpdi_stream_kernel's item claim counter
//   [10]   "fit_kernel has started" (hpdi_stream_kernel waits on the list only then)
//   [16, 19) the wide-window list counters of K4a/K4b (the array entry point)
// then the ready list: uint64[T][kReadyStride] = ~bits of (q, A, c, phi,
// taxon), a spare word; zeroed by K0 every call (so no entry of an earlier
// call or of whatever the buffer held before can pass for a published one: a
// field is non-zero only once this call's fit kernel has written it)
//   [11]   corrupt ready entries met by hpdi_stream_kernel (0; a diagnostic)
//   [32, 36) the defer list's counters (see hpdi_stream_kernel); the list
//          itself (int32 items, kDeferCap at most) ends the workspace
constexpr int kWsReady = 8, kWsClaim = 9, kWsStarted = 10, kWsBad = 11;
// [12] the claim counter as the late launch found it (a diagnostic: the HPDI
// items the early launch took while the fit ran, tests/test_gpu_paths.py)
constexpr int kWsEarlyClaimed = 12;
// the HPDI stream's defer list (hpdi_stream_kernel), on a 128-B line of their
// own (away from the counters the fit kernel's atomics hit): [32] reservations
// (+ kDefClosed once the late launch has closed it), [33] slots written, [34]
// the late launch's claim counter over them, [35] an early wave has deferred
// (the others stop too)
constexpr int kWsDefRes = 32, kWsDefDone = 33, kWsDefClaim = 34, kWsEarlyQuit = 35;
constexpr unsigned kDefClosed = 0x40000000u;
constexpr int kReadyStride = 6;
static_assert(kReadyStride == MDFIT_NSUBFIT, "K0 zeroes the ready list with one thread per (taxon, sub-fit)");
// a ready-list field holds the bit complement of its value: zero = not yet
// written this call (a double's complement is zero only for the all-ones NaN
// pattern, which ready_put canonicalises away; a taxon index's only for -1)
__device__ __forceinline__ void ready_put(uint64_t* f, double v) {
  __hip_atomic_store(f, ~(uint64_t)__double_as_longlong(isnan(v) ? NAN : v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ready_get(const uint64_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kHpdiCtr = 16;  // workspace ints: [16] front-list count, [17] claim counter, [18] back-list count

// ---------------------------------------------------------------------------
// K0: initial points (oracle: init_u)
// ---------------------------------------------------------------------------
// |z|-1 of all-position column i (0..14 forward, 15..29 reverse)
__device__ __forceinline__ int kpos(int i) { return i < kNHalf ? i : i - kNHalf; }

// One thread per (taxon, sub-fit): pooled ratios over the sub-fit's positions
// -> u0 in diag slots 0..3 (K1 / K2 start there; K1 replaces the fwd/rev u0
// by its own mode when it converged -- the warm start).
__global__ __launch_bounds__(256) void init_kernel(const uint32_t* __restrict__ gy,
                                                   const uint32_t* __restrict__ gN, int64_t T,
                                                   double* __restrict__ out, int* __restrict__ ws) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the fit kernel's queue counters (workspace, 256 B): zeroed here instead of
  // by a separate memset launch (stream order puts this before the fit kernel)
  // and the ready list (one double per thread: 6 T of each)
  if (i < 64) ws[i] = 0;
  if (i < MDFIT_NSUBFIT * T) reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + 256)[i] = 0.0;
  if (i >= MDFIT_NSUBFIT * T) return;
  const int64_t taxon = i / MDFIT_NSUBFIT;
  const int sub = (int)(i % MDFIT_NSUBFIT);  // 0 PMD-all 1 null-all 2 PMD-f 3 PMD-r 4 null-f 5 null-r
  const bool pmd = sub == 0 || sub == 2 || sub == 3;
  const int lo = (sub == 3 || sub == 5) ? kNHalf : 0;
  const int hi = sub < 2 ? kNPos : lo + kNHalf;
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // y,N over all, |z|=1, |z|=2, |z|>=10
  for (int c = lo; c < hi; ++c) {
    const double y = (double)gy[taxon * kLD + c], N = (double)gN[taxon * kLD + c];
    const int k = kpos(c);
    s[0] += y;
    s[1] += N;
    if (k == 0) { s[2] += y; s[3] += N; }
    if (k == 1) { s[4] += y; s[5] += N; }
    if (k >= 9) { s[6] += y; s[7] += N; }
  }
  double u0[4];
  u0[3] = flog(100.0);
  if (!pmd) {
    u0[0] = logit(clampd((s[0] + 0.5) / (s[1] + 1.0), 1e-4, 0.9));
    u0[1] = u0[2] = 0.0;
  } else {
    const double c0 = clampd((s[6] + 0.5) / (s[7] + 1.0), 1e-4, 0.3);
    const double r1 = (s[2] + 0.5) / (s[3] + 1.0);
    const double r2 = (s[4] + 0.5) / (s[5] + 1.0);
    const double A0 = clampd(r1 - c0, 1e-3, 0.9 * (1.0 - c0));
    double q0 = 1.0 / 3.0;
    if (r1 - c0 > 1e-3) q0 = clampd(1.0 - (r2 - c0) / (r1 - c0), 0.05, 0.95);
    u0[0] = logit(q0);
    u0[1] = logit(A0);
    u0[2] = c0;
  }
  double* dg = diag(out, taxon, sub);
#pragma unroll
  for (int j = 0; j < 4; ++j) dg[j] = u0[j];
}

// ---------------------------------------------------------------------------
// K1: the persistent fit kernel (all 6 sub-fits of every taxon)
// ---------------------------------------------------------------------------
#ifndef MDFIT_FIT_WAVES_PER_EU
#define MDFIT_FIT_WAVES_PER_EU 2
#endif

// workspace layout (int32): [0, kQueues) per-XCD all-position task counters

// slot modes
constexpr int kIdle = 0, kAllFit = 1, kPairFit = 2, kNextPair = 3;
constexpr int kPrioEvals = 15;  // fit length (evaluations) that raises the wave priority

// Lane layouts (PPL = points per lane), bitwise-identical results:
//  PPL 1: a "slot" = a 32-lane group = 2 rows of 16 (lane = position; row 0
//         z = 1..15, row 1 z = -1..-15, lane 15 of a row a pad); a pair's
//         halves are the two rows.  2 slots per wave.
//  PPL 2: a slot = one 16-lane row.  All-position fit: lane i < 15 holds
//         z = +(i+1) and z = -(i+1), lane 15 two pads; pair: each 8-lane half
//         runs one 15-point sub-fit, lane j holding |z| - 1 = 2j, 2j + 1 (lane
//         7 of a half: 14 and a pad).  4 slots per wave: the Newton logic,
//         sums and task fetch are shared by twice the points.
// Sums: every lane first adds its slot partner's point (PPL 1 all-position:
// the other row, xor 16; PPL 2: its own second point), then one butterfly
// over the positions in the same tree order, so both layouts give the same
// bits (and the same fits).
//
// Work: a free slot claims an all-position task (taxon, model) from its
// XCD's queue (PMD tasks first: the long ones), fits it, then continues in
// place with the forward / reverse pair of the same taxon and model, warm-
// started at the all-position mode (still in registers; the counts too --
// PPL 2 re-deals them to the pair layout with lane shuffles), so a pair costs
// no memory round trip and no hand-off between waves.
// line-search state bits (fit_kernel): the saddle escape's H indefinite at the
// current point, re-evaluation pending, escape line search running,
// exhaustion status OK, the escape count (kEscCount, in units of kEscN: at
// most 4); the flat-tail rescue done / its relaxed acceptance pending
// the polish phase: F in the cancellation-free form from here on / its
// re-evaluation at u pending
// the gradient fallback: its line search running / its re-evaluation at u
// pending, and its count (kEscGradCount, in units of kEscGradN: at most 8)
constexpr unsigned kEscIndef = 1u, kEscProbe = 2u, kEscNc = 4u, kEscExhOk = 8u, kEscN = 16u, kEscCount = 0x70u,
                   kEscRescued = 0x100u, kEscRelax = 0x200u, kEscPolish = 0x400u, kEscPolishProbe = 0x800u,
                   kEscGrad = 0x1000u, kEscGradProbe = 0x2000u, kEscGradN = 0x4000u, kEscGradCount = 0x3C000u;

// ---------------------------------------------------------------------------
// The predictive HPDI's per-position step (K4a, and the fused prep of the PPL-1
// fit kernel): shared definitions
// ---------------------------------------------------------------------------

struct HpdiIO {
  // kFit
  const uint32_t* gN;
  const double* ready;  // the ready list of PMD-all modes (fit_kernel; complete when K4a runs)
  double* out;
  float* pred;
  int per;  // positions per taxon written (30, or 1 without pred)
  // arrays
  const double *N, *a, *b;
  double *lo, *hi;
};

template <bool kFit>
__device__ __forceinline__ void hpdi_write(const HpdiIO& io, int64_t item, double N, double lo, double hi) {
  if (kFit) {
    const int64_t t = item / io.per;
    const int i = (int)(item - t * io.per);
    const double fl = N > 0.0 ? lo / N : NAN, fh = N > 0.0 ? hi / N : NAN;
    if (io.pred != nullptr) {
      io.pred[t * (MDFIT_NPRED * kNPos) + 1 * kNPos + i] = (float)fl;
      io.pred[t * (MDFIT_NPRED * kNPos) + 2 * kNPos + i] = (float)fh;
    }
    if (i == 0) {
      io.out[t * MDFIT_NOUT + MDFIT_F_D_MAX_LOWER_HPDI] = fl;
      io.out[t * MDFIT_NOUT + MDFIT_F_D_MAX_UPPER_HPDI] = fh;
    }
  } else {
    io.lo[item] = lo;
    io.hi[item] = hi;
  }
}

// the position's window (greedy, written here) or its wide record, appended to
// the two-list buffer that K4b drains longest-first: windows whose mode lies
// within 1.5 tau of a support end (log-variable panels, support-end walks,
// one-sided windows: ~2.5 level iterations) from the front (count ctr[0]), the
// clean two-sided ones (~1.45) from the back (count ctr[2]).  Block-collective
// (kPrepBlock threads, every thread calls): one atomic per list per block --
// per wave, the two list counters were 117k same-address atomics at 125k taxa.
#ifndef MDFIT_PREP_BLOCK
#define MDFIT_PREP_BLOCK 256
#endif
constexpr int kPrepBlock = MDFIT_PREP_BLOCK;
template <bool kFit>
__device__ __forceinline__ void hpdi_position(const HpdiIO& io, int64_t item, bool valid, bool skip, double N, double a,
                                              double b, int64_t n_items, int* __restrict__ ctr,
                                              hpdi::WideRec* __restrict__ recs) {
  constexpr int kW = kPrepBlock / kWave;
  __shared__ int s_n[2][kW];
  __shared__ int s_b[2];
  bool wide = false;
  hpdi::WideRec rec;
  if (valid) {
    double lo = NAN, hi = NAN;
    if (!skip) wide = !hpdi::prep_position(N, a, b, lo, hi, rec);
    if (!wide) hpdi_write<kFit>(io, item, N, lo, hi);
  }
  bool near = false;
  if (wide) {
    const double tau = sqrt(rec.sd * rec.sd + (rec.mu - rec.m) * (rec.mu - rec.m));
    near = rec.m < 1.5 * tau || rec.N - rec.m < 1.5 * tau;
  }
  const int w = (int)threadIdx.x / kWave, ln = (int)threadIdx.x % kWave;
  const unsigned long long mf = __ballot(wide && near), mb = __ballot(wide && !near);
  if (ln == 0) {
    s_n[0][w] = __popcll(mf);
    s_n[1][w] = __popcll(mb);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int tf = 0, tb = 0;
#pragma unroll
    for (int k = 0; k < kW; ++k) {
      tf += s_n[0][k];
      tb += s_n[1][k];
    }
    s_b[0] = tf ? atomicAdd(ctr, tf) : 0;
    s_b[1] = tb ? atomicAdd(ctr + 2, tb) : 0;
  }
  __syncthreads();
  if (wide) {
    int bf = s_b[0], bb = s_b[1];
    for (int k = 0; k < w; ++k) {
      bf += s_n[0][k];
      bb += s_n[1][k];
    }
    rec.item = item;
    const unsigned long long below = (1ull << ln) - 1ull;
    const int64_t slot = near ? (int64_t)(bf + __popcll(mf & below)) : n_items - 1 - (bb + __popcll(mb & below));
    recs[slot] = rec;
  }
}

// the butterfly's summation tree over 8 / 16 values in lane order: pairs
// (xor 1), pairs of pairs (xor 2), the two quads (half mirror), the two halves
// (mirror) -- sets, so the order inside each add does not matter
__device__ __forceinline__ double tree8(const double* x) {
  return ((x[0] + x[1]) + (x[2] + x[3])) + ((x[4] + x[5]) + (x[6] + x[7]));
}
__device__ __forceinline__ double tree16(const double* x) { return tree8(x) + tree8(x + 8); }

template <int PPL>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(MDFIT_FIT_WAVES_PER_EU)))
void fit_kernel(const uint32_t* __restrict__ gy, const uint32_t* __restrict__ gN, int64_t T,
                int max_iter, double tol, double* __restrict__ out, int* __restrict__ ws,
                double* __restrict__ ready, int base_prio) {
  static_assert(PPL == 1 || PPL == 2, "points per lane");
  constexpr int kSlot = PPL == 1 ? 32 : 16;  // lanes per slot (one all-position fit or one pair)
  constexpr int kHalf = kSlot / 2;           // lanes per fwd/rev sub-fit of a pair
  const int lane = threadIdx.x;
  const int r = lane & (kSlot - 1);  // lane in the slot
  const int h = r / kHalf;           // half: 0 forward (z > 0), 1 reverse (z < 0)
  const int jh = r & (kHalf - 1);    // lane in the half
  const int leader = lane & ~(kSlot - 1);
  const unsigned long long slot_mask = (kSlot == 32 ? 0xFFFFFFFFull : 0xFFFFull) << leader;
  const int qi = blockIdx.x % kQueues;
  // queue qi owns the taxa [tl, tl + nq): first their PMD fits (the long ones),
  // then their null fits
  const int64_t tl = T * qi / kQueues, nq = T * (qi + 1) / kQueues - tl;

  // this lane's point(s).  Columns: col c of a taxon row is z = c+1 (c < 15)
  // or z = -(c-14); |z|-1 = k.  Per mode (all / pair) the points differ for
  // PPL 2; pads carry y = N = 0.
  PointData pa, pb;
  // loop-carried per-lane flags are ints (VGPRs): as bools they would be held
  // in SGPR lane masks, which the compiler spills to VGPR lanes
  int vA_all, vA_pair, vB_all = 0, vB_pair = 0;
  int kA_all, kA_pair, kB_all = 0, kB_pair = 0, colA_all;
  if (PPL == 1) {
    const int i = r & 15;  // lane in its row = |z|-1
    vA_all = vA_pair = i < kNHalf;
    kA_all = kA_pair = vA_all ? i : 0;
    colA_all = vA_all ? h * kNHalf + i : 0;
  } else {
    vA_all = vB_all = r < kNHalf;
    kA_all = kB_all = vA_all ? r : 0;
    colA_all = vA_all ? r : 0;
    kA_pair = 2 * jh;
    kB_pair = 2 * jh + 1;
    vA_pair = true;
    vB_pair = kB_pair < kNHalf;
    kB_pair = vB_pair ? kB_pair : 0;
  }
  // PPL 2 pair layout: lane j of half h takes the counts at |z|-1 = 2j, 2j+1
  // of its direction from lanes 2j, 2j+1 of the all-position layout (point a
  // = forward, point b = reverse there)
  const int srcA = leader + (PPL == 2 ? kA_pair : 0);
  const int srcB = leader + (PPL == 2 ? (vB_pair ? kB_pair : 0) : 0);
  pa.y = pa.N = pb.y = pb.N = 0.0;
  pa.valid = vA_all;
  pa.k = kA_all;
  pb.valid = vB_all;
  pb.k = kB_all;
  pa.pmd = pb.pmd = true;

  // the sums' LDS: the lanes' terms accumulator-major (row stride padded by 2
  // doubles: a row's 16 lanes then read 16 consecutive 16-B slots, no bank
  // conflict) and the finished sums (PPL 2: one set per half)
  __shared__ __attribute__((aligned(16))) double sAcc[kNAcc][kWave + 2];
  __shared__ __attribute__((aligned(16))) double sSum[2][kWave];
  // the HPDI stream kernel running beside this one waits only once it has
  // seen this flag (no wait on a kernel that may not be running)
  if (blockIdx.x == 0 && lane == 0)
    __hip_atomic_store(ws + kWsStarted, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  int mode = kIdle;
  int drained = 0, allok = 0;
  // the sub-fit of this lane's half (replicated on its lanes; for an
  // all-position fit both halves hold identical state)
  int64_t taxon = 0;
  int sub = 0;
  int running = 0;
  double u[4] = {0, 0, 0, 0}, ut[4] = {0, 0, 0, 0}, d[4] = {0, 0, 0, 0};
  double curF = INFINITY, curMag = 0.0, curPg = 0.0, t = 1.0;
  double curG3 = 0.0, curGd = 0.0;  // g_3 and g.d at the current point (exhaustion rules)
  // the flat-tail rescue and the saddle escape (oracle: fit_one) in one word:
  // kEsc* flags + escapes x kEscN (per-lane bools would cost SGPR-pair masks)
  unsigned esc = 0u;
  int evals = 0, status = MDFIT_MAXITER;
  int first = 1;
#ifdef MDFIT_STAMP
  unsigned long long st_eval = 0, st_red = 0, st_logic = 0, st_fetch = 0, st_trips = 0;
  unsigned long long st_claim1 = 0, st_claim2 = 0;
  const unsigned long long k0 = stamp();
#endif

  while (true) {
#ifdef MDFIT_STAMP
    const unsigned long long f0 = stamp();
#endif
    bool starting = false;
    // ---- 1. idle slots pull an all-position task (one atomic per wave-trip) ---
    const bool need1 = mode == kIdle && !drained;
#ifdef MDFIT_STAMP
    const unsigned long long a0 = stamp();
#endif
    if (__any(need1)) {
      const unsigned long long m = __ballot(need1 && r == 0);
      int base = 0;
      if (lane == 0) base = atomicAdd(ws + qi, __popcll(m));
      base = __shfl(base, 0);
      if (need1) {
        const int64_t task = (int64_t)base + __popcll(m & ((1ull << leader) - 1ull));
        if (task >= 2 * nq) {
          drained = true;
        } else {
          sub = task < nq ? 0 : 1;  // 0 PMD-all, 1 null-all
          taxon = tl + task - (sub ? nq : 0);
          mode = kAllFit;
          starting = true;
          pa.pmd = pb.pmd = sub == 0;
          pa.valid = vA_all;
          pa.k = kA_all;
          pa.y = pa.valid ? (double)gy[taxon * kLD + colA_all] : 0.0;
          pa.N = pa.valid ? (double)gN[taxon * kLD + colA_all] : 0.0;
          if (PPL == 2) {
            pb.valid = vB_all;
            pb.k = kB_all;
            pb.y = pb.valid ? (double)gy[taxon * kLD + kNHalf + colA_all] : 0.0;
            pb.N = pb.valid ? (double)gN[taxon * kLD + kNHalf + colA_all] : 0.0;
          }
          const double* dg = diag(out, taxon, sub);  // u0 from K0
#pragma unroll
          for (int j = 0; j < 4; ++j) u[j] = dg[j];
        }
      }
    }
#ifdef MDFIT_STAMP
    const unsigned long long a1 = stamp();
#ifndef MDFIT_STAMP2
    st_claim1 += a1 - a0;
#endif
#endif
    // ---- 2. a finished all-position fit continues with its fwd/rev pair ----
    const bool next = mode == kNextPair;
    if (__any(next)) {
      if (PPL == 2) {  // wave-wide: every lane takes part in the shuffles
        const double ya = __shfl(pa.y, srcA), Na = __shfl(pa.N, srcA);
        const double yb = __shfl(pb.y, srcA), Nb = __shfl(pb.N, srcA);
        const double ya2 = __shfl(pa.y, srcB), Na2 = __shfl(pa.N, srcB);
        const double yb2 = __shfl(pb.y, srcB), Nb2 = __shfl(pb.N, srcB);
        if (next) {
          pa.valid = vA_pair;
          pa.k = kA_pair;
          pa.y = h ? yb : ya;
          pa.N = h ? Nb : Na;
          pb.valid = vB_pair;
          pb.k = kB_pair;
          pb.y = vB_pair ? (h ? yb2 : ya2) : 0.0;
          pb.N = vB_pair ? (h ? Nb2 : Na2) : 0.0;
        }
      }
      if (next) {
        sub = (pa.pmd ? 2 : 4) + h;  // PMD-f/r or null-f/r
        mode = kPairFit;
        starting = true;
        if (!allok) {  // the all-position fit did not converge: K0's initial point
          const double* dg = diag(out, taxon, sub);
#pragma unroll
          for (int j = 0; j < 4; ++j) u[j] = dg[j];
        }  // else: warm start at the all-position mode, u
      }
    }
#if defined(MDFIT_STAMP) && !defined(MDFIT_STAMP2)
    st_claim2 += stamp() - a1;
#endif
    if (starting) {
#pragma unroll
      for (int j = 0; j < 4; ++j) ut[j] = u[j];
      curF = INFINITY;
      curMag = curPg = 0.0;
      esc = 0u;
      t = 1.0;
      evals = 0;
      status = MDFIT_MAXITER;
      first = true;
      running = true;
    }
    if (!__any(mode != kIdle || !drained)) break;
#ifdef MDFIT_STAMP
    const unsigned long long e0 = stamp();
#endif
    if (!__any(running)) continue;

    // ---- 3. value + gradient + Hessian at the trial point --------------------
    const bool whole = mode == kAllFit;
    const Theta th = make_theta<kHalf>(pa.pmd, ut);  // row-collective: every lane
    double acc[kNAcc];
#pragma unroll
    for (int j = 0; j < kNAcc; ++j) acc[j] = 0.0;
    const int accf = (esc & kEscPolish) != 0u;
    // every slot of the wave fits model_null: a, b from the pads; every slot
    // holds an all-position fit: the two directions at the same |z| share a,
    // b (point_accum: null_row, whole_pair)
    // (slots not running evaluate garbage either way: they do not count)
    const bool null_wave = !__any(running && pa.pmd != 0);
    const bool whole_wave = !__any(running && !whole);
    if (PPL == 1) {
      point_accum<true>(pa, th, acc, accf, null_wave, whole_wave);
    } else {
      // lg3(phi) from a pad: lane 15's point b (all-position: both halves;
      // pair: the reverse half), lane 7's point b (pair: the forward half);
      // for model_null also lg3(a), lg3(b) (point_accum: null_row)
      const bool src15 = whole || h == 1;
      auto pad3 = [&](const LG3& v) -> LG3 { return src15 ? rowb3<15>(v) : rowb3<7>(v); };
      const PointArgs gb = point_args(pb, th);
      const LG3 t3b = lg3<true>(pb.N + th.phi);
      const LG3 t6 = pad3(t3b);
      const LG3 tb1 = lg3<true>(pb.y + gb.a);
      const LG3 tb2 = lg3<true>(pb.N - pb.y + gb.b);
      LG3 tb4, tb5;
      if (null_wave) {
        tb4 = pad3(tb1);
        tb5 = pad3(tb2);
      } else {
        tb4 = lg3<true>(gb.a);
        tb5 = lg3<true>(gb.b);
      }
      double accb[kNAcc];
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) accb[j] = 0.0;
      point_finish(pb, th, gb, tb1, tb2, t3b, tb4, tb5, t6, accb, accf);
      const PointArgs ga = point_args(pa, th);
      const LG3 ta3 = lg3<true>(pa.N + th.phi);
      const LG3 ta1 = lg3<true>(pa.y + ga.a);
      const LG3 ta2 = lg3<true>(pa.N - pa.y + ga.b);
      // (null: a, b are the half's; an all-position fit: point a is z = +k,
      // point b z = -k, the same a, b; a pair: the point's own)
      LG3 ta4 = tb4, ta5 = tb5;
      if (!null_wave && !whole_wave) {
        ta4 = lg3<true>(ga.a);
        ta5 = lg3<true>(ga.b);
      }
      point_finish(pa, th, ga, ta1, ta2, ta3, ta4, ta5, t6, acc, accf);
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) acc[j] = opaque(acc[j]) + opaque(accb[j]);
    }
#ifdef MDFIT_STAMP
    const unsigned long long e1 = stamp();
#endif
    // sums over the slot's positions (all-position fits) or the half's
    // Through LDS, accumulator-major: every lane writes its 16 terms to
    // sAcc[j][lane], then lane i of a row forms the row's sum of accumulator i
    // (tree16 / tree8: a register butterfly's summation tree, so the same bits
    // in both layouts), and the sums come back to every lane of the row from
    // sSum.  ~60 VALU per trip instead of ~240 DPP moves and adds (round 5).
#pragma unroll
    for (int j = 0; j < kNAcc; ++j) sAcc[j][lane] = acc[j];
    __syncthreads();
    if (PPL == 1) {
      // own row (the sub-fit of a pair half; for an all-position fit both rows
      // form the same sum: x_k = row 0 + row 1 at position k, as the butterfly's
      // first step)
      const double* a = &sAcc[jh][leader + 16 * h];
      const double* b = &sAcc[jh][leader + 16 * (1 - h)];
      double x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const double ak = a[k], bk = b[k];
        x[k] = whole ? ak + bk : ak;
      }
      sSum[0][lane] = tree16(x);
      __syncthreads();
      const double* src = &sSum[0][leader + 16 * h];
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) acc[j] = src[j];
    } else {
      // lane r of a 16-lane slot: accumulator r over each 8-lane half (the pair
      // sub-fits' sums), and their sum (the all-position fit's)
      const double* a = &sAcc[r][leader];
      double x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = a[k];
      const double A0 = tree8(x), A1 = tree8(x + 8);
      const double S = A0 + A1;
      sSum[0][lane] = whole ? S : A0;
      sSum[1][lane] = whole ? S : A1;
      __syncthreads();
      const double* src = &sSum[whole ? 0 : h][leader];
#pragma unroll
      for (int j = 0; j < kNAcc; ++j) acc[j] = src[j];
    }
#ifdef MDFIT_STAMP
    const unsigned long long e2 = stamp();
#endif

    // ---- 4. Newton logic (oracle: fit_one) ----------------------------------
    if (running) {
      Eval tr;
      finish_eval(pa.pmd, th, acc, tr);
      ++evals;
      const double pgt = pgnorm(ut, tr.g);  // projected gradient at the trial point
#ifdef MDFIT_STAMP2
      // (-DMDFIT_STAMP2: slots 6 / 7 of the stamp record split the Newton
      // logic -- finish_eval + pgnorm, and newton_dir)
      st_claim1 += stamp() - e2;
#endif
      bool accept = false, done = false;
      // the saddle escape's re-evaluation at u (same F, g, H as the current
      // point) goes through the acceptance below; its H gives the direction
      const bool probed = esc & kEscProbe;
      // the polish phase's re-evaluation at u (F now in the other form): taken
      // as the current point, then the ordinary Newton step (the same d)
      const bool pprobe = esc & kEscPolishProbe;
      // the gradient fallback's re-evaluation at u: its g gives the direction
      const bool gprobe = esc & kEscGradProbe;
      // the trial just evaluated was a full Newton step (not a probe, the first
      // point, a backtracked / escape / gradient-fallback / flat-tail-rescue
      // step), and its size: the quadratic-contraction stop below
      const bool newton_trial = !(probed || pprobe || gprobe) && !first &&
                                !(esc & (kEscNc | kEscGrad | kEscRelax)) && t == 1.0;
      const double dprev = t * maxabs4(d);
      esc &= ~(kEscProbe | kEscPolishProbe | kEscGradProbe);
      if (probed || pprobe || gprobe) {
        accept = true;
      } else if (first) {
        accept = true;
        first = false;
        if (!isfinite(tr.F)) {
          done = true;
          status = MDFIT_NONFINITE;
        }
      } else {
        const double noise = kNoiseF * (curMag + fabs(curF));
        accept = isfinite(tr.F) &&
                 ((esc & kEscNc) ? tr.F < curF - noise : (tr.F < curF || (tr.F <= curF + noise && ((esc & kEscRelax) || pgt < curPg))));
      }
      esc &= ~kEscRelax;
      if (accept) {
#pragma unroll
        for (int j = 0; j < 4; ++j) u[j] = ut[j];
        curF = tr.F;
        curMag = tr.mag;
        curPg = pgt;
        esc &= ~(kEscNc | kEscGrad);
        if (!done) {
          // (the gradient fallback's probe: the projected-gradient direction
          // replaces the Newton step; oracle: fit_one)
#ifdef MDFIT_STAMP2
          const unsigned long long nd0 = stamp();
#endif
          const bool ind = newton_dir<kHalf>(pa.pmd, u, tr.g, tr.H, pgt, d, probed);
#ifdef MDFIT_STAMP2
          st_claim2 += stamp() - nd0;
#endif
          const bool gok = gprobe && pg_direction(u, tr.g, d);
          curG3 = tr.g[3];
          curGd = tr.g[0] * d[0] + tr.g[1] * d[1] + tr.g[2] * d[2] + tr.g[3] * d[3];
          t = 1.0;
          if (gprobe) {
            if (gok) {
              esc |= kEscNc | kEscGrad;
            } else {
              done = true;
              status = (esc & kEscExhOk) ? MDFIT_OK : MDFIT_MAXITER;
            }
          } else if (probed) {
            if (ind) {
              esc += kEscN | kEscNc;
            } else if (!(esc & kEscExhOk) && (esc & kEscGradCount) < 8u * kEscGradN && evals < max_iter) {
              // no escape direction: the gradient fallback, from its own
              // re-evaluation at u (oracle: fit_one)
              esc += kEscGradN;
              esc |= kEscGradProbe;
              d[0] = d[1] = d[2] = d[3] = 0.0;
            } else {
              done = true;
              status = (esc & kEscExhOk) ? MDFIT_OK : MDFIT_MAXITER;
            }
          } else {
            esc = ind ? esc | kEscIndef : esc & ~kEscIndef;
            const double dn = maxabs4(d);
            if (dn <= tol) {
              done = true;
              status = MDFIT_OK;
            } else if (newton_trial && !ind && kQuadK * dn * dn <= tol && dn <= kQuadK * dprev * dprev) {
              // MDFIT-MAP v1.1 (oracle: fit_one): converged by quadratic
              // contraction -- the step is taken without evaluating its end
              // point (the error left is O(|d|^2) <= tol)
#pragma unroll
              for (int j = 0; j < 4; ++j) u[j] = clampd(u[j] + d[j], kULo[j], kUHi[j]);
              done = true;
              status = MDFIT_OK;
            }
          }
        }
      } else if (esc & kEscNc) {  // the escape finds no decrease beyond F's rounding
        t *= 0.5;
        if (t < ((esc & kEscGrad) ? 1e-6 : 1e-3)) {
          if (esc & kEscGrad) {
            // nor does the projected gradient, for steps down to 1e-6: optimal
            // to F's resolution (oracle: fit_one)
            done = true;
            status = MDFIT_OK;
          } else if (!(esc & kEscExhOk) && (esc & kEscGradCount) < 8u * kEscGradN && evals < max_iter) {
            esc += kEscGradN;  // the gradient fallback: re-evaluate at u next trip
            esc |= kEscGradProbe;
            d[0] = d[1] = d[2] = d[3] = 0.0;
            t = 1.0;
          } else {
            done = true;
            status = (esc & kEscExhOk) ? MDFIT_OK : MDFIT_MAXITER;
          }
        }
      } else {
        t *= 0.5;
        const bool unresolved = t * fabs(curGd) <= kNoiseF * (curMag + fabs(curF));
        if (!(esc & kEscPolish) && evals < max_iter && (t < 1e-12 || unresolved)) {
          // the polish phase (oracle: fit_one): the backtracking step's
          // predicted decrease is below F's rounding -- re-evaluate at u with F
          // in the cancellation-free form next trip, then restart at t = 1
          esc |= kEscPolish | kEscPolishProbe;
          d[0] = d[1] = d[2] = d[3] = 0.0;
          t = 1.0;
        } else if (t < 1e-12 || ((esc & kEscPolish) && unresolved)) {
          // line search exhausted (oracle: fit_one), in the polish phase also
          // when even the cancellation-free F cannot resolve the decrease
          if (!(esc & kEscRescued) && u[3] < 0.0 && d[3] < 0.0 && u[3] > kULo[3]) {
            // the flat tail of log delta: jump onto its lower bound once
            esc |= kEscRescued | kEscRelax;
            d[0] = d[1] = d[2] = 0.0;
            d[3] = kULo[3] - u[3];
            curGd = curG3 * d[3];
            t = 1.0;
          } else {
            const bool exh_ok =
                maxabs4(d) <= 1e-5 || curPg <= kPgTol || fabs(curGd) <= kNoiseF * (curMag + fabs(curF));
            esc = exh_ok ? esc | kEscExhOk : esc & ~kEscExhOk;
            if ((esc & kEscIndef) && (esc & kEscCount) < 4u * kEscN && evals < max_iter) {
              // the saddle escape (oracle: fit_one): re-evaluate at u next trip
              esc |= kEscProbe;
              d[0] = d[1] = d[2] = d[3] = 0.0;
              t = 1.0;
            } else if (!exh_ok && (esc & kEscGradCount) < 8u * kEscGradN && evals < max_iter) {
              // the gradient fallback (oracle: fit_one): re-evaluate at u next trip
              esc += kEscGradN;
              esc |= kEscGradProbe;
              d[0] = d[1] = d[2] = d[3] = 0.0;
              t = 1.0;
            } else {
              done = true;
              status = exh_ok ? MDFIT_OK : MDFIT_MAXITER;
            }
          }
        }
      }
      if (!done && evals >= max_iter) {
        done = true;
        status = MDFIT_MAXITER;
      }
      if (!done) {
#pragma unroll
        for (int j = 0; j < 4; ++j) ut[j] = clampd(u[j] + t * d[j], kULo[j], kUHi[j]);
      } else {
        // lanes 0..7 of the half write the diag slots (for an all-position fit
        // the forward half only)
        const int i = jh;
        const bool writer = (!whole || h == 0) && i < 8;
        if (writer) {
          const double v = i < 4 ? sel4(u, i)
                                 : (i == 4 ? curF
                                           : (i == 5 ? (double)evals
                                                     : (i == 6 ? (double)status : ((esc & kEscPolish) ? 1.0 : 0.0))));
          diag(out, taxon, sub)[i] = v;
        }
        allok = status == MDFIT_OK;  // (read after an all-position fit: the pair's warm start)
        running = false;
      }
    }
    // waves holding a long fit (the critical path of small batches) win issue
    // arbitration: +5 % at C2, no change at 100k taxa (A/B of thresholds
    // 12/15/20/30 and of chain- vs fit-length counting: 15 by fit length best)
    // (base_prio: every fit wave above the HPDI stream kernel's waves beside it)
    if (__any(running && evals >= 2 * kPrioEvals)) __builtin_amdgcn_s_setprio(3);
    else if (__any(running && evals >= kPrioEvals)) __builtin_amdgcn_s_setprio(2);
    else if (base_prio) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    // a slot is free when neither half is running: an all-position fit then
    // continues with its pair, a pair with the next task
    const unsigned long long busy = __ballot(running);
    if ((busy & slot_mask) == 0ull) {
      if (mode == kAllFit) {
        if (sub == 0) {
          // the PMD-all fit just ended: publish its (q, A, c, phi) -- make_theta's
          // arithmetic, NaN for invalid input -- as the next entry of the ready
          // list that hpdi_stream_kernel consumes beside this kernel (the
          // predictive HPDI, MDFIT-HPDI v2).  The slot's first lane writes the
          // entry's five fields as relaxed agent-scope atomic stores of their
          // bit complements (ready_put): K0 zeroed the list, so a field reads
          // non-zero exactly once this call has written it, and a reader takes
          // the entry when all five do -- no cross-field ordering is needed,
          // hence no fence (an agent-scope release / acquire pair costs an L2
          // write-back per publication and an L2 invalidate per take on this
          // multi-XCD part: C2 1.24 -> 1.45 ms, measured)
          auto sig = [](double v) {
            const double e = exp(-fabs(v));
            const double rr = rcp(1.0 + e);
            return v >= 0.0 ? rr : e * rr;
          };
          const bool badA = vA_all && pa.y > pa.N;
          const bool badB = PPL == 2 && vB_all && pb.y > pb.N;
          const bool bad = (__ballot(badA || badB) & slot_mask) != 0ull;
          if (r == 0) {
#ifdef MDFIT_DEV_HPTIME
            MDFIT_DEV_T(taxon);
#endif
            const int idx = atomicAdd(ws + kWsReady, 1);
            uint64_t* e = reinterpret_cast<uint64_t*>(ready + (int64_t)idx * kReadyStride);
            ready_put(e + 0, bad ? NAN : sig(u[0]));
            ready_put(e + 1, bad ? NAN : sig(u[1]));
            ready_put(e + 2, bad ? NAN : u[2]);
            ready_put(e + 3, bad ? NAN : exp(u[3]) + 2.0);
            __hip_atomic_store(e + 4, ~(uint64_t)taxon, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        mode = kNextPair;
      } else if (mode == kPairFit) {
#ifdef MDFIT_DEV_HPTIME
        if (r == 0) MDFIT_DEV_T(T + taxon);
#endif
        mode = kIdle;
      }
    }
#ifdef MDFIT_STAMP
    const unsigned long long l1 = stamp();
    st_fetch += e0 - f0;
    st_eval += e1 - e0;
    st_red += e2 - e1;
    st_logic += l1 - e2;
    st_trips += 1;
#endif
  }
#ifdef MDFIT_STAMP
  if (lane == 0 && g_stamp != nullptr) {
    unsigned long long* rr = g_stamp + (int64_t)blockIdx.x * 8;
    rr[0] = st_eval;
    rr[1] = st_red;
    rr[2] = st_logic;
    rr[3] = st_fetch;
    rr[4] = st_trips;
    rr[5] = stamp() - k0;
    rr[6] = st_claim1;
    rr[7] = st_claim2;
  }
#endif
}


// ---------------------------------------------------------------------------
// K3: record assembly, one wave per taxon
// ---------------------------------------------------------------------------
// MAP predictive median of one point (oracle: predict()): D(z), NaN when N = 0
// (the reference divides 0 draws by N = 0); the HPDI bounds are K4's.
__device__ __forceinline__ double predict_median(double A, double q, double c, int k, double N) {
  if (N == 0.0) return NAN;
  return fmin(fma(A, powk(1.0 - q, k), c), 1.0);
}

// n_sigma (fits.py:194-201) over the valid lanes of G-lane groups, from each
// lane's pointwise log-likelihoods under the two models (waic_i = -2 ell_i).
template <int G>
__device__ __forceinline__ double nsigma_group(bool valid, double lP, double lN, double n) {
  const double v = valid ? 1.0 : 0.0;
  const double dd0 = v * ((-2.0 * lP) - (-2.0 * lN));
  const double md = gsum<G>(dd0) / n;
  const double wP = gsum<G>(v * (-2.0 * lP));
  const double wN = gsum<G>(v * (-2.0 * lN));
  const double dd = v * (dd0 - md);
  const double var = gsum<G>(dd * dd) / n;
  return (wN - wP) / sqrt(n * var);
}

// field-wise select (keeps the 6 sub-fit thetas in registers: no dynamic
// indexing of a local array, which would go to scratch)
__device__ __forceinline__ Theta sel(bool c, const Theta& a, const Theta& b) {
  Theta r;
  r.q = c ? a.q : b.q;
  r.omq = c ? a.omq : b.omq;
  r.iomq = c ? a.iomq : b.iomq;
  r.A = c ? a.A : b.A;
  r.JA = c ? a.JA : b.JA;
  r.c = c ? a.c : b.c;
  r.iomc = c ? a.iomc : b.iomc;
  r.delta = c ? a.delta : b.delta;
  r.phi = c ? a.phi : b.phi;
  r.lprior = c ? a.lprior : b.lprior;
  return r;
}

// lane l's theta, read by every lane (wave-uniform l)
__device__ __forceinline__ double read_lane(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ Theta read_theta(const Theta& t, int l) {
  Theta r;
  r.q = read_lane(t.q, l);
  r.omq = read_lane(t.omq, l);
  r.iomq = read_lane(t.iomq, l);
  r.A = read_lane(t.A, l);
  r.JA = read_lane(t.JA, l);
  r.c = read_lane(t.c, l);
  r.iomc = read_lane(t.iomc, l);
  r.delta = read_lane(t.delta, l);
  r.phi = read_lane(t.phi, l);
  r.lprior = read_lane(t.lprior, l);
  return r;
}

// D at |z|-1 = k under theta (D(z) of model_PMD, fits.py:50; q for model_null)
__device__ __forceinline__ double d_of(const Theta& th, bool pmd, int k) {
  return pmd ? fma(th.A, powk(th.omq, k), th.c) : th.q;
}

__global__ __launch_bounds__(kWave) void assemble_kernel(
    const uint32_t* __restrict__ gy, const uint32_t* __restrict__ gN,
    const uint32_t* __restrict__ gmm, int64_t n_taxa, double* __restrict__ out,
    float* __restrict__ pred, int32_t* __restrict__ status) {
  __shared__ double s_y[kLD], s_N[kLD];
  __shared__ uint32_t s_mm[kNPos * kNMM];
  __shared__ double s_rec[MDFIT_NOUT];
  __shared__ double s_tmp[kWave];
  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  if (t >= n_taxa) return;

  if (lane < kLD) {
    s_y[lane] = (double)gy[t * kLD + lane];
    s_N[lane] = (double)gN[t * kLD + lane];
  }
  if (gmm != nullptr)
    for (int i = lane; i < kNPos * kNMM; i += kWave) s_mm[i] = gmm[t * (kNPos * kNMM) + i];
  for (int i = lane; i < MDFIT_NOUT; i += kWave)  // reserved fields 25..31 -> 0
    s_rec[i] = (i >= MDFIT_NRESULT && i < MDFIT_F_DIAG) ? 0.0 : out[t * MDFIT_NOUT + i];
  __syncthreads();

  // invalid input (y > N) -> status 3, NaN record (oracle: fit_taxon)
  const bool bad_lane = lane < kNPos && s_y[lane] > s_N[lane];
  if (__any(bad_lane)) {
    for (int i = lane; i < MDFIT_NOUT; i += kWave) out[t * MDFIT_NOUT + i] = NAN;
    if (pred != nullptr)
      for (int i = lane; i < MDFIT_NPRED * kNPos; i += kWave) pred[t * (MDFIT_NPRED * kNPos) + i] = NAN;
    if (lane == 0) status[t] = MDFIT_INVALID;
    return;
  }

  // modes of the 6 sub-fits (u* in diag slots 0..3) -> constrained parameters:
  // make_theta is row-collective with the same arithmetic on any 16-lane row,
  // so the four rows take sub-fits 0-3, then rows 0-1 sub-fits 4-5, and every
  // lane reads each theta from its row's first lane (2 calls instead of 6; the
  // thetas in SGPRs: 54 VGPRs instead of 88, 8 waves/SIMD instead of 5 --
  // 125k taxa 9.92 -> 9.67 ms, 1M 75.8 -> 73.6 ms per call, C2 within noise)
  Theta ths[MDFIT_NSUBFIT];
  int st = MDFIT_OK;
#pragma unroll
  for (int s = 0; s < MDFIT_NSUBFIT; ++s) st = max(st, (int)s_rec[MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * s + 6]);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int row = lane >> 4;
    const int s = pass == 0 ? row : 4 + (row & 1);
    const double* dg = s_rec + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * s;
    const double uu[4] = {dg[0], dg[1], dg[2], dg[3]};
    const Theta th = make_theta(s == 0 || s == 2 || s == 3, uu);
#pragma unroll
    for (int r = 0; r < (pass == 0 ? 4 : 2); ++r) ths[4 * pass + r] = read_theta(th, 16 * r);
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < MDFIT_NSUBFIT; ++s) {  // diag slots 0..3 <- (q, A, c, phi)
    if (lane == s) {
      double* dg = s_rec + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * s;
      dg[0] = ths[s].q;
      dg[1] = ths[s].A;
      dg[2] = ths[s].c;
      dg[3] = ths[s].phi;
    }
  }

  // ---- all-position fits: lanes 0-31 PMD, 32-63 null (lane = position) -------
  const int pA = lane & 31;
  const bool vA = pA < kNPos;
  const int iA = vA ? pA : 0;
  const int kA = iA < kNHalf ? iA : iA - kNHalf;
  const bool pmdA = lane < 32;
  const Theta thA = sel(pmdA, ths[0], ths[1]);
  const double ellA = point_ell(s_y[iA], s_N[iA], d_of(thA, pmdA, kA), thA.phi);
  const double ellPall = ellA;  // meaningful on lanes 0..29
  {
    const double ellN = __shfl_xor(ellA, 32);
    const double ns = nsigma_group<32>(vA, ellA, ellN, (double)kNPos);  // fits.py:252
    const double med = predict_median(ths[0].A, ths[0].q, ths[0].c, kA, s_N[iA]);
    if (lane < kNPos && pred != nullptr) pred[t * (MDFIT_NPRED * kNPos) + lane] = (float)med;
    if (lane == 0) {
      s_rec[MDFIT_F_N_SIGMA] = ns;
      s_rec[MDFIT_F_D_MAX] = med;  // fits.py:249-250: predictive median at z = +1
      s_rec[MDFIT_F_Q_MEAN] = ths[0].q;
      s_rec[MDFIT_F_CONCENTRATION_MEAN] = ths[0].phi;
      s_rec[MDFIT_F_D_MAX_MARGINALIZED_MEAN] = ths[0].A + ths[0].c;
    }
  }

  // ---- forward / reverse fits: rows PMD-f, PMD-r, null-f, null-r -------------
  {
    const int row = lane >> 4, p = lane & 15;
    const bool vB = p < kNHalf;
    const bool rev = row & 1;
    const int iB = (vB ? p : 0) + (rev ? kNHalf : 0);
    const int kB = vB ? p : 0;
    const bool pmdB = row < 2;
    const Theta thB = sel(row < 2, sel(row == 0, ths[2], ths[3]), sel(row == 2, ths[4], ths[5]));
    const double ellB = point_ell(s_y[iB], s_N[iB], d_of(thB, pmdB, kB), thB.phi);
    const double ellN = __shfl_xor(ellB, 32);
    const double ns = nsigma_group<16>(vB, ellB, ellN, (double)kNHalf);  // fits.py:317-320, 339-342
    // D_max_forward / _reverse: predictive median at data_forward[0]
    // (fits.py:322-327; the reverse one is evaluated on data_forward, :343-348)
    const double med = predict_median(thB.A, thB.q, thB.c, 0, s_N[0]);
    if (lane == 0) {
      s_rec[MDFIT_F_N_SIGMA_FORWARD] = ns;
      s_rec[MDFIT_F_D_MAX_FORWARD] = med;
      s_rec[MDFIT_F_Q_MEAN_FORWARD] = thB.q;
    }
    if (lane == 16) {
      s_rec[MDFIT_F_N_SIGMA_REVERSE] = ns;
      s_rec[MDFIT_F_D_MAX_REVERSE] = med;
      s_rec[MDFIT_F_Q_MEAN_REVERSE] = thB.q;
    }
    // asymmetry (fits.py:352-356, 204-227): PMD-all vs concat(PMD-fwd, PMD-rev);
    // position p of the concatenation lives on lane p (p < 15) or lane p + 1
    const int src = lane < kNHalf ? lane : lane + 1;
    const double ellFR = __shfl(ellB, src & 63);
    const double v = lane < kNPos ? 1.0 : 0.0;
    const double dC = v * ((-2.0 * ellPall) - (-2.0 * ellFR));
    const double md = gsum<64>(dC) / kNPos;
    const double wC = gsum<64>(v * (-2.0 * ellPall));
    const double wFR = gsum<64>(v * (-2.0 * ellFR));
    const double dd = v * (dC - md);
    const double var = gsum<64>(dd * dd) / kNPos;
    if (lane == 0) s_rec[MDFIT_F_ASYMMETRY] = (wFR - wC) / sqrt(kNPos * var);
  }

  record_sums_noise(lane, s_y, s_N, s_mm, gmm != nullptr, s_rec, s_tmp);

  __syncthreads();
  // every field but the two HPDI columns, which K4 writes (it runs beside this
  // kernel on the caller's stream)
  for (int i = lane; i < MDFIT_NOUT; i += kWave)
    if (i != MDFIT_F_D_MAX_LOWER_HPDI && i != MDFIT_F_D_MAX_UPPER_HPDI) out[t * MDFIT_NOUT + i] = s_rec[i];
  if (lane == 0) status[t] = st;
}

// mdfit_noise: the three noise columns (add_noise_estimates, fits.py:359-376)
// of records fitted with mm = NULL, from the mismatch counts -- the record
// assembly's own noise code, so the columns are those of a call with mm bit
// for bit.  One wave per taxon; an invalid taxon (y > N, its record NaN) is
// left alone.  The host's chunked dispatch ships mm while the fit runs and
// fills the columns after (engine.ChunkedFitter).
__global__ __launch_bounds__(kWave) void noise_kernel(const uint32_t* __restrict__ gy,
                                                      const uint32_t* __restrict__ gN,
                                                      const uint32_t* __restrict__ gmm, int64_t n_taxa,
                                                      double* __restrict__ out) {
  __shared__ uint32_t s_mm[kNPos * kNMM];
  __shared__ double s_rec[MDFIT_NOUT];
  __shared__ double s_tmp[kWave];
  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  if (t >= n_taxa) return;
  const bool bad_lane = lane < kNPos && gy[t * kLD + lane] > gN[t * kLD + lane];
  if (__any(bad_lane)) return;
  for (int i = lane; i < kNPos * kNMM; i += kWave) s_mm[i] = gmm[t * (kNPos * kNMM) + i];
  __syncthreads();
  record_noise(lane, s_mm, true, s_rec, s_tmp);
  __syncthreads();
  if (lane < 3) out[t * MDFIT_NOUT + MDFIT_F_NORMALIZED_NOISE + lane] = s_rec[MDFIT_F_NORMALIZED_NOISE + lane];
}

// ---------------------------------------------------------------------------
// K4: 68 % predictive HPDI (MDFIT-HPDI v2, mdfit_hpdi.h) of the PMD-all mode at
// every position (fits.py:112-120, 260-261).  K4a: one lane per (taxon,
// position) -- neighbouring lanes hold neighbouring positions of one taxon;
// windows of sd <= 40 points are finished there (the greedy), wide ones go to
// a compacted list.  K4b: persistent; each lane runs one wide window's state
// machine at a time and refills from the list (mdfit_hpdi.h).
// Sources: the fit record (kFit: PMD-all (q, A, c, phi) + N; pred == nullptr
// -> only z = +1, the D_max_{lower,upper}_hpdi columns) or plain arrays
// (mdfit_hpdi68, parity tests).
// ---------------------------------------------------------------------------
template <bool kFit>
__global__ __launch_bounds__(kPrepBlock) void hpdi_prep_kernel(HpdiIO io, int64_t n_items, int* __restrict__ ctr,
                                                               hpdi::WideRec* __restrict__ recs) {
  const int64_t item = (int64_t)blockIdx.x * kPrepBlock + threadIdx.x;
  const bool valid = item < n_items;
  double N = 0.0, a = 0.0, b = 0.0;
  bool skip = true;
  int64_t oitem = item;  // the output index (kFit: taxon * per + position)
  if (valid) {
    if (kFit) {
      // items in ready-list order: entry item / per, stream-ordered after the
      // fit kernel (every entry written)
      const int64_t ei = item / io.per;
      const int i = (int)(item - ei * io.per);
      // PMD-all: the complements of (q, A, c, phi, taxon) (ready_put)
      const uint64_t* dg = reinterpret_cast<const uint64_t*>(io.ready + ei * kReadyStride);
      const double q = __longlong_as_double(~dg[0]), A = __longlong_as_double(~dg[1]);
      const double c = __longlong_as_double(~dg[2]), phi = __longlong_as_double(~dg[3]);
      const int64_t t = (int64_t)~dg[4];
      oitem = t * io.per + i;
      N = (double)io.gN[t * kLD + i];
      if (N > 0.0 && !isnan(q)) {
        const int k = i < kNHalf ? i : i - kNHalf;
        const double D = fmin(fma(A, powk(1.0 - q, k), c), 1.0);
        a = D * phi;
        b = (1.0 - D) * phi;
        skip = false;
      }
    } else {
      N = io.N[item];
      a = io.a[item];
      b = io.b[item];
      skip = !(N > 0.0);
    }
  }
  hpdi_position<kFit>(io, oitem, valid, skip, N, a, b, n_items, ctr, recs);
}

// one lane per wide window at a time: every trip each busy lane runs one level
// iteration of its window; a settled window is finished (fix-up, write) and
// the lane claims the next record (one atomic per wave-trip on ctr[1]), so the
// wave's evaluation sites stay busy whatever each window's iteration count.
// Exit: a lane that draws an index past the list stops claiming; the wave
// leaves when none of its lanes holds a window.
#ifndef MDFIT_HPDI_WAVES_PER_EU
#define MDFIT_HPDI_WAVES_PER_EU 2
#endif
template <bool kFit>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(MDFIT_HPDI_WAVES_PER_EU))) void hpdi_wide_kernel(HpdiIO io, int64_t n_items, int* __restrict__ ctr,
                                                          const hpdi::WideRec* __restrict__ recs) {
  const int n_front = ctr[0], n_wide = n_front + ctr[2];  // written by K4a (stream-ordered)
  hpdi::Wide W;
  int64_t item = 0;
  bool busy = false, drained = false;
  while (true) {
    const bool need = !busy && !drained;
    const unsigned long long m = __ballot(need);
    if (m != 0ull) {
      int base = 0;
      if (threadIdx.x == 0) base = atomicAdd(ctr + 1, __popcll(m));
      base = __shfl(base, 0);
      if (need) {
        const int idx = base + __popcll(m & ((1ull << threadIdx.x) - 1ull));
        if (idx < n_wide) {
          const hpdi::WideRec r = recs[idx < n_front ? (int64_t)idx : n_items - 1 - (idx - n_front)];
          item = r.item;
          hpdi::wide_start(W, r);
          busy = true;
        } else {
          drained = true;
        }
      }
    }
    if (!__any(busy)) break;
    if (busy && hpdi::wide_iter(W)) {
      double lo, hi;
      hpdi::wide_finish(W, lo, hi);
      hpdi_write<kFit>(io, item, W.P.N, lo, hi);
      busy = false;
    }
  }
}

// ---------------------------------------------------------------------------
// K4 of mdfit_fit_batch: the predictive HPDI streamed beside the fit
// ---------------------------------------------------------------------------
// One lane per (taxon, position) item at a time, items enumerated in ready-list
// order (entry = a PMD-all mode published by fit_kernel as that fit ends, see
// fit_kernel): a lane claims an item (one atomic per wave-trip), waits for its
// entry's tag, then runs the position's window -- the greedy when narrow
// (prep_position), else the wide window's level iterations, one per trip, with
// the lane refilling when it settles (the K4a / K4b arithmetic: the same
// windows bit for bit).  Two launches share the claim counter: kEarly on a side
// stream beside fit_kernel with a small grid (MDFIT_STREAM_WAVES_PER_CU waves
// per CU; the fit kernel's grid leaves them room), so the HPDI work fills the
// fit kernel's idle issue slots and its tail; and one after fit_kernel on the
// caller's stream, full occupancy, for what is left.
// Waiting (round 4: bounded, no wave waits indefinitely while holding a claim):
// a kEarly wave waits on entries only after it has seen fit_kernel's started
// flag, and exits when the flag has not appeared within ~50 us (its launch may
// have been queued behind this one: the two streams can share a hardware
// queue).  While it waits it holds claimed items; when a wave has made no
// progress for `defer_ticks` (100 MHz ticks; MDFIT_STREAM_DEFER_US, default
// 1 ms -- far beyond any wait of a co-resident run) or another
// early wave has already deferred, it hands its pending items to the defer
// list (reservation by CAS on kWsDefRes, one release add on kWsDefDone per
// item written), claims no more, finishes its wide windows and exits -- so a
// fit queue whose waves cannot get a slot (another kernel on the device, a
// concurrent call) only delays the HPDI, it cannot hang the device.  The late
// launch (after fit_kernel in stream order: every entry published) closes the
// defer list (atomicOr of kDefClosed: a reservation after that fails, and the
// early wave then keeps waiting -- fit_kernel is done, its entry is about to
// be seen), waits until every reserved slot is written (its writer is
// resident, one store away) and drains the deferred items after the main
// claim counter.  The late launch never waits on the fit.
// An early HPDI wave hands its pending items to the defer list (see
// hpdi_stream_kernel): true when they were taken (the wave then claims no
// more), false when the late launch has closed the list already (every entry
// is published then: keep waiting).  Out of line: the stream kernel is
// register-bound, and this rarely-run path should not shape its allocation.
__device__ __noinline__ bool defer_items(int* ws, int* defer, bool pending, int item) {
  const int lane = (int)threadIdx.x;
  const unsigned long long pm = __ballot(pending);
  int base = -1;
  if (lane == 0) {
    int old = __hip_atomic_load(ws + kWsDefRes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (!(old & (int)kDefClosed)) {
      if (__hip_atomic_compare_exchange_strong(ws + kWsDefRes, &old, old + __popcll(pm), __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        base = old;
        break;
      }
    }
  }
  base = __shfl(base, 0);
  if (base < 0) return false;
  if (pending) {
    __hip_atomic_store(defer + base + __popcll(pm & ((1ull << lane) - 1ull)), item, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(ws + kWsDefDone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (lane == 0) __hip_atomic_store(ws + kWsEarlyQuit, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

#ifndef MDFIT_STREAM_WAVES_PER_CU
#define MDFIT_STREAM_WAVES_PER_CU 3  // A/B at 10k taxa (tools/_gpu_r05b.sh, profiles/r05_stream_waves.txt): 3 since HPDI v2 (1.08 ms; 4: 1.12, 2: 1.26); round 4: 4
#endif
template <bool kEarly>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(MDFIT_HPDI_WAVES_PER_EU))) void hpdi_stream_kernel(
    const uint32_t* __restrict__ gN, int64_t T, int per, double* __restrict__ out, float* __restrict__ pred,
    int* __restrict__ ws, const double* __restrict__ ready, int* __restrict__ defer, uint32_t defer_ticks) {
  const int lane = threadIdx.x;
  uint64_t t_wait = 0;  // early: when the current run of trips without progress began (0: none)
  if (kEarly) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while (__hip_atomic_load(ws + kWsStarted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 5000u) return;  // 50 us: the fit kernel is not running
      __builtin_amdgcn_s_sleep(8);
    }
    // another early wave has deferred already: nothing for this one to do
    if (__hip_atomic_load(ws + kWsEarlyQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  } else if (blockIdx.x == 0 && lane == 0) {
    __hip_atomic_store(ws + kWsEarlyClaimed, __hip_atomic_load(ws + kWsClaim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  HpdiIO io{};
  io.out = out;
  io.pred = pred;
  io.per = per;
  const int64_t n_items = T * per;
  // a lane's wide-window state lives in LDS between trips (~300 B per lane): in
  // registers it stays live through the item set-up (prep_position) of the
  // other lanes and the kernel spilled
  __shared__ hpdi::Wide sW[kWave];
  hpdi::Wide& W = sW[lane];
  int64_t item = 0, oitem = 0;  // the claimed item; its output index taxon * per + position
  bool busy = false, pending = false, drained = false;
  // late launch: phase 0 claims from the main counter, phase 1 the deferred
  // items (n_def of them, read once the list is closed); early: stop = this
  // wave claims no more (it deferred, or saw another early wave defer),
  // keep = the defer list is closed (keep waiting: every entry is published)
  int phase = 0, n_def = -1;
  bool stop = false, keep = false;
  while (true) {
    const bool need = !busy && !pending && !drained && !stop;
    const unsigned long long m = __ballot(need);
    if (m != 0ull) {
      int base = 0;
      if (!kEarly && phase == 1) {
        if (n_def < 0) {
          // close the list; the count it held is final (reservations are CAS
          // that fail once closed), then wait for its slots' writes.  A wave
          // that finds it closed already reads the count with a plain load
          // (one atomic per call, not per wave, on this line)
          int r0 = 0;
          if (lane == 0) {
            r0 = __hip_atomic_load(ws + kWsDefRes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!(r0 & (int)kDefClosed)) r0 = atomicOr(ws + kWsDefRes, (int)kDefClosed);
          }
          n_def = __shfl(r0, 0) & ~(int)kDefClosed;
          if (n_def > 0)
            while (__hip_atomic_load(ws + kWsDefDone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < n_def)
              __builtin_amdgcn_s_sleep(2);
        }
        if (lane == 0 && n_def > 0) base = atomicAdd(ws + kWsDefClaim, __popcll(m));
      } else if (lane == 0) {
        base = atomicAdd(ws + kWsClaim, __popcll(m));
      }
      base = __shfl(base, 0);
      if (need) {
        const int64_t it = (int64_t)base + __popcll(m & ((1ull << lane) - 1ull));
        if (!kEarly && phase == 1) {
          if (n_def == 0 || it >= n_def) drained = true;
          else {
            item = __hip_atomic_load(defer + it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pending = true;
          }
        } else if (it >= n_items) {
          drained = true;
        } else {
          item = it;
          pending = true;
        }
      }
    }
    bool prog = false;
    if (pending) {
      const int64_t ei = item / per;
      const double* e = ready + ei * kReadyStride;
      const uint64_t* f = reinterpret_cast<const uint64_t*>(e);
      // the taxon field first (written last), then the four values: taken when
      // all five are non-zero (else the lane polls again next trip)
#ifdef MDFIT_LOAD5
      const uint64_t ftax = ready_get(f + 4);
      const uint64_t fq = ready_get(f + 0), fA = ready_get(f + 1), fc = ready_get(f + 2), fphi = ready_get(f + 3);
#else
      const uint64_t ftax = ready_get(f + 4);
      uint64_t fq = 0, fA = 0, fc = 0, fphi = 0;
      if (ftax != 0) {
        fq = ready_get(f + 0);
        fA = ready_get(f + 1);
        fc = ready_get(f + 2);
        fphi = ready_get(f + 3);
      }
#endif
      if (ftax != 0 && fq != 0 && fA != 0 && fc != 0 && fphi != 0) {
        const double q = __longlong_as_double(~fq);
        const double A = __longlong_as_double(~fA);
        const double c = __longlong_as_double(~fc);
        const double phi = __longlong_as_double(~fphi);
        const int64_t taxon = (int64_t)~ftax;
        const int i = (int)(item - ei * per);
        // (never out of range: K0 zeroes the list and only this call's fit
        // kernel tags entries; a corrupt one is dropped and counted, not followed)
        const bool sane = taxon >= 0 && taxon < T;
        if (!sane) atomicAdd(ws + kWsBad, 1);
        oitem = sane ? taxon * per + i : 0;
        const double N = sane ? (double)gN[taxon * kLD + i] : 0.0;
        double lo = NAN, hi = NAN;
        bool wide = false;
        if (sane && N > 0.0 && !isnan(q)) {  // (the arithmetic of hpdi_prep_kernel)
          const int k = i < kNHalf ? i : i - kNHalf;
          const double D = fmin(fma(A, powk(1.0 - q, k), c), 1.0);
          hpdi::WideRec rec;
          wide = !hpdi::prep_position(N, D * phi, (1.0 - D) * phi, lo, hi, rec);
          if (wide) hpdi::wide_start(W, rec);
        }
#ifdef MDFIT_DEV_HPTIME
        if (sane) MDFIT_DEV_T(2 * T + oitem);
        if (sane && !wide) MDFIT_DEV_T(2 * T + n_items + oitem);
#endif
        if (wide) busy = true;
        else if (sane) hpdi_write<true>(io, oitem, N, lo, hi);
        pending = false;
        prog = true;
      }
    }
    if (!kEarly && !__any(busy || pending || !drained)) {
      if (phase == 1) break;
      phase = 1;  // the main counter is drained: the deferred items
      drained = false;
      continue;
    }
    if (kEarly && !__any(busy || pending || (!drained && !stop))) break;
    if (busy) {
      prog = true;
      if (hpdi::wide_iter(W)) {
        double lo, hi;
        hpdi::wide_finish(W, lo, hi);
        hpdi_write<true>(io, oitem, W.P.N, lo, hi);
#ifdef MDFIT_DEV_HPTIME
        MDFIT_DEV_T(2 * T + n_items + oitem);
#endif
        busy = false;
      }
    }
    if (!__any(prog)) {  // every lane waits on an entry still being fitted
#ifndef MDFIT_NO_DEFER
      if (kEarly) {
        // the clock is read only on trips without progress (it is a scalar
        // memory round trip): t_wait = when this run of waiting began
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (t_wait == 0) t_wait = now;
        // (the quit flag is read only by waves already waiting an eighth of
        // the bound: a thousand waves polling one line slow every access to its
        // L2 channel)
        if (!keep && (now - t_wait > defer_ticks ||
                      (now - t_wait > defer_ticks / 8 &&
                       __hip_atomic_load(ws + kWsEarlyQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0))) {
          if (defer_items(ws, defer, pending, (int)item)) {
            pending = false;
            stop = true;
          } else {
            keep = true;  // the late launch runs: fit_kernel is done, every entry is published
          }
        }
      }
#endif
      __builtin_amdgcn_s_sleep(8);
    } else {
      t_wait = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// parity / roofline helper kernels
// ---------------------------------------------------------------------------
__global__ void special_kernel(const double* __restrict__ x, int64_t n, double* __restrict__ o) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const LG3 r = lg3<true>(x[i]);  // (the fit kernel's form, the one its parity test covers)
  o[3 * i + 0] = r.l;
  o[3 * i + 1] = r.p;
  o[3 * i + 2] = r.q;
}

__global__ void betabinom_kernel(const double* __restrict__ y, const double* __restrict__ N,
                                 const double* __restrict__ a, const double* __restrict__ b,
                                 int64_t n, double* __restrict__ o, double* __restrict__ g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double k = y[i], m = N[i], al = a[i], be = b[i];
  // value: the cancellation-free form the record assembly uses (bb_logpmf)
  o[i] = bb_logpmf_ab(k, m, al, be, al + be);
  if (g != nullptr) {
    const LG3 t1 = lg3(k + al), t2 = lg3(m - k + be), t3 = lg3(m + al + be);
    const LG3 t4 = lg3(al), t5 = lg3(be), t6 = lg3(al + be);
    const double ps = t6.p - t3.p;
    g[2 * i + 0] = t1.p - t4.p + ps;
    g[2 * i + 1] = t2.p - t5.p + ps;
  }
}

// mdfit_poison_lds: NaN into the whole dynamic LDS of the block
__global__ __launch_bounds__(1024) void poison_lds_kernel(int n_doubles) {
  extern __shared__ double s_poison[];
  for (int i = (int)threadIdx.x; i < n_doubles; i += (int)blockDim.x) s_poison[i] = __longlong_as_double(0x7FF8DEAD0BADF00Dll);
  __syncthreads();
}

// Register-only throughput probe of the fit kernel's point evaluation
// (make_theta + point_accum<kRowPhi>, the row layout of fit_kernel: lane 15 of
// every row a pad): each wave evaluates `iters` times 60 points on a
// representative argument mix (a needs the small-x shift, the others do not --
// as in typical fits).  Useful work: 60 point-evaluations per wave-iteration.
__global__ __launch_bounds__(kWave) void peak_probe_kernel(int iters, double* __restrict__ sink) {
  const int lane = threadIdx.x;
  const int i = lane & 15;
  PointData pd;
  pd.valid = i < kNHalf;
  pd.pmd = true;
  pd.k = pd.valid ? i : 0;
  pd.N = pd.valid ? 1.0e5 + 1000.0 * lane : 0.0;
  pd.y = 0.01 * pd.N;
  double u[4] = {-0.5, -3.0, 0.01, 6.0};
  double acc[kNAcc];
#pragma unroll
  for (int j = 0; j < kNAcc; ++j) acc[j] = 0.0;
  for (int it = 0; it < iters; ++it) {
    const Theta th = make_theta(true, u);
    point_accum<true>(pd, th, acc);
    u[3] += 1e-12 * rowb<0>(acc[0]);  // loop-carried, row-uniform: no hoisting
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < kNAcc; ++j) s += acc[j];
  sink[(int64_t)blockIdx.x * kWave + lane] = s;
}

// Objective / gradient / Hessian of one sub-fit at a given u, evaluated with
// the fit kernel's own layout and code (all-position: lanes 0..31, halves
// summed; forward / reverse: lanes 0..15) -- the parity test of the objective
// itself.  One wave per item; every lane runs (the row-collective pieces).
template <int KIND>
__device__ void objective_group(const uint32_t* gy, const uint32_t* gN, int64_t i, bool pmd,
                                bool rev, const double u[4], double* F, double* g, double* H,
                                double* ell_out) {
  const int lane = threadIdx.x;
  const int r = lane & 31, h = r >> 4, k = r & 15;
  PointData pd;
  pd.pmd = pmd;
  pd.valid = (KIND == kAll ? lane < 32 : lane < 16) && k < kNHalf;
  pd.k = pd.valid ? k : 0;
  const int col = pd.valid ? (KIND == kAll ? h : (rev ? 1 : 0)) * kNHalf + k : 0;
  pd.y = pd.valid ? (double)gy[i * kLD + col] : 0.0;
  pd.N = pd.valid ? (double)gN[i * kLD + col] : 0.0;
  const Theta th = make_theta(pmd, u);
  double acc[kNAcc];
#pragma unroll
  for (int j = 0; j < kNAcc; ++j) acc[j] = 0.0;
  const double ell = point_accum<true>(pd, th, acc);
#pragma unroll
  for (int j = 0; j < kNAcc; ++j) {
    const double s16 = gsum<16>(acc[j]);
    acc[j] = KIND == kAll ? s16 + __shfl_xor(s16, 16, 64) : s16;
  }
  Eval e;
  finish_eval(pmd, th, acc, e);
  if (pd.valid) ell_out[i * kNPos + col] = ell;
  if (lane == 0) {
    F[i] = e.F;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      g[i * 4 + j] = e.g[j];
#pragma unroll
      for (int m = 0; m < 4; ++m) H[i * 16 + 4 * j + m] = e.H[j <= m ? hidx(j, m) : hidx(m, j)];
    }
  }
}

__global__ __launch_bounds__(kWave) void objective_kernel(
    const int32_t* __restrict__ model, const int32_t* __restrict__ subset,
    const uint32_t* __restrict__ gy, const uint32_t* __restrict__ gN, const double* __restrict__ gu,
    int64_t n, double* __restrict__ F, double* __restrict__ g, double* __restrict__ H,
    double* __restrict__ ell_out) {
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  if (threadIdx.x < kNPos) ell_out[i * kNPos + threadIdx.x] = 0.0;
  __syncthreads();
  double u[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = gu[i * 4 + j];
  const bool pmd = model[i] == 0;
  if (subset[i] == 0) objective_group<kAll>(gy, gN, i, pmd, false, u, F, g, H, ell_out);
  else objective_group<kFR>(gy, gN, i, pmd, subset[i] == 2, u, F, g, H, ell_out);
}

}  // namespace mdfit

// ===========================================================================
// C-ABI
// ===========================================================================
namespace mdfit::host {
thread_local char g_err[512] = "";

int set_err(int code, const char* msg) {
  std::snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    std::snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  g_err[0] = '\0';
  return 0;
}
}  // namespace mdfit::host

namespace {
using mdfit::host::check_launch;
using mdfit::host::fit_grid;
using mdfit::host::g_err;
using mdfit::host::set_err;

// optional HIP-event timing of mdfit_fit_batch (mdfit_profile_enable):
// per call, events around the whole call and around fit_kernel, on the
// caller's stream
constexpr int kProfMax = 256;
// measured crossovers (profiles/r03_layout_crossovers.jsonl):
// the 2-points-per-lane layout from 12.5-15k taxa (with the HPDI streamed
// beside the fit), the HPDI after the fit from 50-65k
constexpr int64_t kPpl2MinTaxa = 13000;
constexpr int64_t kStreamMaxTaxa = 60000;
// the HPDI stream's defer list: one int32 per item an early wave hands back;
// a wave defers at most once, at most its 64 lanes' items, so the early grid
// is clamped to kDeferCap / 64 waves (2048: 8 per CU)
constexpr int64_t kDeferCap = 131072;
int64_t defer_cap(int64_t n_taxa) { return std::min<int64_t>(n_taxa * mdfit::kNPos, kDeferCap); }
struct ProfState {
  bool on = false;
  bool fit_only = false;  // mdfit_profile_enable(2): only the events around fit_kernel
  int n = 0;
  hipEvent_t ev[kProfMax][4];
  bool made = false;
};
ProfState g_prof;

void prof_record(int slot, hipStream_t s) {
  if (g_prof.fit_only && (slot == 0 || slot == 3)) return;
  if (g_prof.on && g_prof.n < kProfMax) (void)hipEventRecord(g_prof.ev[g_prof.n][slot], s);
}
}  // namespace

namespace {
// development A/B knobs (environment; unset = the product configuration)
int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

// MAP workspace: the 256-byte header (mdfit::kWs*), then the ready list
// (kReadyStride doubles per taxon); the array entry point (mdfit_hpdi68) puts
// its K4a / K4b wide-window records right after the header
double* ready_buf(void* ws) { return reinterpret_cast<double*>(static_cast<char*>(ws) + 256); }
mdfit::hpdi::WideRec* hpdi_recs(void* ws) {
  return reinterpret_cast<mdfit::hpdi::WideRec*>(static_cast<char*>(ws) + 256);
}
// (the fit's K4a / K4b path from kStreamMaxTaxa taxa: after the ready list)
mdfit::hpdi::WideRec* hpdi_recs_after_ready(void* ws, int64_t n_taxa) {
  return reinterpret_cast<mdfit::hpdi::WideRec*>(static_cast<char*>(ws) + 256 +
                                                 n_taxa * mdfit::kReadyStride * (int64_t)sizeof(double));
}

// The side streams of mdfit_fit_batch's forks -- [0] the early HPDI stream
// launch beside the fit kernel, [1] the second fork after the fit (below 60k
// taxa the late HPDI launch beside the record assembly, from 60k the record
// assembly beside K4a -> K4b) --
// and their fork / join events: one set per device, created on first use and
// kept for the process (bounded: 2 streams per device, not per calling host
// thread); the streams non-blocking (ordered against the caller's stream by the
// events only).  The events are shared, so a call holds the device's mutex from
// its first fork record to its last join wait: a wait binds to the record
// enqueued before it, and another thread's record in between would rebind it.
struct Fork {
  hipStream_t s[2] = {nullptr, nullptr};
  hipEvent_t fork[2] = {nullptr, nullptr}, join[2] = {nullptr, nullptr};
  bool ok = false;
  std::mutex mu;
};
Fork* side_fork() {
  constexpr int kMaxDev = 64;
  static Fork f[kMaxDev];
  static std::mutex make_mu;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  Fork& x = f[dev];
  std::lock_guard<std::mutex> g(make_mu);
  if (!x.ok) {
    bool ok = true;
    for (int k = 0; k < 2 && ok; ++k)
      ok = (x.s[k] != nullptr || hipStreamCreateWithFlags(&x.s[k], hipStreamNonBlocking) == hipSuccess) &&
           (x.fork[k] != nullptr || hipEventCreateWithFlags(&x.fork[k], hipEventDisableTiming) == hipSuccess) &&
           (x.join[k] != nullptr || hipEventCreateWithFlags(&x.join[k], hipEventDisableTiming) == hipSuccess);
    if (!ok) return nullptr;  // (what was created is kept for the next try)
    x.ok = true;
  }
  return &x;
}

// One fork's scope: when opened, joins side stream k back into the caller's
// stream on EVERY exit of mdfit_fit_batch -- error returns included -- so no
// kernel of the call is still running on a side stream when the caller (whose
// allocator orders frees against its own stream only) gets control back, and a
// graph capture never ends with an open fork.  (The device's mutex is held by
// the call around all its forks.)
struct ForkScope {
  Fork* fk;
  hipStream_t s;
  int k;
  bool open = false;
  ForkScope(Fork* f, hipStream_t st, int which) : fk(f), s(st), k(which) {
    if (fk == nullptr) return;
    open = hipEventRecord(fk->fork[k], s) == hipSuccess && hipStreamWaitEvent(fk->s[k], fk->fork[k], 0) == hipSuccess;
  }
  hipStream_t side() const { return open ? fk->s[k] : s; }  // no side stream: everything in order on s
  int join() {
    if (!open) return 0;
    open = false;
    if (hipEventRecord(fk->join[k], fk->s[k]) != hipSuccess || hipStreamWaitEvent(s, fk->join[k], 0) != hipSuccess)
      return set_err(MDFIT_E_HIP, "stream join");
    return 0;
  }
  ~ForkScope() { (void)join(); }
};

// K4a (unless the fit kernel did its work: prep = false) and K4b
template <bool kFit>
int launch_hpdi(const mdfit::HpdiIO& io, int64_t n_items, int* ctr, mdfit::hpdi::WideRec* recs, hipStream_t s,
                bool prep = true) {
  if (n_items == 0) return 0;
  if (prep) {
    mdfit::host::debug_poison(s);
    hipLaunchKernelGGL(mdfit::hpdi_prep_kernel<kFit>,
                       dim3((unsigned)((n_items + mdfit::kPrepBlock - 1) / mdfit::kPrepBlock)), dim3(mdfit::kPrepBlock),
                       0, s, io, n_items, ctr, recs);
    if (int rc = check_launch("hpdi_prep_kernel")) return rc;
  }
  // no more waves than are resident, and no more than the items need (the
  // kernel strides over the wide list, whose length only the device knows)
  const int64_t g = fit_grid(mdfit::hpdi_wide_kernel<kFit>, n_items, mdfit::kWave, env_int("MDFIT_HPDI_WAVES_PER_CU", 0));
  mdfit::host::debug_poison(s);
  hipLaunchKernelGGL(mdfit::hpdi_wide_kernel<kFit>, dim3((unsigned)g), dim3(mdfit::kWave), 0, s, io, n_items, ctr,
                     recs);
  return check_launch("hpdi_wide_kernel");
}
}  // namespace

void mdfit::host::prof_mark(int slot, hipStream_t s) { prof_record(slot, s); }

extern "C" {

#ifdef MDFIT_DEV_HPTIME
int mdfit_dev_set_hptime(unsigned long long* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dev_hpt), &buf, sizeof(buf)) != hipSuccess;
}
#endif

int mdfit_profile_enable(int on) {
  if (on && !g_prof.made) {
    for (int i = 0; i < kProfMax; ++i)
      for (int j = 0; j < 4; ++j)
        if (hipEventCreate(&g_prof.ev[i][j]) != hipSuccess) return set_err(MDFIT_E_HIP, "hipEventCreate");
    g_prof.made = true;
  }
  g_prof.on = on != 0;
  g_prof.fit_only = on == 2;
  g_prof.n = 0;
  return 0;
}

int mdfit_profile_read(double* call_ms, double* fit_ms, int32_t* n_calls) {
  if (!call_ms || !fit_ms || !n_calls) return set_err(MDFIT_E_ARG, "null argument");
  double a = 0.0, b = 0.0;
  for (int i = 0; i < g_prof.n; ++i) {
    float x = 0.f, y = 0.f;
    if (hipEventSynchronize(g_prof.ev[i][2]) != hipSuccess ||
        (!g_prof.fit_only && (hipEventSynchronize(g_prof.ev[i][3]) != hipSuccess ||
                              hipEventElapsedTime(&x, g_prof.ev[i][0], g_prof.ev[i][3]) != hipSuccess)) ||
        hipEventElapsedTime(&y, g_prof.ev[i][1], g_prof.ev[i][2]) != hipSuccess)
      return set_err(MDFIT_E_HIP, "hipEventElapsedTime");
    a += x;
    b += y;
  }
  *call_ms = g_prof.fit_only ? -1.0 : a;  // not recorded in fit-only mode
  *fit_ms = b;
  *n_calls = g_prof.n;
  g_prof.n = 0;
  return 0;
}

void mdfit_default_opts(mdfit_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->mode = MDFIT_MODE_MAP;
  o->max_iter = 200;
  o->tol_step = 1e-9;
  o->seed = 0;
  o->num_warmup = 500;
  o->num_samples = 1000;
  o->index_base = 0;
}

int64_t mdfit_workspace_bytes(int64_t n_taxa, const mdfit_opts* opts) {
  if (n_taxa < 0) return 0;
  mdfit_opts o;
  mdfit_default_opts(&o);
  if (opts) o = *opts;
  if (o.mode == MDFIT_MODE_NUTS) return mdfit::nuts::workspace_bytes(n_taxa, o.num_samples);
  // the 256-byte header (counters, flags), then the ready list of
  // PMD-all modes (48 B per taxon); from kStreamMaxTaxa taxa (the HPDI after
  // the fit, K4a -> K4b) room for every position's wide-window record
  // (+ the HPDI stream's defer list at the end)
  return 256 + n_taxa * mdfit::kReadyStride * (int64_t)sizeof(double) +
         (n_taxa >= kStreamMaxTaxa ? n_taxa * mdfit::kNPos * (int64_t)sizeof(mdfit::hpdi::WideRec) : 0) +
         defer_cap(n_taxa) * (int64_t)sizeof(int);
}

int mdfit_fit_batch(const uint32_t* y, const uint32_t* N, const uint32_t* mm, int64_t n_taxa,
                    const mdfit_opts* opts, double* out, float* pred, int32_t* status,
                    void* workspace, void* hip_stream) {
  if (n_taxa < 0) return set_err(MDFIT_E_ARG, "n_taxa < 0");
  if (n_taxa == 0) return 0;
  if (!y || !N || !out || !status) return set_err(MDFIT_E_ARG, "null required pointer");
  if (!workspace) return set_err(MDFIT_E_ARG, "workspace (mdfit_workspace_bytes() bytes) required");
  mdfit_opts o;
  mdfit_default_opts(&o);
  if (opts) o = *opts;
  if (o.mode != MDFIT_MODE_MAP && o.mode != MDFIT_MODE_NUTS) return set_err(MDFIT_E_ARG, "unsupported mode");
  if (o.max_iter < 1) return set_err(MDFIT_E_ARG, "max_iter < 1");
  // the HPDI item counters are int32 over T * 30 positions: 2^25 taxa (1e9
  // positions) per call at most
  if (n_taxa > ((int64_t)1 << 25)) return set_err(MDFIT_E_ARG, "n_taxa exceeds 2^25 per call");
  hipStream_t s = (hipStream_t)hip_stream;
  int* ws = (int*)workspace;
  prof_record(0, s);
  if (o.mode == MDFIT_MODE_NUTS) {
    if (hipMemsetAsync(ws, 0, 256, s) != hipSuccess) return check_launch("hipMemsetAsync(workspace)");
    if (int rc = mdfit::nuts::fit_batch(y, N, mm, n_taxa, o, out, pred, status, workspace, s)) return rc;
    prof_record(3, s);
    if (g_prof.on && g_prof.n < kProfMax) ++g_prof.n;
    return 0;
  }
  const int64_t n_init = MDFIT_NSUBFIT * n_taxa;
  // (MDFIT_DEBUG_POISON_LDS: on the caller's stream ahead of K0, so the early
  // HPDI launch on the side stream starts on the poisoned LDS without the
  // poison grid delaying it past its wait for the fit kernel's start)
  mdfit::host::debug_poison(s);
  hipLaunchKernelGGL(mdfit::init_kernel, dim3((unsigned)((n_init + 255) / 256)), dim3(256), 0, s, y, N,
                     n_taxa, out, ws);
  if (int rc = check_launch("init_kernel")) return rc;
  // lane layout of the fit kernel (bitwise-identical results): 2 points per
  // lane for batches that fill the chip several times over, 1 below (lower
  // latency per evaluation).  MDFIT_FIT_PPL=1|2 overrides (development A/B).
  int ppl = n_taxa >= kPpl2MinTaxa ? 2 : 1;
  if (const char* e = std::getenv("MDFIT_FIT_PPL")) ppl = std::atoi(e) == 2 ? 2 : 1;
  const int per = pred != nullptr ? mdfit::kNPos : 1;
  const int64_t n_items = n_taxa * per;
  double* ready = ready_buf(workspace);
  // the call's forks share the device's events: hold its mutex throughout
  // (declared before the scopes, so it is released after their joins)
  Fork* fk = side_fork();
  std::unique_lock<std::mutex> fork_lock;
  if (fk != nullptr) fork_lock = std::unique_lock<std::mutex>(fk->mu);
  // K4 (early): the predictive HPDI streamed beside the fit kernel, on side
  // stream 0 from after K0; its grid -- MDFIT_STREAM_WAVES_PER_CU waves per CU
  // -- is the room the fit kernel's grid leaves
  // The HPDI streams beside the fit below kStreamMaxTaxa taxa -- the regime where
  // the call is bounded by the fit kernel's tail, which the stream fills --
  // and runs after the fit from there (the fit kernel fills the chip by itself;
  // K4a -> K4b at full occupancy, longest windows first).  MDFIT_HPDI_STREAM=1
  // streams at any size (A/B; the workspace has no wide-window list below).
  bool stream = n_taxa < kStreamMaxTaxa;
  if (const char* e = std::getenv("MDFIT_HPDI_STREAM")) stream = stream || std::atoi(e) != 0;
  const int early_per_cu =
      (fk != nullptr && stream) ? env_int("MDFIT_STREAM_WAVES_PER_CU", MDFIT_STREAM_WAVES_PER_CU) : 0;
  // the defer list ends the workspace (mdfit_workspace_bytes); an early wave
  // that waited defer_us without progress hands its items to the late launch
  int* defer = reinterpret_cast<int*>(static_cast<char*>(workspace) + mdfit_workspace_bytes(n_taxa, &o) -
                                      defer_cap(n_taxa) * (int64_t)sizeof(int));
  const uint32_t defer_ticks = (uint32_t)std::max(0, env_int("MDFIT_STREAM_DEFER_US", 1000)) * 100u;
  ForkScope fork_hp(early_per_cu > 0 ? fk : nullptr, s, 0);
  if (early_per_cu > 0) {
    const int64_t g = std::min<int64_t>(fit_grid(mdfit::hpdi_stream_kernel<true>, n_items, mdfit::kWave, early_per_cu),
                                        kDeferCap / mdfit::kWave);
    hipLaunchKernelGGL(mdfit::hpdi_stream_kernel<true>, dim3((unsigned)g), dim3(mdfit::kWave), 0, fork_hp.side(), N,
                       n_taxa, per, out, pred, ws, (const double*)ready, defer, defer_ticks);
    if (int rc = check_launch("hpdi_stream_kernel")) return rc;
  }
  prof_record(1, s);
  {
    // fit waves above the HPDI stream's (whose waves then take the issue slots
    // the fits leave): C2 1.42 -> 1.23 ms with 4 stream waves per CU
    const int fit_prio = env_int("MDFIT_FIT_BASE_PRIO", 1) != 0 ? 1 : 0;
    int occ = 8;  // waves per CU the fit kernel may take: its occupancy, less the HPDI stream's
    const int cap_env = env_int("MDFIT_FIT_WAVES_PER_CU", 0);
    if (ppl == 2) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, mdfit::fit_kernel<2>, mdfit::kWave, 0) != hipSuccess) occ = 8;
      const int cap = cap_env > 0 ? cap_env : std::max(1, occ - early_per_cu);
      const int64_t g = fit_grid(mdfit::fit_kernel<2>, 2 * n_taxa, 4, cap);
      hipLaunchKernelGGL(mdfit::fit_kernel<2>, dim3((unsigned)g), dim3(mdfit::kWave), 0, s, y, N, n_taxa,
                         o.max_iter, o.tol_step, out, ws, ready, fit_prio);
    } else {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, mdfit::fit_kernel<1>, mdfit::kWave, 0) != hipSuccess) occ = 8;
      const int cap = cap_env > 0 ? cap_env : std::max(1, occ - early_per_cu);
      const int64_t g = fit_grid(mdfit::fit_kernel<1>, 2 * n_taxa, 2, cap);
      hipLaunchKernelGGL(mdfit::fit_kernel<1>, dim3((unsigned)g), dim3(mdfit::kWave), 0, s, y, N, n_taxa,
                         o.max_iter, o.tol_step, out, ws, ready, fit_prio);
    }
  }
  if (int rc = check_launch("fit_kernel")) return rc;
  prof_record(2, s);
  // then a fork onto side stream 1: the record assembly (K3) and the HPDI's
  // late launch / K4a -> K4b run side by side; they write disjoint fields of
  // the record and join before the call returns
  ForkScope fork_as(fk, s, 1);
  // Below kStreamMaxTaxa the record assembly follows the fit on the caller's
  // stream (it starts as soon as the fit ends; on the side stream it waited
  // ~30 us longer for the fork event) and the HPDI's late launch -- a short
  // drain of what the early launch left -- takes the side stream.  From
  // kStreamMaxTaxa the HPDI (K4a -> K4b) is the long part and keeps the
  // caller's stream.
  const bool asm_main = stream;
  const hipStream_t s_asm = asm_main ? s : fork_as.side();
  const hipStream_t s_hp = asm_main ? fork_as.side() : s;
  mdfit::host::debug_poison(s_asm);
  hipLaunchKernelGGL(mdfit::assemble_kernel, dim3((unsigned)n_taxa), dim3(mdfit::kWave), 0, s_asm, y, N,
                     mm, n_taxa, out, pred, status);
  if (int rc = check_launch("assemble_kernel")) return rc;
  if (stream) {
    const int64_t g = fit_grid(mdfit::hpdi_stream_kernel<false>, n_items, mdfit::kWave,
                               env_int("MDFIT_HPDI_WAVES_PER_CU", 0));
    mdfit::host::debug_poison(s_hp);
    hipLaunchKernelGGL(mdfit::hpdi_stream_kernel<false>, dim3((unsigned)g), dim3(mdfit::kWave), 0, s_hp, N, n_taxa, per,
                       out, pred, ws, (const double*)ready, defer, defer_ticks);
    if (int rc = check_launch("hpdi_stream_kernel")) return rc;
  } else {
    mdfit::HpdiIO io{};
    io.gN = N;
    io.ready = ready;
    io.out = out;
    io.pred = pred;
    io.per = per;
    if (int rc = launch_hpdi<true>(io, n_items, ws + mdfit::kHpdiCtr, hpdi_recs_after_ready(workspace, n_taxa), s))
      return rc;
  }
  if (int rc = fork_as.join()) return rc;
  if (int rc = fork_hp.join()) return rc;
  prof_record(3, s);
  if (g_prof.on && g_prof.n < kProfMax) ++g_prof.n;
  return 0;
}

int mdfit_noise(const uint32_t* y, const uint32_t* N, const uint32_t* mm, int64_t n_taxa, double* out,
                void* hip_stream) {
  if (n_taxa < 0 || (n_taxa > 0 && (!y || !N || !mm || !out))) return set_err(MDFIT_E_ARG, "bad arguments");
  if (n_taxa == 0) return 0;
  hipLaunchKernelGGL(mdfit::noise_kernel, dim3((unsigned)n_taxa), dim3(mdfit::kWave), 0, (hipStream_t)hip_stream, y,
                     N, mm, n_taxa, out);
  return check_launch("noise_kernel");
}

int mdfit_betabinom_logpmf(const double* y, const double* N, const double* alpha,
                           const double* beta, int64_t n, double* out, double* grad,
                           void* hip_stream) {
  if (n < 0 || (n > 0 && (!y || !N || !alpha || !beta || !out)))
    return set_err(MDFIT_E_ARG, "bad arguments");
  if (n == 0) return 0;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(mdfit::betabinom_kernel, dim3(blocks), dim3(256), 0,
                     (hipStream_t)hip_stream, y, N, alpha, beta, n, out, grad);
  return check_launch("betabinom_kernel");
}

#ifdef MDFIT_HPDI_COUNT
// diagnostic: read (and zero) the HPDI loop counters
int mdfit_hpdi_counts(unsigned long long* out32) {
  if (hipMemcpyFromSymbol(out32, HIP_SYMBOL(mdfit::hpdi::g_hpdi_cnt), 256) != hipSuccess) return 1;
  const unsigned long long z[32] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(mdfit::hpdi::g_hpdi_cnt), z, 256) != hipSuccess;
}
#endif

int mdfit_hpdi68(const double* N, const double* alpha, const double* beta, int64_t n, double* lo,
                 double* hi, void* hip_stream) {
  if (n < 0 || (n > 0 && (!N || !alpha || !beta || !lo || !hi))) return set_err(MDFIT_E_ARG, "bad arguments");
  if (n == 0) return 0;
  hipStream_t s = (hipStream_t)hip_stream;
  void* ws = nullptr;
  const size_t bytes = 256 + (size_t)n * sizeof(mdfit::hpdi::WideRec);
  if (hipMallocAsync(&ws, bytes, s) != hipSuccess) return set_err(MDFIT_E_HIP, "hipMallocAsync");
  if (hipMemsetAsync(ws, 0, 256, s) != hipSuccess) return set_err(MDFIT_E_HIP, "hipMemsetAsync");
  mdfit::HpdiIO io{};
  io.N = N;
  io.a = alpha;
  io.b = beta;
  io.lo = lo;
  io.hi = hi;
  int rc = launch_hpdi<false>(io, n, static_cast<int*>(ws) + mdfit::kHpdiCtr, hpdi_recs(ws), s);
  (void)hipFreeAsync(ws, s);
  return rc;
}

int mdfit_special(const double* x, int64_t n, double* out3, void* hip_stream) {
  if (n < 0 || (n > 0 && (!x || !out3))) return set_err(MDFIT_E_ARG, "bad arguments");
  if (n == 0) return 0;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(mdfit::special_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)hip_stream,
                     x, n, out3);
  return check_launch("special_kernel");
}

int mdfit_poison_lds(void* hip_stream) {
  int dev = 0, n_cu = 256, lds_block = 65536, lds_cu = 163840;
  if (hipGetDevice(&dev) != hipSuccess) return set_err(MDFIT_E_HIP, "hipGetDevice");
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipDeviceGetAttribute(&lds_block, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
  (void)hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
  lds_block = std::max(1024, std::min(lds_block, lds_cu));
  const int per_cu = std::max(1, lds_cu / lds_block);
  // several rounds of blocks per CU: every CU gets blocks whatever the dispatch order
  hipLaunchKernelGGL(mdfit::poison_lds_kernel, dim3((unsigned)(4 * n_cu * per_cu)), dim3(1024), (size_t)lds_block,
                     (hipStream_t)hip_stream, lds_block / (int)sizeof(double));
  return check_launch("poison_lds_kernel");
}

}  // extern "C" (reopened below)

void mdfit::host::debug_poison(hipStream_t s) {
  const char* e = std::getenv("MDFIT_DEBUG_POISON_LDS");
  if (e != nullptr && std::atoi(e) != 0) (void)mdfit_poison_lds(s);
}

extern "C" {

int mdfit_peak_probe(int64_t n_waves, int32_t iters, double* sink, void* hip_stream) {
  if (n_waves <= 0 || iters <= 0 || !sink) return set_err(MDFIT_E_ARG, "bad arguments");
  hipLaunchKernelGGL(mdfit::peak_probe_kernel, dim3((unsigned)n_waves), dim3(mdfit::kWave), 0,
                     (hipStream_t)hip_stream, iters, sink);
  return check_launch("peak_probe_kernel");
}

int mdfit_objective(const int32_t* model, const int32_t* subset, const uint32_t* y,
                    const uint32_t* N, const double* u, int64_t n, double* F, double* g,
                    double* H, double* ell, void* hip_stream) {
  if (n < 0 || (n > 0 && (!model || !subset || !y || !N || !u || !F || !g || !H || !ell)))
    return set_err(MDFIT_E_ARG, "bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(mdfit::objective_kernel, dim3((unsigned)n), dim3(mdfit::kWave), 0,
                     (hipStream_t)hip_stream, model, subset, y, N, u, n, F, g, H, ell);
  return check_launch("objective_kernel");
}

#ifdef MDFIT_STAMP
int mdfit_set_stamp(unsigned long long* buf) {
  hipMemcpyToSymbol(HIP_SYMBOL(mdfit::g_stamp), &buf, sizeof(buf));
  return 0;
}
#endif

int mdfit_nuts_potential(const int32_t* model, const int32_t* subset, const uint32_t* y, const uint32_t* N,
                         const double* v, int64_t n, double* U, double* g, void* hip_stream) {
  if (n < 0 || (n > 0 && (!model || !subset || !y || !N || !v || !U || !g)))
    return set_err(MDFIT_E_ARG, "bad arguments");
  return mdfit::nuts::potential(model, subset, y, N, v, n, U, g, (hipStream_t)hip_stream);
}

int mdfit_nuts_peak_probe(int64_t n_waves, int32_t iters, double* sink, void* hip_stream) {
  if (n_waves <= 0 || iters <= 0 || !sink) return set_err(MDFIT_E_ARG, "bad arguments");
  return mdfit::nuts::peak_probe(n_waves, iters, sink, (hipStream_t)hip_stream);
}

const char* mdfit_last_error(void) { return g_err; }

int mdfit_abi_version(void) { return MDFIT_ABI_VERSION; }

}  // extern "C"
