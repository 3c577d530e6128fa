// mdfit_nuts.hip — MI355X (gfx950) sampling mode: MDFIT-NUTS v1.
//
// The reference samples every sub-fit with numpyro NUTS (fits.py:382-387,
// num_warmup 500 / num_samples 1000, one chain) and post-processes the draws
// (fits.py:89-172, 230-356).  Two launches:
//
//   nuts_chain_cd      persistent, component-distributed: a 16-lane slot is
//                      one chain (an all-position chain two slots), lane =
//                      position (lane 15 of a row a pad), and lane i also
//                      holds component i & 3 of the chain's 4-vectors.  Every
//                      trip every running chain does ONE potential + gradient
//                      evaluation -- a leapfrog step, an initial-point probe
//                      or a step-size-search step -- and then advances its
//                      state machine (iterative NUTS tree, Stan-window
//                      adaptation).  Kept draws go to the workspace:
//                      double[T][6][S][4] = (q, A, c, phi).
//   nuts_post_kernel   one wave per taxon, lanes over draws: pointwise
//                      log-likelihood -> lppd / pWAIC / waic_i, n_sigma x3,
//                      asymmetry, posterior means, predictive Beta-Binomial
//                      draws -> median / 68 % HPDI by a bitonic sort in LDS,
//                      sums, noise.
//
// Same algorithm and the same Philox4x32-10 streams as oracle/mdfit_nuts.c
// (written separately; see its header for the counter layout), so GPU chains
// follow the oracle's draw for draw until a floating-point difference flips
// a decision.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/mdfit.h"
#include "mdfit_host.h"
#include "mdfit_model.h"
#include "mdfit_special.h"

namespace mdfit::nuts {

#ifdef MDFIT_STAMP
// diagnostic build (-DMDFIT_STAMP): per-wave cycle split of the chain loop
// (tools/nuts_stamp_profile.py).  The wave clock (s_memtime) is written to LDS
// by whichever lanes reach a point; the loop top (converged) books the split of
// the previous trip.  Never quote this build's run time.
__device__ unsigned long long* g_nuts_stamp = nullptr;
__device__ __forceinline__ unsigned long long nstamp() {
  __builtin_amdgcn_sched_barrier(0);
  unsigned long long t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define NSTAMP(k) (sstamp[k] = nstamp())
#else
#define NSTAMP(k) ((void)0)
#endif

constexpr int kMaxDepth = 10;
constexpr double kMaxDelta = 1000.0;
constexpr double kTarget = 0.8;
constexpr double kTiny = 2.2250738585072014e-308;
constexpr double kHuge = 1.7976931348623157e308;
constexpr int kMaxSamples = 4096;  // LDS bound of the post kernel
constexpr int kMaxWin = 16;        // adaptation windows (windows() stops at 15 + the terminal one)

// ---------------------------------------------------------------------------
// Philox4x32-10 and the draw helpers (oracle: philox4x32, nuniform, nnormal)
// ---------------------------------------------------------------------------
struct Stream {
  uint32_t k0, k1, c0, c1;
};

__device__ __forceinline__ Stream make_stream(uint64_t seed, int64_t g, int sub) {
  Stream s;
  s.k0 = (uint32_t)seed;
  s.k1 = (uint32_t)(seed >> 32);
  s.c0 = (uint32_t)(uint64_t)g;
  s.c1 = (uint32_t)((uint64_t)g >> 32) + ((uint32_t)sub << 24);
  return s;
}

#ifndef MDFIT_PHILOX_MAD
#define MDFIT_PHILOX_MAD 0
#endif
__device__ __forceinline__ uint4 block(const Stream& s, uint32_t w2, uint32_t w3) {
  uint32_t c0 = s.c0, c1 = s.c1, c2 = w2, c3 = w3, k0 = s.k0, k1 = s.k1;
  // The key is the seed in every stream (make_stream), so it is wave-uniform:
  // held in SGPRs and opaque here, so the round-key schedule is recomputed on
  // the scalar unit at each call instead of being hoisted out of the chain
  // loop as 20 loop-invariant SGPRs (which the chain kernels spill to VGPR lanes).
  k0 = __builtin_amdgcn_readfirstlane(k0);
  k1 = __builtin_amdgcn_readfirstlane(k1);
  asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
#if MDFIT_PHILOX_MAD  // one v_mad_u64_u32 per product (hi and lo together)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#else
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
#endif
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {  // [0, 1)
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ double uniform(const Stream& s, uint32_t w2, uint32_t w3) {
  const uint4 o = block(s, w2, w3);
  return u53(o.x, o.y);
}

// (not inlined: their log / sincos / sqrt temporaries then stay out of the chain
// loop's register allocation -- fewer spills on the hot path)
// normal k of the Box-Muller pair of one block (k = 0: cos, 1: sin; oracle:
// nnormal_k) -- the chain's momenta (draw convention 2)
__device__ __noinline__ double normal_k(const Stream& s, uint32_t w2, uint32_t w3, int k) {
  const uint4 o = block(s, w2, w3);
  const double u1 = 1.0 - u53(o.x, o.y), u2 = u53(o.z, o.w);
  double sn, cs;
  sincos(6.283185307179586 * u2, &sn, &cs);
  return sqrt(-2.0 * log(u1)) * (k ? sn : cs);
}
// both normals of the pair
__device__ __noinline__ double2 normal_pair(const Stream& s, uint32_t w2, uint32_t w3) {
  const uint4 o = block(s, w2, w3);
  const double u1 = 1.0 - u53(o.x, o.y), u2 = u53(o.z, o.w);
  double sn, cs;
  sincos(6.283185307179586 * u2, &sn, &cs);
  const double r = sqrt(-2.0 * log(u1));
  return make_double2(r * cs, r * sn);
}
// (MDFIT_POST_FAST) the post kernel's transcendentals by the table forms:
// the WAIC's log-sum-exp exponentials and the predictive draws' exponentials
// and logs (positive normal arguments; absolute accuracy ~1e-16 near 1, which
// is what their comparisons and the draws need) -- fexp_t / flog_t for the
// library's exp / log
#ifndef MDFIT_POST_FAST
#define MDFIT_POST_FAST 1
#endif
// (MDFIT_WAIC_GROUP) the null sub-fits' WAIC takes G columns per pass over the
// draws: a, b and a + b do not depend on the column there (D = q), so their
// three lnGamma values are formed once per draw for G columns -- the same
// values in the same expression, bit for bit (1: one column per pass)
#ifndef MDFIT_WAIC_GROUP
#define MDFIT_WAIC_GROUP 3
#endif
// the post kernel's occupancy floor (waves per SIMD; LDS allows ~6): 5 leaves
// the grouped WAIC 96 VGPRs (26 spilled); at 6 it spills 44 and runs slower,
// unbounded it takes 118 (4 waves), also slower (profiles/r06_ab_waic.txt)
#ifndef MDFIT_POST_WAVES
#define MDFIT_POST_WAVES 5
#endif
// (MDFIT_REG_SORT) the predictive counts of 513..1024 draws sorted in
// registers (reg_sort_u32); else the LDS bitonic sort
#ifndef MDFIT_REG_SORT
#define MDFIT_REG_SORT 1
#endif
#ifndef MDFIT_NUTS_SST
#define MDFIT_NUTS_SST 1
#endif
__device__ __forceinline__ double pexp(double x) { return MDFIT_POST_FAST ? fexp_t(x) : exp(x); }
__device__ __forceinline__ double plog(double x) { return MDFIT_POST_FAST ? flog_t<true>(x) : log(x); }

__device__ __forceinline__ bool active(bool pmd, int j) { return pmd || j == 0 || j == 3; }

// out[j] = v of lane j of this chain slot (G = 16: a DPP row; G = 8: one half
// of it) -- the slot's lanes 0-3 each computed one component of a 4-vector;
// the row must be converged
template <int G>
__device__ __forceinline__ void slot4(double v, double out[4]) {
  if (G == 16) {
    out[0] = rowb<0>(v);
    out[1] = rowb<1>(v);
    out[2] = rowb<2>(v);
    out[3] = rowb<3>(v);
  } else {
    const bool hi8 = threadIdx.x & 8;
    out[0] = hi8 ? rowb<8>(v) : rowb<0>(v);
    out[1] = hi8 ? rowb<9>(v) : rowb<1>(v);
    out[2] = hi8 ? rowb<10>(v) : rowb<2>(v);
    out[3] = hi8 ? rowb<11>(v) : rowb<3>(v);
  }
}

// ---------------------------------------------------------------------------
// adaptation schedule (oracle: adapt_windows) -- end of window w, or -1
// ---------------------------------------------------------------------------
__device__ __forceinline__ void windows(int nw, int w, int* end_w, int* nwin) {
  int n = 0, e = -1;
  if (nw < 20) {
    *end_w = w == 0 ? nw - 1 : -1;
    *nwin = 1;
    return;
  }
  int init_buffer = 75, term_buffer = 50, base_window = 25;
  if (nw < init_buffer + term_buffer + base_window) {
    init_buffer = (int)(0.15 * nw);
    term_buffer = (int)(0.1 * nw);
    base_window = nw - init_buffer - term_buffer;
  }
  if (w == n) e = init_buffer - 1;
  n++;
  const int end_start = nw - term_buffer;
  int next_size = base_window, next_start = init_buffer;
  while (next_start < end_start && n < 15) {
    const int cs = next_start;
    int csz = next_size;
    if (3 * csz <= end_start - cs) next_size = 2 * csz;
    else csz = end_start - cs;
    next_start = cs + csz;
    if (w == n) e = next_start - 1;
    n++;
  }
  if (w == n) e = nw - 1;
  *end_w = e;
  *nwin = n + 1;
}

// checkpoint index range of leaf n (oracle: ckpt_idxs)
__device__ __forceinline__ void ckpt_idxs(int n, int* imin, int* imax) {
  const int mx = __popc((unsigned)(n >> 1));
  const int ns = __builtin_ctz(~(unsigned)n);  // trailing ones
  *imax = mx;
  *imin = mx - ns + 1;
}

constexpr int kInit = 1, kFind = 2, kIter = 3, kDone = 4;

// ---------------------------------------------------------------------------
// chain kernel, component-distributed layout
// ---------------------------------------------------------------------------
// A 16-lane slot runs one chain; a task group of two slots runs one
// all-position chain (both slots hold identical state, their sums added) or the
// forward / reverse pair of one model (a chain per slot).  The chain's
// 4-vectors (position, momentum, gradient, inverse mass, momentum sums, the
// trajectory ends and proposals) are held one component per lane: lane i of a
// slot holds component i & 3 (the slot's quads hold copies).  A leapfrog is
// then 3 instructions, a vector costs 2 VGPRs, and the hot chain state
// (dynamics, subtree, step size, counters) lives in registers; the cold vectors
// (trajectory ends, proposals, Welford) are per-slot LDS arrays of 4.  Dot
// products (kinetic energy, U-turn criteria) gather the four components and
// add them in the oracle's order without contraction (oracle/mdfit_nuts.c:
// kinetic, is_turning).  A wave serves its XCD's task queue, then the other
// queues in turn once that one runs dry.
// a wave whose chain has run long takes issue priority over its SIMD's other
// waves (s_setprio 1 / 2 / 3 past 32k / 64k / 128k wave-trips since the chain
// started): the kernel ends with its longest chain (C3: 2-4.5e5 trips, ~15 us
// a trip at full load, 4.8 s -- as long as the call), so those trips are the
// critical path; checked every 256 trips
#ifndef MDFIT_NUTS_PRIO
#define MDFIT_NUTS_PRIO 1
#endif
#ifndef MDFIT_NUTS_PRIO_T
#define MDFIT_NUTS_PRIO_T 32768.0  // trips of the first level (x2, x4 for the next)
#endif
#ifndef MDFIT_NUTS_CD_WAVES
#define MDFIT_NUTS_CD_WAVES 4  // 128 VGPRs, no spill with MachineLICM off (build_hip)
#endif

// The multinomial weights of an iteration's trajectory (MDFIT_NUTS_LINW):
// numpyro / the oracle carry the tree's and the subtree's log-weights and
// combine them by log-sum-exp (an exp and a log per leaf and per merge, and
// another exp for the acceptance statistic).  Here they are linear, relative
// to the iteration's largest log-weight so far w_ref (>= 0: the initial
// point's is 0): a leaf of log-weight w adds exp(w - w_ref), or, when it is
// the new largest, rescales the tree's and the subtree's sums by
// exp(w_ref - w) -- one exp per leaf either way, which is also the leaf's
// acceptance probability min(1, e^w) while w_ref = 0; the progressive
// sampling probabilities are ratios of the sums (one reciprocal), the merge
// an add.  Mathematically the oracle's numbers; a decision differs only when
// a uniform falls within rounding of a probability.
#ifndef MDFIT_NUTS_LINW
#define MDFIT_NUTS_LINW 1
#endif
// (MDFIT_NUTS_EREF) and the acceptance probability e^w of a leaf below zero
// after a rescale as its linear weight times exp(w_ref) -- kept as the
// product of the rescale factors' reciprocals -- instead of a second exp;
// beyond w_ref = 700 (the product's range) the exp
#ifndef MDFIT_NUTS_EREF
#define MDFIT_NUTS_EREF 1
#endif
// the sampler's exponentials: the table exp (fexp_t, ~1 ulp) or the library's
#ifndef MDFIT_TEXP
#define MDFIT_TEXP 1
#endif
__device__ __forceinline__ double nexp(double x) { return MDFIT_TEXP ? fexp_t(x) : exp(x); }


// ln(1 + e) of the multinomial weights' log-sum-exp, e = exp(-|w1 - w2|) in
// [0, 1]: the log-weights enter only through exp differences, so absolute
// accuracy is what counts, and the fast form takes the table log of the
// rounded 1 + e (absolute error <= 1.2e-16; MDFIT_TLOG_NUTS)
__device__ __forceinline__ double lae1p(double e) { return MDFIT_TLOG_NUTS ? flog_t(1.0 + e) : flog1p(e); }

struct PotC {
  double U;
  double g;  // this lane's component of the gradient
};

// -(log density + log|J|) of the slot's (or, `whole`, the task group's) points
// at x and its gradient (oracle: nuts_potential), with the input and the
// gradient component-distributed: every lane resolves its own component (c < 3:
// sigmoid, c == 3: exp), lanes 0-3 of the slot are broadcast; the phi pair is
// the pad lane's lg(0 + phi).
template <int PPL>
__device__ __forceinline__ PotC potential_cd(const PointData pt[PPL], double x, bool whole, bool run = true) {
  constexpr int kG = PPL == 1 ? 16 : 8;
  const int c = (int)(threadIdx.x & 3);
  const bool hi8 = PPL == 2 && (threadIdx.x & 8);
  const double e = nexp(c < 3 ? -fabs(x) : x);
  // ln(1 + e), e = exp(-|x|) in (0, 1]: it enters only the log prior, whose
  // absolute (not relative) accuracy matters in U ~ 1e5..1e7, so the fast form
  // takes the table log of the rounded 1 + e (absolute error <= 1.2e-16)
  const double sp = MDFIT_TLOG_NUTS ? flog_t(1.0 + e) : flog1p(e);
  const double rr = rcp(1.0 + e);
  const bool pos = x >= 0.0;
  const double p = pos ? rr : e * rr, omp = pos ? e * rr : rr;
  const double lp = pos ? -sp : x - sp, l1p = pos ? -(x + sp) : -sp;
  const double pr = c == 2 ? lp + 9.0 * l1p : 2.0 * lp + 3.0 * l1p;
  auto bc = [=](double y, auto n) {
    constexpr int N = decltype(n)::value;
    if constexpr (PPL == 1) return rowb<N>(y);
    else return hi8 ? rowb<8 + N>(y) : rowb<N>(y);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  const double q = bc(p, I0{}), omq = bc(omp, I0{}), prq = bc(pr, I0{});
  const double A0 = bc(p, I1{}), prA = bc(pr, I1{});
  const double c0 = bc(p, I2{}), prc = bc(pr, I2{});
  const double delta = bc(e, I3{}), v3 = bc(x, I3{});
  const double phi = delta + 2.0;
  const bool pmd = pt[0].pmd;
  // (PPL 1; chains not running evaluate garbage either way and do not count)
  const bool null_wave = !__any(run && pmd);      // the pad lanes give lg3(a), lg3(b)
  const bool whole_wave = !__any(run && !whole);  // the two rows of a chain share a, b
  const double A = pmd ? A0 : 0.0, cc = pmd ? c0 : 0.0;
  double lprior = prq + v3 - delta * 1e-3;
  if (pmd) lprior += prA + prc;

  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  bool bad_lane = pmd && A + cc >= 1.0;
  double t6l, t6p;
  LG3 t3b;
  if constexpr (PPL == 1) {
    t3b = lg3<false, MDFIT_TLOG_NUTS>(pt[0].N + phi);
    t6l = rowb<15>(t3b.l);  // pad lane: lg(0 + phi)
    t6p = rowb<15>(t3b.p);
  } else {
    t3b = lg3<false, MDFIT_TLOG_NUTS>(pt[1].N + phi);
    const bool src15 = whole || hi8;
    t6l = src15 ? rowb<15>(t3b.l) : rowb<7>(t3b.l);
    t6p = src15 ? rowb<15>(t3b.p) : rowb<7>(t3b.p);
  }
#pragma unroll
  for (int pi = 0; pi < PPL; ++pi) {
    const PointData& pd = pt[pi];
    double D, dq, dA;
    if (pmd) {
      const double w = powk(omq, pd.k);
      D = fma(A, w, cc);
      dq = pd.k > 0 ? -A * (double)pd.k * (w * rcp(omq)) : 0.0;
      dA = w;
    } else {
      D = q;
      dq = 1.0;
      dA = 0.0;
    }
    bad_lane = bad_lane || (pd.valid && !(D < 1.0));
    const double a = D * phi, b = (1.0 - D) * phi;
    const LG3 t1 = lg3<false, MDFIT_TLOG_NUTS>(pd.y + a);
    const LG3 t2 = lg3<false, MDFIT_TLOG_NUTS>(pd.N - pd.y + b);
    LG3 t4, t5;
    if (PPL == 1 && null_wave) {
      // every chain of the wave samples model_null: a = q phi is the row's, and
      // the pad lane's lg3(0 + a) IS lg3(a), bitwise (likewise b)
      t4.l = rowb<15>(t1.l);
      t4.p = rowb<15>(t1.p);
      t5.l = rowb<15>(t2.l);
      t5.p = rowb<15>(t2.p);
    } else if (PPL == 1 && whole_wave) {
      // every chain of the wave is an all-position chain: rows z > 0 and z < 0
      // hold the same |z| lane by lane, so a lane and its partner 16 away share
      // a, b -- the even row takes lg3(a), the odd row lg3(b), exchanged (xrow)
      const bool odd = (threadIdx.x & 16) != 0;
      const LG3 mine = lg3<false, MDFIT_TLOG_NUTS>(odd ? b : a);
      LG3 other;
      other.l = xrow(mine.l);
      other.p = xrow(mine.p);
      other.q = 0.0;
      t4 = odd ? other : mine;
      t5 = odd ? mine : other;
    } else {
      t4 = lg3<false, MDFIT_TLOG_NUTS>(a);
      t5 = lg3<false, MDFIT_TLOG_NUTS>(b);
    }
    const double la = t1.l - t4.l, Pa = t1.p - t4.p;
    const double lb = t2.l - t5.l, Pb = t2.p - t5.p;
    const LG3 t3 = (PPL == 1 || pi == 1) ? t3b : lg3<false, MDFIT_TLOG_NUTS>(pd.N + phi);
    const double ell = (la + lb) - (t3.l - t6l);
    const double lD = phi * (Pa - Pb);
    const double lF = D * Pa + (1.0 - D) * Pb + (t6p - t3.p);
    if (PPL == 1) {
      acc[0] = ell;
      acc[1] = lD * dq;
      acc[2] = lD * dA;
      acc[3] = lD;
      acc[4] = lF;
    } else if (pd.valid) {
      acc[0] += ell;
      acc[1] += lD * dq;
      acc[2] += lD * dA;
      acc[3] += lD;
      acc[4] += lF;
    }
  }
  const int ok = PPL == 1 ? pt[0].valid : 1;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    if constexpr (PPL == 1) {
      const double s16 = gsum<16>(ok ? acc[j] : 0.0);
      acc[j] = whole ? s16 + __shfl_xor(s16, 16, 64) : s16;
    } else {
      const double s8 = gsum<8>(acc[j]);
      acc[j] = whole ? s8 + dpp<0x140>(s8) : s8;
    }
  }
  const unsigned long long bm = __ballot(bad_lane);
  const int sh = (int)(threadIdx.x & (whole ? ~(2 * kG - 1) : ~(kG - 1)));
  const unsigned long long wm = whole ? (kG == 16 ? 0xFFFFFFFFull : 0xFFFFull) : (kG == 16 ? 0xFFFFull : 0xFFull);
  const bool bad = ((bm >> sh) & wm) != 0ull;
  PotC o;
  o.U = -(acc[0] + lprior);
  // component c: -(sum * J + prior slope), J = p (1 - p) (c < 3) or delta
  const double X = c == 0 ? acc[1] : (c == 1 ? acc[2] : (c == 2 ? acc[3] : acc[4]));
  const double Y = c == 3 ? e : p * omp;
  const double Z = c == 3 ? 1.0 - e * 1e-3 : (c == 2 ? 1.0 - 10.0 * p : 2.0 - 5.0 * p);
  o.g = (!pmd && (c == 1 || c == 2)) ? 0.0 : -(X * Y + Z);
  if (bad || !isfinite(o.U)) {
    o.U = INFINITY;
    o.g = 0.0;
  }
  return o;
}

// ((t0 + t1) + t2) + t3 of the slot's four component terms (lanes 0-3 of the
// slot), the oracle's loop order; the terms of inactive components are 0
template <int G>
__device__ __forceinline__ double sum4(double t) {
  double o[4];
  slot4<G>(t, o);
  return ((o[0] + o[1]) + o[2]) + o[3];
}

// kinetic energy (oracle: kinetic), component-distributed
template <int G>
__device__ __forceinline__ double kinetic_cd(bool act, double im, double r) {
#pragma clang fp contract(off)
  return 0.5 * sum4<G>(act ? im * r * r : 0.0);
}

// the U-turn criterion (oracle: is_turning), component-distributed
template <int G>
__device__ __forceinline__ bool turning_cd(bool act, double im, double rl, double rr, double rsum) {
#pragma clang fp contract(off)
  const double rs = rsum - 0.5 * (rl + rr);
  const double dl = sum4<G>(act ? im * rl * rs : 0.0);
  const double dr = sum4<G>(act ? im * rr * rs : 0.0);
  return dl <= 0.0 || dr <= 0.0;
}

// the same on full vectors (a checkpoint's criterion on its own lane)
__device__ __forceinline__ bool turning_full(bool pmd, const double invm[4], const double rl[4], const double rr[4],
                                             const double rsum[4]) {
#pragma clang fp contract(off)
  double dl = 0.0, dr = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (!active(pmd, j)) continue;
    const double rs = rsum[j] - 0.5 * (rl[j] + rr[j]);
    dl += invm[j] * rl[j] * rs;
    dr += invm[j] * rr[j] * rs;
  }
  return dl <= 0.0 || dr <= 0.0;
}

// per-slot LDS vectors (component c at [c])
enum { kVlz, kVlr, kVlg, kVrz, kVrr, kVrg, kVtz, kVtg, kVsz, kVsg, kVwm, kVw2, kVim, kVis, kVtr, kVss, kNVec };

// cold per-chain scalars (row-uniform, LDS)
struct ColdState {
  Stream st;
  int64_t taxon;
  double tpe, spe;  // potential energy of the tree / subtree proposal
  double eps, t_w, t_acc, u_tr;
  double x_avg, g_avg, mu;
  double st_div, st_leap;
  int sub, attempt, f_call, f_m, f_last, f_dir, t_da, widx, wn, nm_chunk, db_chunk;
  int t_n, t_depth;
  double t_start;  // the wave's trip count when the chain started (MDFIT_NUTS_PRIO)
  double w_ref;    // (MDFIT_NUTS_LINW) the largest log-weight of the iteration so far
  double e_ref;    // exp(w_ref), by the product of the rescales (MDFIT_NUTS_EREF)
  double s_acc;    // the subtree's acceptance sum,
  int s_n, ul_chunk;  // size and the chunk of leaf uniforms in sul
#ifdef MDFIT_DEV_TRIPS  // development: per-chain start / end clock and trips in diag 4, 5, 7
  double dev_t0, dev_c0;
#endif
};

template <int PPL>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(MDFIT_NUTS_CD_WAVES))) void nuts_chain_cd(
    const uint32_t* __restrict__ gy, const uint32_t* __restrict__ gN, int64_t T, mdfit_opts o,
    double* __restrict__ out, int* __restrict__ ws, double* __restrict__ samples) {
  static_assert(PPL == 1 || PPL == 2, "points per lane");
  constexpr int kG = PPL == 1 ? 16 : 8;  // lanes per chain slot
  constexpr int kNSlot = kWave / kG;
  constexpr int kTaskL = 2 * kG;
  constexpr unsigned long long kTaskMask = kTaskL == 32 ? 0xFFFFFFFFull : 0xFFFFull;
  constexpr unsigned long long kSlotMask = kG == 16 ? 0xFFFFull : 0xFFull;
  __shared__ double sv[kNSlot][kNVec][4];
  __shared__ ColdState scold[kNSlot];
  __shared__ double sck[8][kWave];                   // checkpoint i of a slot on its lane i: r[4], rsum[4]
  __shared__ double sck8[PPL == 2 ? kNSlot : 1][8];  // PPL 2: checkpoint 8 of a slot
  // draw caches per slot (draw convention 2: two draws per Philox block):
  // sul 32 leaf uniforms, snm the momenta of 8 iterations, sut / sdb the
  // transition uniforms / direction bits of depths 0-7 of 2 iterations
  // (entries 0-15) and of depths 8-9 of this one (16-17)
  __shared__ double sut[18 * kNSlot], sul[32 * kNSlot], snm[32 * kNSlot];
  __shared__ int sdb[18 * kNSlot];
  __shared__ int swin_end[kMaxWin];
  __shared__ int swin_n;
  // lane layout (re-derived from an opaque lane index at every trip of the
  // chain loop: its masks and LDS addresses are recomputed on the fly instead
  // of being held across the loop, which costs registers)
#define MDFIT_CD_LAYOUT(LANE)                                                             \
  const int lane = (LANE);                                                                \
  const int r = lane & (kTaskL - 1), h = r / kG, i = r & (kG - 1), row = lane / kG;       \
  const int c = i & 3; /* this lane's vector component */                                 \
  const int row18 = row * 18, row32 = row * 32;                                            \
  const int leader = lane & ~(kTaskL - 1);                                                \
  double(*V)[4] = sv[row];                                                                \
  ColdState& C = scold[row];                                                              \
  (void)h, (void)c, (void)row18, (void)row32, (void)leader, (void)V, (void)C
  MDFIT_CD_LAYOUT(threadIdx.x);
  // a wave serves its XCD's queue, then the next queues in
  // turn once that one runs dry: the chains are ~1e4 trips long, so the last
  // ones started decide the kernel's end (which wave runs a chain changes no
  // draw: the streams are keyed by taxon and sub-fit)
  int qi = blockIdx.x % kQueues, qs = 0;
  int64_t tl = T * qi / kQueues, nq = T * (qi + 1) / kQueues - tl;
  const int W = o.num_warmup, S = o.num_samples;

  // the lane's points: counts kept as integers across the loop (converted at
  // each evaluation: 2 VGPRs per point instead of 4)
  struct PointQ {
    uint32_t y, N;
    int k, valid;
  } pq[PPL];
  int pmdq = 1;
#pragma unroll
  for (int p = 0; p < PPL; ++p) {
    pq[p].valid = PPL == 1 ? i < kNHalf : 0;
    pq[p].k = PPL == 1 && i < kNHalf ? i : 0;
    pq[p].y = pq[p].N = 0u;
  }
  for (int j = 0; j < 8; ++j) sck[j][lane] = 0.0;
  if (PPL == 2 && i == 0)
    for (int j = 0; j < 8; ++j) sck8[row][j] = 0.0;
  for (int v = 0; v < kNVec; ++v) V[v][c] = (v == kVim || v == kVis) ? 1.0 : 0.0;
  C.st = make_stream(0, 0, 0);
  C.taxon = 0;
  C.tpe = C.spe = C.x_avg = C.g_avg = C.mu = C.st_div = C.st_leap = 0.0;
  C.eps = 1.0;
  C.t_w = C.t_acc = C.u_tr = 0.0;
  C.t_n = C.t_depth = 0;
  C.sub = C.attempt = C.f_call = C.f_m = C.f_last = C.f_dir = C.t_da = C.widx = C.wn = 0;
  C.nm_chunk = C.db_chunk = -1;
  if (lane < kMaxWin) {
    int e, n;
    windows(W, lane, &e, &n);
    swin_end[lane] = e;
    if (lane == 0) swin_n = n;
  }
  __syncthreads();
#ifdef MDFIT_STAMP
  // the split's sections: the time from each NSTAMP(k) to the next stamp
  // reached (their names: tools/nuts_stamp_profile.py)
  constexpr int kNStamp = 10;
  __shared__ unsigned long long sstamp[kNStamp];
  unsigned long long acc_t[kNStamp] = {};
  const unsigned long long t_begin = nstamp();
  sstamp[0] = 0;
#endif

  // hot chain state, row-uniform (the vectors: component c)
  int mode = 0, drained = 0, whole = 0, it = 0;
  double z = 0.0, rm = 0.0, gr = 0.0, im = 1.0;
  // (the subtree's momentum sum: V[kVss], component c -- a register it was spilled)
  // (the tree's scalars -- weight, acceptance sum, size, depth, merge uniform --
  // and the step size are touched once per doubling: ColdState)
  double step = 0.0, e0 = 0.0;
  // (the subtree's acceptance sum and size and the leaf-uniform chunk live in
  // the row's ColdState: touched once a leaf, they were the kernel's spills)
  double s_w = 0.0;
  int leaf_ctr = 0, nleap = 0, n_leaf = 0, nmax = 1;
  C.s_acc = 0.0;
  C.s_n = 0;
  C.ul_chunk = -1;
  int right = 1, t_turn = 0, t_div = 0, s_div = 0;
// slot utilisation and the point-evaluation count (bench.py's compute
// roofline): wave-trips with a running slot, and running slot-trips (each one
// potential evaluation of 15 points), added into the workspace header
// (uint64 at byte 128 / 136; zeroed per call) when the wave exits
#ifndef MDFIT_NO_UTIL
  unsigned long long util_trips = 0, util_busy = 0;
#endif

  while (true) {
#ifdef MDFIT_STAMP
    {
      const unsigned long long now = nstamp();
      if (sstamp[0] != 0) {
        constexpr int order[9] = {0, 1, 2, 5, 6, 7, 8, 3, 4};
        int cur = 0;
        unsigned long long last = sstamp[0];
#pragma unroll
        for (int j = 1; j < 9; ++j) {
          const int k = order[j];
          if (sstamp[k] == 0) continue;
          const unsigned long long d = sstamp[k] - last;
#pragma unroll
          for (int q = 0; q < 9; ++q)
            if (q == cur) acc_t[q] += d;
          last = sstamp[k];
          cur = k;
        }
#pragma unroll
        for (int q = 0; q < 9; ++q)
          if (q == cur) acc_t[q] += now - last;
        acc_t[9] += 1;
      }
      sstamp[0] = now;
      for (int j = 1; j < kNStamp; ++j) sstamp[j] = 0;
    }
#endif
    // (-DMDFIT_CD_HOIST_LAYOUT, development: the layout of the prologue held
    // across the loop instead -- 33 VGPRs spilled at 4 waves/SIMD)
#ifndef MDFIT_CD_HOIST_LAYOUT
    int lane_o = (int)threadIdx.x;
    asm volatile("" : "+v"(lane_o));
    MDFIT_CD_LAYOUT(lane_o);
#endif
    // ---- 1. free groups start a task (one atomic per wave-trip) --------------
    const unsigned long long busy_m = __ballot(mode != 0 && mode != kDone);
    const bool group_free = ((busy_m >> leader) & kTaskMask) == 0ull;
    if (group_free) mode = 0;
    const bool need = group_free && !drained;
    bool starting = false;
    if (__any(need)) {
      const unsigned long long m = __ballot(need && r == 0);
      int base = 0;
      if (lane == 0) base = atomicAdd(ws + qi, __popcll(m));
      base = __builtin_amdgcn_readfirstlane(base);
      const bool dry = (int64_t)base + __popcll(m) > 4 * nq;  // wave-uniform
      if (need) {
        const int64_t task = (int64_t)base + __popcll(m & ((1ull << leader) - 1ull));
        if (task >= 4 * nq) {
          drained = qs + 1 >= kQueues ? 1 : 0;  // (else: the next queue next trip)
          mode = 0;
        } else {
          const int kind = (int)(task / nq);
          C.taxon = tl + task % nq;
          whole = kind == 0 || kind == 2;
          C.sub = kind == 0 ? 0 : (kind == 2 ? 1 : (kind == 1 ? 2 : 4) + h);
          starting = true;
        }
      }
      if (dry && qs + 1 < kQueues) {
        ++qs;
        qi = (qi + 1) % kQueues;
        tl = T * qi / kQueues;
        nq = T * (qi + 1) / kQueues - tl;
      }
    }
    if (starting) {
      const int64_t taxon = C.taxon;
      const int sub = C.sub;
      const int pmd_task = sub == 0 || sub == 2 || sub == 3;
      pmdq = pmd_task;
#pragma unroll
      for (int p = 0; p < PPL; ++p) {
        int colv;
        if (PPL == 1) {
          colv = h * kNHalf + pq[p].k;
        } else if (whole) {
          pq[p].valid = r < kNHalf;
          pq[p].k = r < kNHalf ? r : 0;
          colv = p * kNHalf + pq[p].k;
        } else {
          pq[p].valid = 2 * i + p < kNHalf;
          pq[p].k = pq[p].valid ? 2 * i + p : 0;
          colv = h * kNHalf + pq[p].k;
        }
        pq[p].y = pq[p].valid ? gy[taxon * kLD + colv] : 0u;
        pq[p].N = pq[p].valid ? gN[taxon * kLD + colv] : 0u;
      }
      C.st = make_stream(o.seed, o.index_base + taxon, sub);
      C.nm_chunk = C.db_chunk = -1;
#ifndef MDFIT_NO_UTIL
      C.t_start = (double)util_trips;
#endif
#ifdef MDFIT_DEV_TRIPS
      C.dev_t0 = (double)util_trips;
      C.dev_c0 = (double)__builtin_amdgcn_s_memrealtime();
#endif
      mode = kInit;
      C.attempt = 0;
      it = 0;
      C.st_div = C.st_leap = 0.0;
      C.eps = 1.0;
      step = 0.0;
      C.f_call = C.f_m = C.f_last = C.f_dir = 0;
      C.x_avg = C.g_avg = C.mu = 0.0;
      C.t_da = C.widx = C.wn = 0;
      const bool act = active(pmd_task, c);
      z = act ? -2.0 + 4.0 * uniform(C.st, 0xFFFF0000u, (uint32_t)c) : 0.0;
      rm = gr = 0.0;
      im = 1.0;
      V[kVwm][c] = V[kVw2][c] = V[kVtr][c] = 0.0;
      V[kVim][c] = V[kVis][c] = 1.0;
    }
    if (!__any(mode != 0 || !drained)) break;
    const bool running = mode == kInit || mode == kFind || mode == kIter;
    if (!__any(running)) continue;
#ifndef MDFIT_NO_UTIL
    {
      const unsigned long long rb = __ballot(running && i == 0);
      util_trips += 1;
      util_busy += __popcll(rb);
    }
#if MDFIT_NUTS_PRIO
    if ((util_trips & 255ull) == 0ull) {
      const double age = running ? (double)util_trips - C.t_start : 0.0;
      if (__any(age > 4.0 * MDFIT_NUTS_PRIO_T)) __builtin_amdgcn_s_setprio(3);
      else if (__any(age > 2.0 * MDFIT_NUTS_PRIO_T)) __builtin_amdgcn_s_setprio(2);
      else if (__any(age > MDFIT_NUTS_PRIO_T)) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
#endif
#endif
    const bool pmd = pmdq;
    const bool act = active(pmd, c);
    PointData pd[PPL];
#pragma unroll
    for (int p = 0; p < PPL; ++p) {
      pd[p].y = (double)pq[p].y;
      pd[p].N = (double)pq[p].N;
      pd[p].k = pq[p].k;
      pd[p].valid = pq[p].valid;
      pd[p].pmd = pmdq;
    }

    NSTAMP(1);
    // ---- 2. one evaluation: the initial point, or a leapfrog step ------------
    const double rh = rm - 0.5 * step * gr;
    const double zev = mode == kInit ? z : z + step * im * rh;
#ifdef MDFIT_DEV_NOPOT  // development: register demand of the state machine alone
    PotC P;
    P.U = zev * zev + pd[0].y;
    P.g = 2.0 * zev;
#elif defined(MDFIT_NUTS_POT_TWICE)  // development: marginal cost of one potential evaluation
    const PotC P0 = potential_cd<PPL>(pd, zev * (1.0 + 1e-300 * (double)it), whole);
    PotC P = potential_cd<PPL>(pd, zev, whole);
    P.U += 0.0 * P0.U * (double)(it > (1 << 30));
#else
    const PotC P = potential_cd<PPL>(pd, zev, whole, running);
#endif
    NSTAMP(2);
    if (!running) continue;
    const double rn = rh - 0.5 * step * P.g;
    z = zev;

    bool begin_iter = false, begin_find = false;
    if (mode == kInit) {
      if (isfinite(P.U)) {
        V[kVtz][c] = zev;
        V[kVtg][c] = P.g;
        C.tpe = P.U;
        C.eps = 1.0;
        C.f_call = 0;
        begin_find = true;
      } else if (++C.attempt >= 100) {
        // no finite initial point: NaN draws, status 2
        const int64_t taxon = C.taxon;
        const int sub = C.sub;
        for (int s = i; s < S; s += kG)
          if (!whole || h == 0)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              samples[((taxon * MDFIT_NSUBFIT + sub) * (int64_t)S + s) * 4 + j] = NAN;
        if ((!whole || h == 0) && i < 4) {
          double* dg = out + taxon * MDFIT_NOUT + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * sub;
          dg[4 + i] = i == 2 ? (double)MDFIT_NONFINITE : NAN;
        }
        mode = kDone;
      } else {
        z = act ? -2.0 + 4.0 * uniform(C.st, 0xFFFF0000u + (uint32_t)C.attempt, (uint32_t)c) : 0.0;
      }
    } else if (mode == kFind) {
      const double de = (P.U + kinetic_cd<kG>(act, im, rn)) - e0;
      const int dnew = log(kTarget) < -de ? 1 : -1;
      const int f_last = C.f_dir;
      C.f_last = f_last;
      C.f_dir = dnew;
      const int f_m = ++C.f_m;
      const bool cont = (C.eps > kTiny || dnew >= 0) && (C.eps < kHuge || dnew <= 0) && (f_last == 0 || dnew == f_last) &&
                        f_m < 4000;
      if (cont) {
        begin_find = true;
      } else {
        C.mu = log(10.0 * C.eps);
        C.x_avg = C.g_avg = 0.0;
        C.t_da = 0;
        begin_iter = true;
      }
    } else {  // kIter: a leaf of the subtree
      ++nleap;
      double rn4[4], im4[4];
      slot4<kG>(rn, rn4);
#pragma unroll
      for (int j = 0; j < 4; ++j) im4[j] = V[kVim][j];
      double de;
      {
#pragma clang fp contract(off)
        double k = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (active(pmd, j)) k += im4[j] * rn4[j] * rn4[j];
        de = (P.U + 0.5 * k) - e0;
      }
      if (isnan(de)) de = INFINITY;
      const double w = -de;
      const int dv = de > kMaxDelta;
#if MDFIT_NUTS_LINW
      // s_w: the subtree's weight, C.t_w the tree's, both relative to w_ref
      double ew, acc;
      {
        const double wr = C.w_ref;
        const double d = w - wr;
        const double ed = nexp(-fabs(d));  // (w = -inf: 0)
        if (d > 0.0) {  // the new largest log-weight: rescale the sums
          C.t_w *= ed;
          s_w *= ed;
          C.w_ref = w;
          if (MDFIT_NUTS_EREF) C.e_ref = C.e_ref * rcp(ed);
          ew = 1.0;
          acc = 1.0;  // (w > w_ref >= 0)
        } else {
          ew = ed;
          acc = w >= 0.0 ? 1.0
                         : (wr == 0.0 ? ed : (MDFIT_NUTS_EREF && wr < 700.0 ? fmin(1.0, ed * C.e_ref) : nexp(w)));
        }
      }
#else
      const double acc = de > 0.0 ? nexp(-de) : 1.0;
#endif
      if (n_leaf == 0) {
        V[kVsz][c] = zev;
        V[kVsg][c] = P.g;
        C.spe = P.U;
        V[kVss][c] = rn;
#if MDFIT_NUTS_LINW
        s_w = ew;
#else
        s_w = w;
#endif
        C.s_acc = acc;
        C.s_n = 1;
      } else {
#if MDFIT_NUTS_LINW
        const double nw = s_w + ew;
        const double prob = ew * rcp(nw);  // (nw = 0: NaN, never taken -- the oracle's NaN too)
#else
        const double m = fmax(s_w, w);
        const double e = nexp(-fabs(s_w - w));
        const double nw = m == -INFINITY ? -INFINITY : m + lae1p(e);
        const double prob = (w >= s_w ? 1.0 : e) * rcp(1.0 + e);
#endif
        if ((leaf_ctr >> 5) != C.ul_chunk) {  // next 32 leaf uniforms: 2 per block, 32 / kG per lane
#pragma unroll
          for (int e2 = 0; e2 < 16 / kG; ++e2) {
            const int ix = i + kG * e2;
            const uint4 b = block(C.st, (uint32_t)it, 32u + ((uint32_t)(leaf_ctr & ~31) >> 1) + (uint32_t)ix);
            sul[row32 + 2 * ix] = u53(b.x, b.y);
            sul[row32 + 2 * ix + 1] = u53(b.z, b.w);
          }
          C.ul_chunk = leaf_ctr >> 5;
        }
        if (sul[row32 + (leaf_ctr & 31)] < prob) {
          V[kVsz][c] = zev;
          V[kVsg][c] = P.g;
          C.spe = P.U;
        }
        s_w = nw;
        V[kVss][c] += rn;
        C.s_acc += acc;
        C.s_n += 1;
      }
      s_div = dv;
      ++leaf_ctr;
      NSTAMP(5);
      int imin, imax;
      ckpt_idxs(n_leaf, &imin, &imax);
      const double srs = V[kVss][c];
      double srs4[4];
      slot4<kG>(srs, srs4);
      if ((n_leaf & 1) == 0 && i == imax) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sck[j][lane] = rn4[j];
          sck[4 + j][lane] = srs4[j];
        }
      }
      if (PPL == 2 && (n_leaf & 1) == 0 && imax == 8 && i == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sck8[row][j] = rn4[j];
          sck8[row][4 + j] = srs4[j];
        }
      }
      bool my_turn = false;
      if (i >= imin && i <= imax) {
#pragma clang fp contract(off)
        double ck_r[4], sub_rsum[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ck_r[j] = sck[j][lane];
          sub_rsum[j] = srs4[j] - sck[4 + j][lane] + ck_r[j];
        }
        my_turn = turning_full(pmd, im4, ck_r, rn4, sub_rsum);
      }
      if (PPL == 2 && i == 0 && imin <= 8 && imax >= 8) {
#pragma clang fp contract(off)
        double ck_r[4], sub_rsum[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          ck_r[j] = sck8[row][j];
          sub_rsum[j] = srs4[j] - sck8[row][4 + j] + ck_r[j];
        }
        my_turn = my_turn || turning_full(pmd, im4, ck_r, rn4, sub_rsum);
      }
      const unsigned long long tm = __ballot(my_turn);
      const int s_turn = ((tm >> (lane & ~(kG - 1))) & kSlotMask) != 0ull;
      ++n_leaf;
      rm = rn;
      gr = P.g;
      if (s_turn || s_div || n_leaf == nmax) {
        NSTAMP(6);
        // merge the subtree into the tree: biased progressive sampling
#if MDFIT_NUTS_LINW
        const double prob = (s_turn || s_div) ? 0.0 : (s_w > C.t_w ? 1.0 : s_w * rcp(C.t_w));
#else
        const double em = nexp(-fabs(C.t_w - s_w));
        const double prob = (s_turn || s_div) ? 0.0 : (s_w > C.t_w ? 1.0 : em);
#endif
        if (C.u_tr < prob) {
          V[kVtz][c] = V[kVsz][c];
          V[kVtg][c] = V[kVsg][c];
          C.tpe = C.spe;
        }
        const double olr = right ? V[kVlr][c] : V[kVrr][c];  // r of the untouched end
        if (right) {
          V[kVrz][c] = z;
          V[kVrr][c] = rm;
          V[kVrg][c] = gr;
        } else {
          V[kVlz][c] = z;
          V[kVlr][c] = rm;
          V[kVlg][c] = gr;
        }
#if MDFIT_NUTS_LINW
        C.t_w = C.t_w + s_w;
#else
        {
          const double m = fmax(C.t_w, s_w);
          C.t_w = m == -INFINITY ? -INFINITY : m + lae1p(em);
        }
#endif
        const double trs = V[kVtr][c] + V[kVss][c];
        V[kVtr][c] = trs;
        t_turn = s_turn || (right ? turning_cd<kG>(act, im, olr, rm, trs) : turning_cd<kG>(act, im, rm, olr, trs));
        t_div = s_div;
        C.t_acc += C.s_acc;
        C.t_n += C.s_n;
        ++C.t_depth;
        if (C.t_depth >= kMaxDepth || t_turn || t_div) {
          NSTAMP(7);
          // ---- the transition is complete: adapt or keep the draw ----------
          const double accp = C.t_acc / (double)C.t_n;
          if (it < W) {
            const int t_da = ++C.t_da;
            const double gg = kTarget - accp;
            const double inv = 1.0 / (t_da + 10.0);
            const double g_avg = (1.0 - inv) * C.g_avg + gg * inv;
            C.g_avg = g_avg;
            const double x_t = C.mu - sqrt((double)t_da) * 20.0 * g_avg;  // / gamma (0.05)
            const double sq = sqrt((double)t_da);
            const double wt = 1.0 / (sq * sqrt(sq));  // t^-0.75
            const double x_avg = (1.0 - wt) * C.x_avg + wt * x_t;
            C.x_avg = x_avg;
            C.eps = nexp(it == W - 1 ? x_avg : x_t);
            if (C.eps < kTiny) C.eps = kTiny;
            const int widx = C.widx;
            const int wend = widx < kMaxWin ? swin_end[widx] : -1, nwin = swin_n;
            const bool middle = widx > 0 && widx < nwin - 1;
            if (middle) {
              const int wn = ++C.wn;
              if (act) {
                const double tz = V[kVtz][c], wmean = V[kVwm][c];
                const double d0 = tz - wmean;
                const double wm1 = wmean + d0 / wn;
                V[kVwm][c] = wm1;
                V[kVw2][c] = V[kVw2][c] + d0 * (tz - wm1);
              }
            }
            const bool at_end = it == wend;
            if (at_end && middle) {
              const int wn = C.wn;
              if (act) {
                const double var = V[kVw2][c] / (wn - 1);
                im = ((double)wn / (wn + 5.0)) * var + 1e-3 * (5.0 / (wn + 5.0));
                V[kVis][c] = sqrt(1.0 / im);
                V[kVim][c] = im;
                V[kVwm][c] = V[kVw2][c] = 0.0;
              }
              C.wn = 0;
              ++C.f_call;
              begin_find = true;
            }
            if (at_end) C.widx = widx + 1;
          } else {
            const int64_t sidx = ((C.taxon * MDFIT_NSUBFIT + C.sub) * (int64_t)S + (it - W)) * 4;
            if ((!whole || h == 0) && i < 4) {
              const double zj = V[kVtz][c];
#if MDFIT_NUTS_SST  // one exponential per lane: exp(z3) + 2 on lane 3, the sigmoid on lanes 0-2
              const double ez = nexp(i == 3 ? zj : -zj);
              samples[sidx + i] = i == 3 ? ez + 2.0 : ((i == 0 || pmd) ? rcp(1.0 + ez) : 0.0);
#else
              samples[sidx + i] = i == 3 ? nexp(zj) + 2.0 : ((i == 0 || pmd) ? 1.0 / (1.0 + nexp(-zj)) : 0.0);
#endif
            }
            C.st_div += t_div ? 1.0 : 0.0;
            C.st_leap += (double)nleap;
          }
          ++it;
          if (it == W + S) {
            if ((!whole || h == 0) && i < 4) {
              double* dg = out + C.taxon * MDFIT_NOUT + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * C.sub;
#ifdef MDFIT_DEV_TRIPS
              dg[4 + i] = i == 0 ? C.dev_c0 : (i == 1 ? (double)__builtin_amdgcn_s_memrealtime() : (i == 2 ? (double)MDFIT_OK : (double)util_trips - C.dev_t0));
#else
              dg[4 + i] = i == 0 ? C.eps : (i == 1 ? C.st_leap / S : (i == 2 ? (double)MDFIT_OK : C.st_div));
#endif
            }
            mode = kDone;
          } else if (!begin_find) {
            begin_iter = true;
          }
        } else {
          NSTAMP(8);
          // next doubling
          const int j = C.t_depth;
          if (j == 8) {  // the draws of depths 8 and 9 (entries 16, 17 of the caches)
            if (i < 2) {
              const uint4 b = block(C.st, (uint32_t)it, 12u + (uint32_t)i);
              sdb[row18 + 16 + i] = (int)(b.z & 1u);
              sut[row18 + 16 + i] = u53(b.x, b.y);
            }
          }
          const int e = j < 8 ? 8 * (it & 1) + j : 8 + j;
          right = sdb[row18 + e] != 0;
          C.u_tr = sut[row18 + e];
          n_leaf = 0;
          nmax = 1 << j;
          step = right ? C.eps : -C.eps;
          z = right ? V[kVrz][c] : V[kVlz][c];
          rm = right ? V[kVrr][c] : V[kVlr][c];
          gr = right ? V[kVrg][c] : V[kVlg][c];
        }
      }  // (else: the next leaf of the subtree continues from (z, r, g) with the same step)
    }

    NSTAMP(3);
    if (begin_find) {
      // one probe of find_reasonable_step_size from the current state
      if (mode != kFind || C.f_m == 0) {
        C.f_m = 0;
        C.f_last = C.f_dir = 0;
      }
      mode = kFind;
      C.eps = ldexp(C.eps, C.f_dir);
      const double nj =
          normal_k(C.st, 0xFFFE0000u + 4096u * (uint32_t)C.f_call + (uint32_t)C.f_m, (uint32_t)(c >> 1), c & 1);
      rm = act ? nj * V[kVis][c] : 0.0;
      z = V[kVtz][c];
      gr = V[kVtg][c];
      e0 = C.tpe + kinetic_cd<kG>(act, im, rm);
      step = C.eps;
    }
    if (begin_iter) {
      mode = kIter;
      // this iteration's momenta from the 4-iteration cache
      if ((it >> 3) != C.nm_chunk) {  // the momenta of 8 iterations: lane ix the pair (it, dims 2m, 2m + 1)
#pragma unroll
        for (int e2 = 0; e2 < 16 / kG; ++e2) {
          const int ix = i + kG * e2;
          const double2 np = normal_pair(C.st, (uint32_t)((it & ~7) + (ix >> 1)), (uint32_t)(ix & 1));
          snm[row32 + 2 * ix] = np.x;
          snm[row32 + 2 * ix + 1] = np.y;
        }
        C.nm_chunk = it >> 3;
      }
      const double nj = snm[row32 + 4 * (it & 7) + c];
      rm = act ? nj * V[kVis][c] : 0.0;
      z = V[kVtz][c];
      gr = V[kVtg][c];
      V[kVlz][c] = V[kVrz][c] = z;
      V[kVlr][c] = V[kVrr][c] = rm;
      V[kVlg][c] = V[kVrg][c] = gr;
      V[kVtr][c] = rm;
      e0 = C.tpe + kinetic_cd<kG>(act, im, rm);
#if MDFIT_NUTS_LINW
      C.t_w = 1.0;  // the initial point's weight exp(0 - w_ref)
      C.w_ref = 0.0;
      C.e_ref = 1.0;
#else
      C.t_w = 0.0;
#endif
      C.t_acc = 0.0;
      C.t_n = 0;
      C.t_depth = 0;
      t_turn = t_div = 0;
      leaf_ctr = 0;
      nleap = 0;
      // the doubling draws of depths 0-7 of this iteration and the next, one
      // Philox block per (iteration, depth) -- its direction bit and merge
      // uniform -- at entry 8 (iteration & 1) + depth (depths 8-9, reached by
      // a few iterations, at that doubling)
      if ((it >> 1) != C.db_chunk) {
#pragma unroll
        for (int e2 = 0; e2 < 16 / kG; ++e2) {
          const int ix = i + kG * e2;
          const uint4 b = block(C.st, (uint32_t)((it & ~1) + (ix >> 3)), 4u + (uint32_t)(ix & 7));
          sdb[row18 + ix] = (int)(b.z & 1u);
          sut[row18 + ix] = u53(b.x, b.y);
        }
        C.db_chunk = it >> 1;
      }
      C.ul_chunk = -1;
      right = sdb[row18 + 8 * (it & 1)] != 0;
      C.u_tr = sut[row18 + 8 * (it & 1)];
      n_leaf = 0;
      nmax = 1;
      step = right ? C.eps : -C.eps;
    }
    NSTAMP(4);
  }
#ifdef MDFIT_STAMP
  if (lane == 0 && g_nuts_stamp) {
    unsigned long long* w = g_nuts_stamp + 16 * (size_t)blockIdx.x;
    for (int j = 0; j < kNStamp; ++j) w[j] = acc_t[j];
    w[10] = nstamp() - t_begin;
  }
#endif
#ifndef MDFIT_NO_UTIL
  if (threadIdx.x == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(ws + 32), util_trips);
    atomicAdd(reinterpret_cast<unsigned long long*>(ws + 34), util_busy);
  }
#endif
}

// ---------------------------------------------------------------------------
// post kernel: one wave per taxon
// ---------------------------------------------------------------------------
// frac = obs / N of one predictive Beta-Binomial draw (oracle: predictive_frac)
// (predictive draw convention 2, round 6: a block gives two uniforms -- words
// 0-1, then 2-3 -- or a Box-Muller pair of normals -- cos, then sin; the two
// kinds take blocks from one counter in the order they run dry; oracle: ndraw)
struct Draw {
  const Stream* st;
  uint32_t w2, w3;
  double uc = 0.0, nc = 0.0;  // the block's second uniform / normal
  bool uh = false, nh = false;
  __device__ double uni() {
    if (uh) {
      uh = false;
      return uc;
    }
    const uint4 o = block(*st, w2, w3++);
    uc = u53(o.z, o.w);
    uh = true;
    return u53(o.x, o.y);
  }
  __device__ double nrm() {
    if (nh) {
      nh = false;
      return nc;
    }
    const uint4 o = block(*st, w2, w3++);
    const double u1 = 1.0 - u53(o.x, o.y), u2 = u53(o.z, o.w);
    double sn, cs;
    sincos(6.283185307179586 * u2, &sn, &cs);
    const double r = sqrt(-2.0 * plog(u1));
    nc = r * sn;
    nh = true;
    return r * cs;
  }
};

__device__ double log_gamma_draw(Draw& d, double alpha) {
  double boost = 0.0;
  if (alpha < 1.0) {
    boost = plog(1.0 - d.uni()) / alpha;
    alpha += 1.0;
  }
  // (rsqrt for the oracle's 1 / sqrt: a last-bit difference in cc, which no
  // draw of the 20k-taxon A/B felt -- profiles/r06_ab_rsq.txt)
  const double dd = alpha - 1.0 / 3.0, cc = rsqrt(9.0 * dd);
  for (int k = 0; k < 256; ++k) {
    const double x = d.nrm();
    double v = 1.0 + cc * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = d.uni();
    if (u < 1.0 - 0.0331 * x * x * x * x) return plog(dd * v) + boost;
    if (plog(u) < 0.5 * x * x + dd * (1.0 - v + plog(v))) return plog(dd * v) + boost;
  }
  return plog(dd) + boost;
}

__device__ double binomial_draw(Draw& d, double n, double p) {
  if (n <= 0.0 || p <= 0.0) return 0.0;
  if (p >= 1.0) return n;
  const bool flip = p > 0.5;
  const double pp = flip ? 1.0 - p : p, qq = 1.0 - pp;
  double k;
  if (n * pp < 10.0) {
    const double u = d.uni();
    double pmf = pexp(n * log1p(-pp)), cdf = pmf;
    k = 0.0;
    const double ratio = pp / qq;
    while (u > cdf && k < n && k < 10000.0) {
      pmf *= (n - k) / (k + 1.0) * ratio;
      k += 1.0;
      cdf += pmf;
    }
  } else {
    const double spq = sqrt(n * pp * qq), bb = 1.15 + 2.53 * spq;
    const double aa = -0.0873 + 0.0248 * bb + 0.01 * pp, cc = n * pp + 0.5;
    const double rb = 1.0 / bb;  // (one division for the two: last-bit differences only)
    const double vr = 0.92 - 4.2 * rb, alpha = (2.83 + 5.1 * rb) * spq;
    const double lpq = plog(pp / qq), m = floor((n + 1.0) * pp);
    const double hh = lg3<false>(m + 1.0).l + lg3<false>(n - m + 1.0).l;
    k = floor(cc);
    for (int it = 0; it < 256; ++it) {
      const double u = d.uni() - 0.5, v = d.uni();
      const double us = 0.5 - fabs(u);
      const double kk = floor((2.0 * aa / us + bb) * u + cc);
      if (kk < 0.0 || kk > n) continue;
      if (us >= 0.07 && v <= vr) {
        k = kk;
        break;
      }
      const double lv = plog(v * alpha / (aa / (us * us) + bb));
      if (lv <= hh - lg3<false>(kk + 1.0).l - lg3<false>(n - kk + 1.0).l + (kk - m) * lpq) {
        k = kk;
        break;
      }
    }
  }
  return flip ? n - k : k;
}

__device__ __forceinline__ double d_at(const double* th, bool pmd, int k) {
  double D = pmd ? th[1] * powk(1.0 - th[0], k) + th[2] : th[0];
  return D < 0.0 ? 0.0 : (D > 1.0 ? 1.0 : D);
}

// One predictive Beta-Binomial draw as its integer count obs <= N (the
// oracle's predictive_frac is obs / N: the post kernel sorts the counts and
// forms the fractions after).  A draw that is not a count in [0, N] (NaN theta
// or p) returns -1: the oracle's NaN fraction makes median and HPDI NaN.
__device__ int64_t predictive_count(const Stream& st, int s, int col, int k, double Nn, const double* th) {
  const double D = d_at(th, true, k);
  Draw d{&st, 0xFFFD0000u + (uint32_t)s, (uint32_t)col << 16};
  const double lx = log_gamma_draw(d, D * th[3]), ly = log_gamma_draw(d, (1.0 - D) * th[3]);
  const double p = 1.0 / (1.0 + pexp(ly - lx));
  const double obs = binomial_draw(d, Nn, p);
  return (obs >= 0.0 && obs <= Nn) ? (int64_t)obs : -1;
}

// wave-wide reductions
__device__ __forceinline__ double wsum(double v) { return gsum<64>(v); }
__device__ __forceinline__ double wmax(double v) {
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// bitonic sort of n counts in LDS (padded to a power of two with UINT32_MAX)
__device__ void lds_sort_u32(uint32_t* v, int n) {
  int m = 1;
  while (m < n) m <<= 1;
  for (int j = n + threadIdx.x; j < m; j += kWave) v[j] = 0xFFFFFFFFu;
  __syncthreads();
  for (int k = 2; k <= m; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int x = threadIdx.x; x < m; x += kWave) {
        const int y = x ^ j;
        if (y > x) {
          const uint32_t a = v[x], b = v[y];
          const bool up = (x & k) == 0;
          if ((a > b) == up) {
            v[x] = b;
            v[y] = a;
          }
        }
      }
      __syncthreads();
    }
  }
}
// the same sort of n <= 64 R counts with the values in registers: lane L holds
// elements 16 L .. 16 L + 15 (R = 16: n <= 1024, the reference's 1000 draws);
// strides below R are compare-exchanges inside the lane, the others one
// cross-lane exchange per value -- no LDS round trip and no barrier per stage.
// The sorted sequence is the LDS sort's (a sort's result is unique).
template <int R>
__device__ void reg_sort_u32(uint32_t* v_lds, int n) {
  const int lane = threadIdx.x;
  uint32_t v[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int e = lane * R + j;
    v[j] = e < n ? v_lds[e] : 0xFFFFFFFFu;
  }
#pragma unroll
  for (int k = 2; k <= kWave * R; k <<= 1) {
#pragma unroll
    for (int s = k >> 1; s > 0; s >>= 1) {
      if (s >= R) {
        const int ls = s / R;
        const bool upper = (lane & ls) != 0;
        const bool asc = ((lane * R) & k) == 0;
        const bool take_max = upper == asc;
#pragma unroll
        for (int j = 0; j < R; ++j) {
          const uint32_t p = (uint32_t)__shfl_xor((int)v[j], ls, kWave);
          v[j] = take_max ? max(v[j], p) : min(v[j], p);
        }
      } else {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          if (j & s) continue;
          const int jj = j | s;
          const bool asc = k >= R ? (((lane * R) & k) == 0) : ((j & k) == 0);
          const uint32_t a = v[j], b = v[jj];
          const uint32_t lo = min(a, b), hi = max(a, b);
          v[j] = asc ? lo : hi;
          v[jj] = asc ? hi : lo;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int e = lane * R + j;
    if (e < n) v_lds[e] = v[j];
  }
  __syncthreads();
}

// np.median + numpyro hpdi(prob 0.68) over the fractions c / N of the S sorted
// counts c: each fraction is formed as the oracle's predictive_frac forms it,
// so the result is its median_hpdi on the sorted fractions bit for bit
// (c -> c / N is monotone: the same order, ties where the fractions tie)
__device__ void median_hpdi_counts(const uint32_t* c, int S, double Nn, double out3[3]) {
  auto f = [&](int x) { return (double)c[x] / Nn; };
  out3[0] = (S & 1) ? f(S / 2) : 0.5 * (f(S / 2 - 1) + f(S / 2));
  const int len = (int)(0.68 * S);
  double bw = INFINITY;
  int best = 0;
  for (int x = threadIdx.x; x < S - len; x += kWave) {
    const double w = f(x + len) - f(x);
    if (w < bw) {  // first minimum per lane
      bw = w;
      best = x;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const double ow = __shfl_xor(bw, o, 64);
    const int ob = __shfl_xor(best, o, 64);
    if (ow < bw || (ow == bw && ob < best)) {
      bw = ow;
      best = ob;
    }
  }
  out3[1] = f(best);
  out3[2] = f(best + len);
}

#if MDFIT_WAIC_GROUP > 1
// waic_i (fits.py:126-172) of G columns whose draws share D (so a, b, a + b):
// one pass over the draws, their three lnGamma values formed once per draw;
// per column the same expression and accumulators as the one-column pass
template <int G>
__device__ __forceinline__ void waic_cols(int lane, int S, const double* smp, bool pmd, int k, const int* cols,
                                          const double* s_y, const double* s_N, double* waic_row) {
#pragma clang fp contract(off)
  double lc[G], mxl[G], sel[G], mul[G], m2l[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const double yy = s_y[cols[g]], nn = s_N[cols[g]];
    lc[g] = lg3<false, MDFIT_TLOG_NUTS>(nn + 1.0).l - lg3<false, MDFIT_TLOG_NUTS>(yy + 1.0).l -
            lg3<false, MDFIT_TLOG_NUTS>(nn - yy + 1.0).l;
    mxl[g] = -INFINITY;
    sel[g] = mul[g] = m2l[g] = 0.0;
  }
  double cnt = 0.0;
  for (int x = lane; x < S; x += kWave) {
    const double* th = smp + (int64_t)x * 4;
    const double D = d_at(th, pmd, k), phi = th[3];
    const double a = D * phi, b = (1.0 - D) * phi;
    const double la = lg3<false, MDFIT_TLOG_NUTS>(a).l, lb = lg3<false, MDFIT_TLOG_NUTS>(b).l,
                 lab = lg3<false, MDFIT_TLOG_NUTS>(a + b).l;
    cnt += 1.0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const double yy = s_y[cols[g]], nn = s_N[cols[g]];  // (LDS broadcasts: no registers held)
      const double lp = lc[g] + (lg3<false, MDFIT_TLOG_NUTS>(yy + a).l - la) +
                        (lg3<false, MDFIT_TLOG_NUTS>(nn - yy + b).l - lb) -
                        (lg3<false, MDFIT_TLOG_NUTS>(nn + phi).l - lab);
      if (lp == -INFINITY) {
      } else if (lp > mxl[g]) {
        sel[g] = sel[g] * pexp(mxl[g] - lp) + 1.0;
        mxl[g] = lp;
      } else {
        sel[g] += pexp(lp - mxl[g]);
      }
      const double dlt = lp - mul[g];
      mul[g] += dlt / cnt;
      m2l[g] = fma(dlt, lp - mul[g], m2l[g]);
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const double mx = wmax(mxl[g]);
    const double se = wsum(cnt > 0.0 ? sel[g] * pexp(mxl[g] - mx) : 0.0);
    const double mean = wsum(cnt * mul[g]) / S;
    const double dm = mul[g] - mean;
    const double var = wsum(m2l[g] + cnt * dm * dm) / S;
    const double lppd = mx + log(se) - log((double)S);
    if (lane == 0) waic_row[cols[g]] = -2.0 * (lppd - var);
  }
  __syncthreads();
}
#endif

__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(MDFIT_POST_WAVES))) void nuts_post_kernel(const uint32_t* __restrict__ gy,
                                                          const uint32_t* __restrict__ gN,
                                                          const uint32_t* __restrict__ gmm, int64_t n_taxa,
                                                          mdfit_opts o, const double* __restrict__ samples,
                                                          double* __restrict__ out, float* __restrict__ pred,
                                                          int32_t* __restrict__ status) {
  __shared__ double s_y[kLD], s_N[kLD];
  __shared__ double s_rec[MDFIT_NOUT];
  __shared__ double s_waic[MDFIT_NSUBFIT][kNPos];
  // the per-draw values (pointwise log-likelihoods, predictive fractions): the
  // launch sizes it to the sort's power of two >= S (8 KB at S = 1000; a
  // fixed kMaxSamples array made the block 37 KB and capped the kernel at one
  // wave per SIMD)
  extern __shared__ double s_v[];
  uint32_t* s_c = reinterpret_cast<uint32_t*>(s_v);  // the predictive draws' counts
  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  const int S = o.num_samples;
  if (t >= n_taxa) return;
  if (lane < kLD) {
    s_y[lane] = (double)gy[t * kLD + lane];
    s_N[lane] = (double)gN[t * kLD + lane];
  }
  for (int x = lane; x < MDFIT_NOUT; x += kWave)
    s_rec[x] = (x >= MDFIT_NRESULT && x < MDFIT_F_DIAG) ? 0.0 : out[t * MDFIT_NOUT + x];
  __syncthreads();
  const bool bad_lane = lane < kNPos && s_y[lane] > s_N[lane];
  if (__any(bad_lane)) {
    for (int x = lane; x < MDFIT_NOUT; x += kWave) out[t * MDFIT_NOUT + x] = NAN;
    if (pred != nullptr)
      for (int x = lane; x < MDFIT_NPRED * kNPos; x += kWave) pred[t * (MDFIT_NPRED * kNPos) + x] = NAN;
    if (lane == 0) status[t] = MDFIT_INVALID;
    return;
  }
  int stt = MDFIT_OK;
  for (int s = 0; s < MDFIT_NSUBFIT; ++s) stt = max(stt, (int)s_rec[MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * s + 6]);
  const double* smp = samples + t * MDFIT_NSUBFIT * (int64_t)S * 4;

  // ---- posterior means of (q, A, c, phi) per chain -> diag slots 0..3 ---------
  for (int s = 0; s < MDFIT_NSUBFIT; ++s) {
    double m[4] = {0, 0, 0, 0};
    for (int x = lane; x < S; x += kWave)
#pragma unroll
      for (int j = 0; j < 4; ++j) m[j] += smp[((int64_t)s * S + x) * 4 + j];
#pragma unroll
    for (int j = 0; j < 4; ++j) m[j] = wsum(m[j]) / S;
    if (lane == 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) s_rec[MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * s + j] = m[j];
  }
  __syncthreads();
  if (stt != MDFIT_OK) {
    for (int x = lane; x < MDFIT_NRESULT; x += kWave) s_rec[x] = NAN;
    if (pred != nullptr)
      for (int x = lane; x < MDFIT_NPRED * kNPos; x += kWave) pred[t * (MDFIT_NPRED * kNPos) + x] = NAN;
    __syncthreads();
    for (int x = lane; x < MDFIT_NOUT; x += kWave) out[t * MDFIT_NOUT + x] = s_rec[x];
    if (lane == 0) status[t] = stt;
    return;
  }

  // ---- waic_i per chain and point (fits.py:126-172), lanes over draws ----------
  // (-DMDFIT_DEV_NOWAIC / -DMDFIT_DEV_NOPRED, development: the post kernel's
  // split with one part compiled out -- never a product build)
#ifdef MDFIT_DEV_NOWAIC
  for (int x = lane; x < MDFIT_NSUBFIT * kNPos; x += kWave) (&s_waic[0][0])[x] = 1.0 + x;
  for (int s = 0; s < 0; ++s) {
#else
  for (int s = 0; s < MDFIT_NSUBFIT; ++s) {
#endif
    // (no contraction: the grouped and the per-column passes then round every
    // lp alike -- fusing D * phi into yy + a depends on how often a is used)
#pragma clang fp contract(off)
    const bool pmd = s == 0 || s == 2 || s == 3;
    const int lo = (s == 3 || s == 5) ? kNHalf : 0, hi = s < 2 ? kNPos : lo + kNHalf;
#if MDFIT_WAIC_GROUP > 1
    // columns sharing D share a, b and a + b: every column of a null sub-fit
    // (D = q; groups of MDFIT_WAIC_GROUP), and in the PMD all-position sub-fit
    // the pair z = k+1 / -(k+1) (one k)
    if (!pmd) {
      for (int c0 = lo; c0 < hi; c0 += MDFIT_WAIC_GROUP) {
        int cols[MDFIT_WAIC_GROUP];
#pragma unroll
        for (int g = 0; g < MDFIT_WAIC_GROUP; ++g) cols[g] = c0 + g;
        waic_cols<MDFIT_WAIC_GROUP>(lane, S, smp + (int64_t)s * S * 4, false, 0, cols, s_y, s_N, s_waic[s]);
      }
      continue;
    }
    if (s == 0) {
      for (int k = 0; k < kNHalf; ++k) {
        const int cols[2] = {k, kNHalf + k};
        waic_cols<2>(lane, S, smp, true, k, cols, s_y, s_N, s_waic[0]);
      }
      continue;
    }
#endif
    for (int col = lo; col < hi; ++col) {
      const double yy = s_y[col], nn = s_N[col];
      const int k = col < kNHalf ? col : col - kNHalf;
      const double lc = lg3<false, MDFIT_TLOG_NUTS>(nn + 1.0).l - lg3<false, MDFIT_TLOG_NUTS>(yy + 1.0).l - lg3<false, MDFIT_TLOG_NUTS>(nn - yy + 1.0).l;
      // one pass: per lane a running max with its sum of exp (log-sum-exp) and
      // Welford's mean / M2 over its draws, combined across the wave -- the
      // lppd and variance of the two passes, to rounding, with no per-draw store
      double mxl = -INFINITY, sel = 0.0, mul = 0.0, m2l = 0.0, cnt = 0.0;
      for (int x = lane; x < S; x += kWave) {
        const double* th = smp + ((int64_t)s * S + x) * 4;
        const double D = d_at(th, pmd, k), phi = th[3];
        const double a = D * phi, b = (1.0 - D) * phi;
        const double lp = lc + (lg3<false, MDFIT_TLOG_NUTS>(yy + a).l - lg3<false, MDFIT_TLOG_NUTS>(a).l) + (lg3<false, MDFIT_TLOG_NUTS>(nn - yy + b).l - lg3<false, MDFIT_TLOG_NUTS>(b).l) -
                          (lg3<false, MDFIT_TLOG_NUTS>(nn + phi).l - lg3<false, MDFIT_TLOG_NUTS>(a + b).l);
        if (lp == -INFINITY) {
          // exp(lp - mx) = 0 for every mx: nothing to add (and with mxl still
          // -inf the else branch would form exp(-inf + inf) = NaN)
        } else if (lp > mxl) {
          sel = sel * pexp(mxl - lp) + 1.0;
          mxl = lp;
        } else {
          sel += pexp(lp - mxl);
        }
        cnt += 1.0;
        const double dlt = lp - mul;
        mul += dlt / cnt;
        m2l = fma(dlt, lp - mul, m2l);
      }
      const double mx = wmax(mxl);
      const double se = wsum(cnt > 0.0 ? sel * pexp(mxl - mx) : 0.0);
      const double mean = wsum(cnt * mul) / S;
      const double dm = mul - mean;
      const double var = wsum(m2l + cnt * dm * dm) / S;
      const double lppd = mx + log(se) - log((double)S);
      if (lane == 0) s_waic[s][col] = -2.0 * (lppd - var);
      __syncthreads();
    }
  }
  __syncthreads();
  // ---- n_sigma x3, asymmetry (fits.py:194-227): lane = point ------------------
  {
    const double v30 = lane < kNPos ? 1.0 : 0.0;
    const int p = lane < kNPos ? lane : 0;
    const double dP = s_waic[0][p], dN = s_waic[1][p];
    const double d = v30 * (dP - dN);
    const double md = wsum(d) / kNPos;
    const double var = wsum(v30 * (d - md) * (d - md)) / kNPos;
    const double ns = (wsum(v30 * dN) - wsum(v30 * dP)) / sqrt(kNPos * var);
    // forward / reverse: 15 points each
    const double vf = lane < kNHalf ? 1.0 : 0.0;
    const int pf = lane < kNHalf ? lane : 0;
    const double df = vf * (s_waic[2][pf] - s_waic[4][pf]);
    const double mdf = wsum(df) / kNHalf;
    const double varf = wsum(vf * (df - mdf) * (df - mdf)) / kNHalf;
    const double nsf = (wsum(vf * s_waic[4][pf]) - wsum(vf * s_waic[2][pf])) / sqrt(kNHalf * varf);
    const int pr_ = lane < kNHalf ? kNHalf + lane : kNHalf;
    const double dr = vf * (s_waic[3][pr_] - s_waic[5][pr_]);
    const double mdr = wsum(dr) / kNHalf;
    const double varr = wsum(vf * (dr - mdr) * (dr - mdr)) / kNHalf;
    const double nsr = (wsum(vf * s_waic[5][pr_]) - wsum(vf * s_waic[3][pr_])) / sqrt(kNHalf * varr);
    // asymmetry: PMD-all vs concat(PMD-fwd, PMD-rev).  Lanes >= 30 (v30 = 0) read
    // a written entry: s_waic[3][0..14] is never written (the reverse fit has
    // points 15..29 only), and 0 * a stale LDS NaN there made the sums NaN --
    // whenever the kernel before on that CU had left one (round 4)
    const double fr = lane < kNHalf ? s_waic[2][p] : s_waic[3][lane < kNPos ? p : kNHalf];
    const double dc = v30 * (dP - fr);
    const double mdc = wsum(dc) / kNPos;
    const double varc = wsum(v30 * (dc - mdc) * (dc - mdc)) / kNPos;
    const double asy = (wsum(v30 * fr) - wsum(v30 * dP)) / sqrt(kNPos * varc);
    if (lane == 0) {
      s_rec[MDFIT_F_N_SIGMA] = ns;
      s_rec[MDFIT_F_N_SIGMA_FORWARD] = nsf;
      s_rec[MDFIT_F_N_SIGMA_REVERSE] = nsr;
      s_rec[MDFIT_F_ASYMMETRY] = asy;
    }
  }
  // ---- means (fits.py:266-270, 329, 350) ---------------------------------------
  {
    double mdm = 0.0;
    for (int x = lane; x < S; x += kWave) mdm += smp[(int64_t)x * 4 + 1] + smp[(int64_t)x * 4 + 2];
    mdm = wsum(mdm) / S;
    if (lane == 0) {
      s_rec[MDFIT_F_Q_MEAN] = s_rec[MDFIT_F_DIAG + 0];
      s_rec[MDFIT_F_CONCENTRATION_MEAN] = s_rec[MDFIT_F_DIAG + 3];
      s_rec[MDFIT_F_D_MAX_MARGINALIZED_MEAN] = mdm;
      s_rec[MDFIT_F_Q_MEAN_FORWARD] = s_rec[MDFIT_F_DIAG + 2 * MDFIT_DIAG_STRIDE + 0];
      s_rec[MDFIT_F_Q_MEAN_REVERSE] = s_rec[MDFIT_F_DIAG + 3 * MDFIT_DIAG_STRIDE + 0];
    }
  }
  __syncthreads();
  // ---- posterior predictive median / HPDI (fits.py:89-120) ---------------------
  // columns 0..29 of the PMD-all chain, then position 0 of data_forward under the
  // forward and the reverse PMD chains (the latter is the :343-348 quirk)
  for (int job = 0; job < kNPos + 2; ++job) {
    const int s = job < kNPos ? 0 : job - kNPos + 2;
    const int col = job < kNPos ? job : 0;
    const int k = col < kNHalf ? col : col - kNHalf;
    const double nn = s_N[col];
    double m3[3];
#ifdef MDFIT_DEV_NOPRED
    if (true) {
      m3[0] = m3[1] = m3[2] = nn;
#else
    if (nn == 0.0) {
      m3[0] = m3[1] = m3[2] = NAN;
#endif
    } else {
      const Stream st = make_stream(o.seed, o.index_base + t, s);
      bool bad = false;
      for (int x = lane; x < S; x += kWave) {
        const int64_t cnt = predictive_count(st, x, col, k, nn, smp + ((int64_t)s * S + x) * 4);
        bad = bad || cnt < 0;
        s_c[x] = (uint32_t)(cnt < 0 ? 0 : cnt);
      }
      __syncthreads();
      if (__any(bad)) {  // (wave-uniform) the oracle: any NaN fraction -> NaN median and HPDI
        m3[0] = m3[1] = m3[2] = NAN;
      } else {
#if MDFIT_REG_SORT
        if (S > kWave * 8 && S <= kWave * 16)
          reg_sort_u32<16>(s_c, S);
        else
#endif
          lds_sort_u32(s_c, S);
        median_hpdi_counts(s_c, S, nn, m3);
      }
      __syncthreads();
    }
    if (lane == 0) {
      if (job < kNPos && pred != nullptr)
#pragma unroll
        for (int q = 0; q < 3; ++q) pred[t * (MDFIT_NPRED * kNPos) + q * kNPos + col] = (float)m3[q];
      if (job == 0) {
        s_rec[MDFIT_F_D_MAX] = m3[0];
        s_rec[MDFIT_F_D_MAX_LOWER_HPDI] = m3[1];
        s_rec[MDFIT_F_D_MAX_UPPER_HPDI] = m3[2];
      }
      if (job == kNPos) s_rec[MDFIT_F_D_MAX_FORWARD] = m3[0];
      if (job == kNPos + 1) s_rec[MDFIT_F_D_MAX_REVERSE] = m3[0];
    }
  }
  __syncthreads();
  // the mismatch counts and the noise scratch reuse the draws' LDS (the kernel
  // is LDS-limited: 8.6 -> 6.7 KB per wave; the launch sizes it >= 2 KB)
  uint32_t* s_mm = s_c;
  double* s_tmp = reinterpret_cast<double*>(s_c + kNPos * kNMM);
  if (gmm != nullptr)
    for (int x = lane; x < kNPos * kNMM; x += kWave) s_mm[x] = gmm[t * (kNPos * kNMM) + x];
  __syncthreads();
  record_sums_noise(lane, s_y, s_N, s_mm, gmm != nullptr, s_rec, s_tmp);
  __syncthreads();
  for (int x = lane; x < MDFIT_NOUT; x += kWave) out[t * MDFIT_NOUT + x] = s_rec[x];
  if (lane == 0) status[t] = stt;
}

// potential + gradient of item i (model 0 PMD / 1 null, subset 0 all / 1 fwd /
// 2 rev) at v, by the chain kernel's own layout and code (parity tests)
__global__ __launch_bounds__(kWave) void nuts_potential_kernel(const int32_t* __restrict__ model,
                                                               const int32_t* __restrict__ subset,
                                                               const uint32_t* __restrict__ gy,
                                                               const uint32_t* __restrict__ gN,
                                                               const double* __restrict__ gv, int64_t n,
                                                               double* __restrict__ U, double* __restrict__ g) {
  const int64_t it = blockIdx.x;
  if (it >= n) return;
  const int lane = threadIdx.x;
  const bool whole = subset[it] == 0;
  const int dir = subset[it] == 2 ? 1 : 0;
  // the component-distributed potential of nuts_chain_cd (PPL 1): lane k of a
  // row = |z| - 1, rows 0 / 1 = forward / reverse (whole) or the subset's row
  const int k = lane & 15, hh = (lane & 31) >> 4;
  PointData pd[1];
  pd[0].pmd = model[it] == 0;
  pd[0].valid = (whole ? lane < 32 : lane < 16) && k < kNHalf;
  pd[0].k = pd[0].valid ? k : 0;
  const int col = pd[0].valid ? (whole ? hh : dir) * kNHalf + k : 0;
  pd[0].y = pd[0].valid ? (double)gy[it * kLD + col] : 0.0;
  pd[0].N = pd[0].valid ? (double)gN[it * kLD + col] : 0.0;
  const PotC pc = potential_cd<1>(pd, gv[it * 4 + (lane & 3)], whole);
  if (lane < 4) {
    if (lane == 0) U[it] = pc.U;
    g[it * 4 + lane] = pc.g;
  }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
// Register-only throughput probe of the sampler's point evaluation: the chain
// kernel's potential_cd (value + gradient of 15 points per 16-lane slot, the
// transform of the position, the five row sums) in the chain kernel's lane
// layout and at its occupancy (MDFIT_NUTS_CD_WAVES waves per SIMD), on a
// representative argument mix (a = D phi below 10: the shifted lnGamma, the
// others not -- as in typical chains).  Useful work: 60 point-evaluations per
// wave-iteration (4 slots x 15 points), the unit of bench.py's NUTS
// compute_roofline.
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(MDFIT_NUTS_CD_WAVES))) void nuts_probe_kernel(
    int iters, double* __restrict__ sink) {
  const int lane = threadIdx.x;
  const int i = lane & 15;
  PointData pd[1];
  pd[0].valid = i < kNHalf;
  pd[0].pmd = true;
  pd[0].k = pd[0].valid ? i : 0;
  pd[0].N = pd[0].valid ? 1.0e5 + 1000.0 * lane : 0.0;
  pd[0].y = 0.01 * pd[0].N;
  const int c = lane & 3;
  double x = c == 0 ? -0.5 : (c == 1 ? -3.0 : (c == 2 ? -4.0 : 6.0));
  double acc = 0.0;
  for (int it = 0; it < iters; ++it) {
    const PotC P = potential_cd<1>(pd, x, false);
    acc += P.U;
    x += 1e-12 * P.g;  // loop-carried: no hoisting
  }
  sink[(int64_t)blockIdx.x * kWave + lane] = acc + x;
}

int peak_probe(int64_t n_waves, int iters, double* sink, hipStream_t s) {
  hipLaunchKernelGGL(nuts_probe_kernel, dim3((unsigned)n_waves), dim3(kWave), 0, s, iters, sink);
  return host::check_launch("nuts_probe_kernel");
}

int potential(const int32_t* model, const int32_t* subset, const uint32_t* y, const uint32_t* N, const double* v,
              int64_t n, double* U, double* g, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(nuts_potential_kernel, dim3((unsigned)n), dim3(kWave), 0, s, model, subset, y, N, v, n, U, g);
  return host::check_launch("nuts_potential_kernel");
}

int64_t workspace_bytes(int64_t n_taxa, int num_samples) {
  return kSamplesOffset + n_taxa * MDFIT_NSUBFIT * (int64_t)(num_samples > 0 ? num_samples : 0) * 4 * 8;
}

int fit_batch(const uint32_t* y, const uint32_t* N, const uint32_t* mm, int64_t n_taxa, const mdfit_opts& o,
              double* out, float* pred, int32_t* status, void* workspace, hipStream_t s) {
  if (o.num_samples < 2 || o.num_samples > kMaxSamples)
    return host::set_err(MDFIT_E_ARG, "num_samples must be in [2, 4096]");
  if (o.num_warmup < 0) return host::set_err(MDFIT_E_ARG, "num_warmup < 0");
  int* ws = (int*)workspace;
  double* samples = (double*)((char*)workspace + kSamplesOffset);
  // diag slots 4..7 are written by the chains; zero the record first
  if (hipMemsetAsync(out, 0, (size_t)n_taxa * MDFIT_NOUT * sizeof(double), s) != hipSuccess)
    return host::check_launch("hipMemsetAsync(out)");
  constexpr int kPPL = 1;  // (PPL 2, two points per lane: 0.91x at C3, DESIGN_HISTORY)
  // (MDFIT_DEV_PER_CU: waves per CU forced, development A/B; the chain
  // kernel's waves never wait on each other, so any grid drains)
  const char* force = std::getenv("MDFIT_DEV_PER_CU");
  auto chain = nuts_chain_cd<kPPL>;
  const int64_t g = host::fit_grid(chain, 4 * n_taxa, kPPL == 1 ? 2 : 4, 0, force ? std::atoi(force) : 0);
  host::prof_mark(1, s);
  host::debug_poison(s);
  hipLaunchKernelGGL(chain, dim3((unsigned)g), dim3(kWave), 0, s, y, N, n_taxa, o, out, ws, samples);
  if (int rc = host::check_launch("nuts_chain_cd")) return rc;
  host::prof_mark(2, s);
  const size_t elt = sizeof(uint32_t);
  size_t sv_bytes = elt;
  while (sv_bytes < (size_t)o.num_samples * elt) sv_bytes <<= 1;  // the sort pads to 2^k
  // (the noise's counts and scratch reuse it after the draws: 1440 + 512 B)
  sv_bytes = sv_bytes < 2048 ? 2048 : sv_bytes;
  host::debug_poison(s);
  hipLaunchKernelGGL(nuts_post_kernel, dim3((unsigned)n_taxa), dim3(kWave), sv_bytes, s, y, N, mm, n_taxa, o,
                     samples, out, pred, status);
  return host::check_launch("nuts_post_kernel");
}

}  // namespace mdfit::nuts

#ifdef MDFIT_STAMP
extern "C" int mdfit_nuts_set_stamp(unsigned long long* buf) {
  (void)hipMemcpyToSymbol(HIP_SYMBOL(mdfit::nuts::g_nuts_stamp), &buf, sizeof(buf));
  return 0;
}
#endif
