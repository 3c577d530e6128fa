// mdfit_hpdi.h — MDFIT-HPDI v1 on the device: the 68 % highest-probability
// window of the MAP predictive BetaBinomial(alpha, beta, N), the MAP counterpart
//  of numpyro.diagnostics.hpdi(obs / N, prob=0.68) over the
// reference's predictive draws (/root/reference/metadamage/fits.py:112-120,
// :260-261).
//
// Definition (oracle/mdfit_hpdi.c has the full statement and the point-by-point
// reference `hp_greedy`): the pmf is unimodal for phi > 2, so the shortest 68 %
// window grows from the mode by adding the more probable neighbour (a tie adds
// the lower one) until it holds >= 0.68.  Same spec as the oracle's `hp_window`:
//   * sd <= 100 points, or the mode alone holds 0.68: that greedy, one point per
//     step through the ratio p(y+1)/p(y) -- `prep_position`, inline in K4a;
//   * otherwise ("wide" windows) Newton on the level t of
//     {y : ln p(y) >= ln p(m) + t} (or, when the window is clamped at 0 / N, on
//     its free end in a log variable), the window mass by Euler-Maclaurin over
//     exact end sums + 6-point Gauss-Legendre panels of the continuous pmf, then
//     the point-by-point fix-up that enforces the greedy's stopping rule and
//     level-set property -- `Wide`, a per-lane state machine run by K4b.
//
// GPU shape.  K4a (one lane per position) classifies, runs the greedy windows
// and appends the wide ones (their setup: mode, p(mode), sd, the lnGamma
// anchors) to a compacted list; K4b is persistent: every lane owns one wide
// window at a time and refills from the list when it finishes, and every trip
// each lane advances its state machine to its next pmf evaluation, so the ~250
// FP64 instructions of ln p(x) sit at ONE site that all busy lanes execute
// together whatever phase (root, quadrature node, fix-up) they are in.
// ln p(x) - ln p(m) comes from lnGamma differences against the mode
// (lgdiff-style: no subtraction of two ~1e11 lnGamma values at N ~ 4e9), with
// the digamma of the same arguments from the same log / reciprocal.
#pragma once

#include <hip/hip_runtime.h>

#include "mdfit_special.h"

namespace mdfit {
namespace hpdi {

#ifndef MDFIT_HPDI_UNROLL
#define MDFIT_HPDI_UNROLL 1
#endif
#ifndef MDFIT_HPDI_FLAT_ROOT
#define MDFIT_HPDI_FLAT_ROOT 1  // the two ends' Newton root steps as one per-lane loop (wide_iter)
#endif
#ifndef MDFIT_HPDI_FLAT_GL
#define MDFIT_HPDI_FLAT_GL 1  // the Gauss-Legendre panels as one per-lane loop (wide_mass)
#endif

// diagnostic builds only (-DMDFIT_HPDI_COUNT): per site k, lane executions
// [2k] and wave issues [2k+1] -- the SIMD efficiency of the loops
#ifdef MDFIT_HPDI_COUNT
__device__ unsigned long long g_hpdi_cnt[32];
#define HPDI_CNT(k)                                                                  \
  do {                                                                               \
    atomicAdd(&::mdfit::hpdi::g_hpdi_cnt[2 * (k)], 1ull);                                         \
    if ((int)__lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1)            \
      atomicAdd(&::mdfit::hpdi::g_hpdi_cnt[2 * (k) + 1], 1ull);                                   \
  } while (0)
#else
#define HPDI_CNT(k) ((void)0)
#endif

constexpr double kMass = 0.68;
#ifndef MDFIT_HPDI_SIG_GREEDY
#define MDFIT_HPDI_SIG_GREEDY 100.0
#endif
constexpr double kSigGreedy = MDFIT_HPDI_SIG_GREEDY;
constexpr double kT0 = -0.49447329849;  // -Z68^2 / 2
constexpr double kK0 = 16.0;
constexpr double kLV = 4.0;
constexpr double kLX = 2.5;
#ifndef MDFIT_HPDI_STOP
#define MDFIT_HPDI_STOP 16.0
#endif
constexpr double kStop = MDFIT_HPDI_STOP;  // counts: the exact fix-up walk finishes
#ifndef MDFIT_HPDI_ROOT_TOL
#define MDFIT_HPDI_ROOT_TOL 0.05
#endif
constexpr double kRootTol = MDFIT_HPDI_ROOT_TOL;  // counts: a window end's Newton root is settled
constexpr double kGLX[3] = {0.2386191860831969, 0.6612093864662645, 0.9324695142031521};
constexpr double kGLW[3] = {0.4679139345726910, 0.3607615730481386, 0.1713244923791704};

// Stirling remainder from r = 1/z (z >= 10)
__device__ __forceinline__ double rem_r(double r) {
  const double r2 = r * r;
  double sl = fma(r2, -1.0 / 156.0, 691.0 / 360360.0);
  sl = fma(r2, -sl, 1.0 / 1188.0);
  sl = fma(r2, -sl, 1.0 / 1680.0);
  sl = fma(r2, -sl, 1.0 / 1260.0);
  sl = fma(r2, -sl, 1.0 / 360.0);
  sl = fma(r2, -sl, 1.0 / 12.0);
  return r * sl;
}

// psi(z) - ln z from r = 1/z (z >= 10)
__device__ __forceinline__ double psi_rem_r(double r) {
  const double r2 = r * r;
  double sp = fma(r2, -1.0 / 12.0, 691.0 / 32760.0);
  sp = fma(r2, -sp, 1.0 / 132.0);
  sp = fma(r2, -sp, 1.0 / 240.0);
  sp = fma(r2, -sp, 1.0 / 252.0);
  sp = fma(r2, -sp, 1.0 / 120.0);
  sp = fma(r2, -sp, 1.0 / 12.0);
  return -0.5 * r - r2 * sp;
}

// One lnGamma pair anchored at z = base argument at the mode: precomputed
// ln z, 1/z and the remainder (z >= 10) or lnGamma(z) (z < 10).
struct Anchor {
  double z, lz, iz, c;  // c = rem(z) (z >= 10) or lnGamma(z) (z < 10)
};

__device__ __forceinline__ Anchor make_anchor(double z) {
  Anchor A;
  A.z = z;
  if (z >= 10.0) {
    A.iz = rcp(z);
    A.lz = flog(z);
    A.c = rem_r(A.iz);
  } else {
    A.iz = 0.0;
    A.lz = 0.0;
    A.c = lgam(z);
  }
  return A;
}

// lnGamma(z + h) - lnGamma(z) and psi(z + h) (want_ps)
template <bool kPs>
__device__ __forceinline__ double pair(const Anchor& A, double h, double& ps) {
  const double z1 = A.z + h;
  if (A.z >= 10.0 && z1 >= 10.0) {
    const double t = flog1p(h * A.iz);
    const double r1 = rcp(z1);
    if (kPs) ps = (A.lz + t) + psi_rem_r(r1);
    return fma(A.z - 0.5 + h, t, h * (A.lz - 1.0)) + (rem_r(r1) - A.c);
  }
  const LG3 l = lg3<false>(z1);
  if (kPs) ps = l.p;
  return l.l - (A.z >= 10.0 ? lgam(A.z) : A.c);
}

struct Pmf {
  double N, a, b, m, pm;
  Anchor Aa, A1, Bb, B1;  // m+alpha, m+1, N-m+beta, N-m+1
};

// g(x) = ln p(x) - ln p(m); with kS also s(x) = d/dx ln p(x)
template <bool kS>
__device__ __forceinline__ double gfun(const Pmf& P, double x, double& s) {
  const double h = x - P.m;
  double p1 = 0.0, p2 = 0.0, p3 = 0.0, p4 = 0.0;
  const double g = (pair<kS>(P.Aa, h, p1) - pair<kS>(P.A1, h, p2)) + (pair<kS>(P.Bb, -h, p3) - pair<kS>(P.B1, -h, p4));
  if (kS) s = (p1 - p2) - (p3 - p4);
  return g;
}
__device__ __forceinline__ double g_of(const Pmf& P, double x) {
  double s;
  return gfun<false>(P, x, s);
}
__device__ __forceinline__ double f_of(const Pmf& P, double x) { return exp(g_of(P, x)); }

// p(y+1) / p(y)
__device__ __forceinline__ double ratio(const Pmf& P, double y) {
  return ((P.N - y) * (y + P.a)) * rcp((y + 1.0) * (P.N - y - 1.0 + P.b));
}


__device__ __forceinline__ double fexp_g(const Pmf& P, double x) {
  double s;
  return exp(gfun<false>(P, x, s));
}

// ---------------------------------------------------------------------------
// K4a: classification + the greedy (the definition, one point per step)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void greedy_window(const Pmf& P, double& lo, double& hi) {
  double A = P.m, B = P.m;
  const double N = P.N;
  double M = P.pm;
  double pl = A > 0.0 ? P.pm * rcp(ratio(P, A - 1.0)) : 0.0;
  double pr = B < N ? P.pm * ratio(P, B) : 0.0;
  while (M < kMass && (pl > 0.0 || pr > 0.0)) {
    if (pl >= pr) {
      A -= 1.0;
      M += pl;
      pl = A > 0.0 ? pl * rcp(ratio(P, A - 1.0)) : 0.0;
    } else {
      B += 1.0;
      M += pr;
      pr = B < N ? pr * ratio(P, B) : 0.0;
    }
  }
  lo = A;
  hi = B;
}

// the setup of a wide window, as K4a hands it to K4b
struct WideRec {
  double N, a, b, m, pm, sd, mu;
  double lz[4], iz[4], c[4];  // anchors m+alpha, m+1, N-m+beta, N-m+1 (z recomputed)
  int64_t item;               // taxon * 30 + position (or the array index)
};

__device__ __forceinline__ void set_pmf(Pmf& P, double N, double a, double b, double m, double pm) {
  P.N = N;
  P.a = a;
  P.b = b;
  P.m = m;
  P.pm = pm;
}

// window of one position: returns true when done here (lo, hi set), false
// when it is wide (rec filled)
__device__ __forceinline__ bool prep_position(double N, double a, double b, double& lo, double& hi, WideRec& rec) {
  if (!(a > 0.0)) {
    lo = hi = 0.0;
    return true;
  }
  if (!(b > 0.0)) {
    lo = hi = N;
    return true;
  }
  const double phi = a + b;
  double m = ceil(((a - 1.0) * N - (b - 1.0)) / (phi - 2.0));
  m = m < 0.0 ? 0.0 : (m > N ? N : m);
  const double pm = exp(bb_logpmf_ab(m, N, a, b, phi));
  const double sd = sqrt(N * a * b * (phi + N) / (phi * phi * (phi + 1.0)));
  if (sd <= kSigGreedy || pm >= kMass) {
    Pmf P;
    set_pmf(P, N, a, b, m, pm);
    greedy_window(P, lo, hi);
    return true;
  }
  rec.N = N;
  rec.a = a;
  rec.b = b;
  rec.m = m;
  rec.pm = pm;
  rec.sd = sd;
  rec.mu = N * a / phi;
  const double z[4] = {m + a, m + 1.0, N - m + b, N - m + 1.0};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const Anchor A = make_anchor(z[j]);
    rec.lz[j] = A.lz;
    rec.iz[j] = A.iz;
    rec.c[j] = A.c;
  }
  return false;
}

// ---------------------------------------------------------------------------
// K4b: a wide window (oracle: hp_window's Newton branch), straight-line per
// lane.  Every lane of a wave runs the same loops (the windows differ only in
// trip counts), and each pmf evaluation sits at one site per loop.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_pmf(Pmf& P, const WideRec& r) {
  set_pmf(P, r.N, r.a, r.b, r.m, r.pm);
  const double z[4] = {r.m + r.a, r.m + 1.0, r.N - r.m + r.b, r.N - r.m + 1.0};
  Anchor* an[4] = {&P.Aa, &P.A1, &P.Bb, &P.B1};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    an[j]->z = z[j];
    an[j]->lz = r.lz[j];
    an[j]->iz = r.iz[j];
    an[j]->c = r.c[j];
  }
}

// sum_{y=A}^{B} p(y)/p(m) by the recurrence from one evaluation at A
__device__ __forceinline__ double walk_sum(const Pmf& P, double A, double B, double gA) {
  double v = fexp(gA), s = 0.0;
  for (double y = A; y <= B; y += 1.0) {
    HPDI_CNT(6);
    s += v;
    if (y < B) v *= ratio(P, y);
  }
  return s;
}

// sum_{y=A}^{B} p(y)/p(m) (oracle: hp_mass): exact within kK0 of the support
// ends and for short windows, Euler-Maclaurin elsewhere
__device__ __forceinline__ double wide_mass(const Pmf& P, double A, double B, double sd) {
  const double N = P.N;
  double tot = 0.0, A1 = A, B1 = B;
  // up to three exact walks (left head, right head, or the whole short window):
  // one evaluation site
  for (int w = 0; w < 3; ++w) {
    double ws = 0.0, we = -1.0;
    if (w == 0 && A1 < kK0) {
      ws = A1;
      we = fmin(kK0 - 1.0, B);
    } else if (w == 1 && B1 > N - kK0 && B1 >= A1) {
      ws = fmax(N - kK0 + 1.0, A1);
      we = B1;
    } else if (w == 2 && B1 >= A1 && B1 - A1 < 32.0) {
      ws = A1;
      we = B1;
    }
    if (we >= ws) {
      HPDI_CNT(10);
      tot += walk_sum(P, ws, we, g_of(P, ws));
      if (w == 0) A1 = we + 1.0;
      else if (w == 1) B1 = ws - 1.0;
      else B1 = A1 - 1.0;  // all summed
    }
  }
  if (B1 < A1) return tot;
  const double c = fmin(fmax(P.m, A1), B1);
  double I = 0.0;
#if MDFIT_HPDI_FLAT_GL
  // The same panels and nodes in the same order (part, panel, node), as ONE
  // per-lane loop: a wave issues the largest per-lane node count instead of
  // the sum over parts of the largest panel counts.  Part setup when a lane
  // enters its next non-empty part.
  double v0 = 0.0, dv = 0.0, acc = 0.0;
  bool lg = false, snl = false;
  int kp = 0, j = 0, nd = 0, pi = 0;
  auto setup = [&](int q) -> bool {
    const int part = q >> 1, sub = q & 1;
    const double u0 = part == 0 ? A1 : c, u1 = part == 0 ? c : B1;
    if (!(u1 > u0)) return false;
    const double L = u1 - u0;
    const bool nl = (u0 + P.a) < L, nr = (N - u1 + P.b) < L;
    double a0 = u0, a1 = u1;
    bool snl_ = nl, snr = nr;
    if (nl && nr) {
      const double cm = 0.5 * (u0 + u1), L2 = cm - u0;
      if (sub == 0) {
        a1 = cm;
        snl_ = (u0 + P.a) < L2;
        snr = false;
      } else {
        a0 = cm;
        snl_ = false;
        snr = (N - u1 + P.b) < L2;
      }
    } else if (sub == 1) {
      return false;
    }
    lg = snl_ || snr;
    snl = snl_;
    v0 = lg ? (snl_ ? flog(a0 + P.a) : flog(N - a1 + P.b)) : a0;
    const double v1 = lg ? (snl_ ? flog(a1 + P.a) : flog(N - a0 + P.b)) : a1;
    int k = lg ? (int)ceil((v1 - v0) / kLV) : (int)ceil((a1 - a0) / (kLX * sd));
    kp = k < 1 ? 1 : k;
    dv = (v1 - v0) / kp;
    return true;
  };
  bool have = false;
  while (pi < 4 && !(have = setup(pi))) ++pi;
  while (have) {
    const double w0 = v0 + dv * j, w1 = v0 + dv * (j + 1);
    const double h = 0.5 * (w1 - w0), cc = 0.5 * (w1 + w0);
    const double gx = nd < 3 ? -kGLX[2 - nd] : kGLX[nd - 3];
    const double gw = kGLW[nd < 3 ? 2 - nd : nd - 3];
    HPDI_CNT(2);
    const double v = cc + h * gx;
    const double ev = lg ? fexp(v) : 1.0;
    const double x = lg ? (snl ? ev - P.a : N + P.b - ev) : v;
    acc += gw * ev * fexp(g_of(P, x));
    if (++nd == 6) {
      I += h * acc;
      acc = 0.0;
      nd = 0;
      if (++j == kp) {
        j = 0;
        have = false;
        while (++pi < 4 && !(have = setup(pi))) {
        }
      }
    }
  }
#else
  // parts [A1, c], [c, B1]; a part near both support ends splits at its midpoint
  for (int pi = 0; pi < 4; ++pi) {
    const int part = pi >> 1, sub = pi & 1;
    const double u0 = part == 0 ? A1 : c, u1 = part == 0 ? c : B1;
    if (!(u1 > u0)) continue;
    const double L = u1 - u0;
    const bool nl = (u0 + P.a) < L, nr = (N - u1 + P.b) < L;
    double a0 = u0, a1 = u1;
    bool snl = nl, snr = nr;
    if (nl && nr) {
      const double cm = 0.5 * (u0 + u1), L2 = cm - u0;
      if (sub == 0) {
        a1 = cm;
        snl = (u0 + P.a) < L2;
        snr = false;
      } else {
        a0 = cm;
        snl = false;
        snr = (N - u1 + P.b) < L2;
      }
    } else if (sub == 1) {
      continue;
    }
    const bool lg = snl || snr;
    const double v0 = lg ? (snl ? flog(a0 + P.a) : flog(N - a1 + P.b)) : a0;
    const double v1 = lg ? (snl ? flog(a1 + P.a) : flog(N - a0 + P.b)) : a1;
    int k = lg ? (int)ceil((v1 - v0) / kLV) : (int)ceil((a1 - a0) / (kLX * sd));
    k = k < 1 ? 1 : k;
    const double dv = (v1 - v0) / k;
    for (int j = 0; j < k; ++j) {
      const double w0 = v0 + dv * j, w1 = v0 + dv * (j + 1);
      const double h = 0.5 * (w1 - w0), cc = 0.5 * (w1 + w0);
      double acc = 0.0;
#pragma unroll MDFIT_HPDI_UNROLL
      for (int i = 0; i < 6; ++i) {  // independent evaluations (ILP vs registers: MDFIT_HPDI_UNROLL)
        const double gx = i < 3 ? -kGLX[2 - i] : kGLX[i - 3];
        const double gw = kGLW[i < 3 ? 2 - i : i - 3];
        HPDI_CNT(2);
        const double v = cc + h * gx;
        const double ev = lg ? fexp(v) : 1.0;
        const double x = lg ? (snl ? ev - P.a : N + P.b - ev) : v;
        acc += gw * ev * fexp(g_of(P, x));
      }
      I += h * acc;
    }
  }
#endif
  // Euler-Maclaurin ends: one site for both
  double fe[2], se[2];
#pragma unroll 1
  for (int e = 0; e < 2; ++e) {
    double sx;
    HPDI_CNT(3);
    const double gx = gfun<true>(P, e == 0 ? A1 : B1, sx);
    fe[e] = fexp(gx);
    se[e] = sx;
  }
  return tot + I + 0.5 * (fe[0] + fe[1]) + (fe[1] * se[1] - fe[0] * se[0]) * (1.0 / 12.0);
}

// window [A, B] with absolute mass M -> the greedy's window (oracle: hp_fixup)
__device__ __forceinline__ void wide_fixup(const Pmf& P, double A, double B, double M, double pA, double pB,
                                           double& lo, double& hi) {
  const double N = P.N;
  double pl = A > 0.0 ? pA * rcp(ratio(P, A - 1.0)) : 0.0;
  double pr = B < N ? pB * ratio(P, B) : 0.0;
  for (int guard = 0; guard < (1 << 26); ++guard) {
    HPDI_CNT(7);
    if (M < kMass && (pl > 0.0 || pr > 0.0)) {  // grow
      if (pl >= pr) {
        A -= 1.0;
        M += pl;
        pA = pl;
        pl = A > 0.0 ? pl * rcp(ratio(P, A - 1.0)) : 0.0;
      } else {
        B += 1.0;
        M += pr;
        pB = pr;
        pr = B < N ? pr * ratio(P, B) : 0.0;
      }
      continue;
    }
    if (M < kMass) break;
    const double pe = pB <= pA ? pB : pA;
    if (A < B && M - pe >= kMass) {  // drop the less probable end
      if (pB <= pA) {
        M -= pB;
        pr = pB;
        B -= 1.0;
        pB = pB * rcp(ratio(P, B));
      } else {
        M -= pA;
        pl = pA;
        A += 1.0;
        pA = pA * ratio(P, A - 1.0);
      }
      continue;
    }
    const double pn = pl >= pr ? pl : pr;
    if (!(pn > pe)) break;
    if (pl >= pr) {  // slide toward the level set
      A -= 1.0;
      M += pl;
      pA = pl;
      pl = A > 0.0 ? pl * rcp(ratio(P, A - 1.0)) : 0.0;
    } else {
      B += 1.0;
      M += pr;
      pB = pr;
      pr = B < N ? pr * ratio(P, B) : 0.0;
    }
  }
  lo = A;
  hi = B;
}

// A wide window's state between level iterations: K4b's lanes run one
// iteration per trip and refill with the next window when theirs is settled,
// so a wave's evaluation sites stay busy whatever each window's iteration
// count (the per-window arithmetic is the straight-line sequence of the
// oracle's hp_window; the order windows are processed in changes nothing).
struct Wide {
  Pmf P;
  double sd, mu, g0, gN;
  double t, tL, tH;     // two-sided: the level and its bracket
  double x, lb, hb;     // one-sided: the free end and its bracket
  double xe0, xe1;      // two-sided: the ends (root starts)
  double A, B, M;       // the current window and its mass
  int one, it;
};

__device__ __forceinline__ void wide_start(Wide& W, const WideRec& r) {
  HPDI_CNT(8);
  load_pmf(W.P, r);
  const double N = W.P.N, m = W.P.m, sd = r.sd, mu = r.mu;
  W.sd = sd;
  W.mu = mu;
  // g(0), g(N) (one site) only when that end is within 4 tau of the mode
  const double tau = sqrt(sd * sd + (mu - m) * (mu - m));
  double gE[2];
#pragma unroll 1
  for (int e = 0; e < 2; ++e) {
    const bool inside = e == 0 ? m > 0.0 : m < N;
    const bool near = (e == 0 ? m : N - m) <= 4.0 * tau;
    if (inside && near) HPDI_CNT(0);
    gE[e] = inside ? (near ? g_of(W.P, e == 0 ? 0.0 : N) : -INFINITY) : 0.0;
  }
  W.g0 = gE[0];
  W.gN = gE[1];
  W.t = kT0;
  const bool L0 = m == 0.0 || W.g0 >= W.t, R0 = m == N || W.gN >= W.t;
  W.one = (L0 && !R0) ? 0 : ((R0 && !L0) ? 1 : -1);
  W.x = W.one == 0 ? fmax(mu, m + 1.0) : fmin(mu, m - 1.0);
  W.lb = W.one == 0 ? m : 0.0;
  W.hb = W.one == 0 ? N : m;
  W.tL = -INFINITY;
  W.tH = 0.0;
  W.xe0 = m - sd;  // two-sided ends
  W.xe1 = m + sd;
  W.A = W.B = m;
  W.M = W.P.pm;
  W.it = 0;
}

// one level iteration (oracle: hp_window's loop body); true when settled
__device__ __forceinline__ bool wide_iter(Wide& W) {
  HPDI_CNT(9);
  const Pmf& P = W.P;
  const double N = P.N, m = P.m;
  const int one = W.one, it = W.it;
  const double t = W.t;
  double A, B;
  double xe[2] = {W.xe0, W.xe1};
  bool cl = false, cr = false;
  if (one < 0) {
    cl = m == 0.0 || W.g0 >= t;
    cr = m == N || W.gN >= t;
    // the free ends' roots of g = t (oracle: hp_root): one site for both
#if MDFIT_HPDI_FLAT_ROOT
    // both ends' Newton steps as ONE per-lane loop (end 0's steps, then end
    // 1's: the same arithmetic per end), so a wave issues the largest per-lane
    // total instead of the sum of the per-end maxima
    int e = cl ? (cr ? 2 : 1) : 0;
    if (cl) xe[0] = 0.0;
    double rlo = 0.0, rhi = m, xr = 0.0;
    bool rising = true;
    int k = 0;
    auto start_end = [&](int ee) {
      rlo = ee == 0 ? 0.0 : m;
      rhi = ee == 0 ? m : N;
      rising = ee == 0;
      xr = fmin(fmax(ee == 0 ? xe[0] : xe[1], rlo), rhi);
      k = 0;
    };
    if (e < 2) start_end(e);
    while (e < 2) {
      double sx;
      HPDI_CNT(1);
      const double gx = gfun<true>(P, xr, sx) - t;
      bool fin = fabs(gx) < 1e-12;
      if (!fin) {
        if ((gx < 0.0) == rising) rlo = xr;
        else rhi = xr;
        double xn = sx != 0.0 ? xr - gx / sx : 0.5 * (rlo + rhi);
        if (!(rlo < xn && xn < rhi)) xn = 0.5 * (rlo + rhi);
        const bool conv = fabs(xn - xr) < kRootTol;
        xr = xn;
        fin = conv || ++k >= 60;
      }
      if (fin) {
        if (e == 0) {
          xe[0] = xr;
          e = cr ? 2 : 1;
          if (e == 1) start_end(1);
        } else {
          xe[1] = xr;
          e = 2;
        }
      }
    }
    if (cr) xe[1] = N;
#else
#pragma unroll 1
    for (int e = 0; e < 2; ++e) {
      const bool clamped = e == 0 ? cl : cr;
      if (clamped) {
        xe[e] = e == 0 ? 0.0 : N;
        continue;
      }
      double rlo = e == 0 ? 0.0 : m, rhi = e == 0 ? m : N;
      const bool rising = e == 0;
      double xr = fmin(fmax(xe[e], rlo), rhi);
      for (int k = 0; k < 60; ++k) {
        double sx;
        HPDI_CNT(1);
        const double gx = gfun<true>(P, xr, sx) - t;
        if (fabs(gx) < 1e-12) break;
        if ((gx < 0.0) == rising) rlo = xr;
        else rhi = xr;
        double xn = sx != 0.0 ? xr - gx / sx : 0.5 * (rlo + rhi);
        if (!(rlo < xn && xn < rhi)) xn = 0.5 * (rlo + rhi);
        const bool conv = fabs(xn - xr) < kRootTol;
        xr = xn;
        if (conv) break;
      }
      xe[e] = xr;
    }
#endif
    W.xe0 = xe[0];
    W.xe1 = xe[1];
    A = ceil(xe[0]);
    B = floor(xe[1]);
  } else {
    A = one == 0 ? 0.0 : ceil(W.x);
    B = one == 0 ? floor(W.x) : N;
  }
  const double M = wide_mass(P, A, B, W.sd) * P.pm;
  W.A = A;
  W.B = B;
  W.M = M;
  // the evaluations after the mass: f(x) (one-sided) or s at the two ends
  double pe[2] = {0.0, 0.0};
#pragma unroll 1
  for (int e = 0; e < 2; ++e) {
    const bool need = one >= 0 ? e == 0 : (e == 0 ? !cl : !cr);
    if (!need) continue;
    double sx;
    HPDI_CNT(4);
    const double gx = gfun<true>(P, one >= 0 ? W.x : xe[e], sx);
    pe[e] = one >= 0 ? fexp(gx) * P.pm : sx;
  }
  W.it = it + 1;
  if (one >= 0) {
    const double x = W.x;
    const double fx = pe[0];
    const double F = log(M / (1.0 - M)) - log(kMass / (1.0 - kMass));
    const double jac = one == 0 ? x + P.a : N - x + P.b;
    const double dF = fx * jac * (1.0 / M + 1.0 / (1.0 - M));
    double xn;
    if (one == 0) {
      if (F > 0.0) W.hb = x;
      else W.lb = x;
      xn = exp(log(x + P.a) - F / dF) - P.a;
    } else {
      if (F > 0.0) W.lb = x;
      else W.hb = x;
      xn = N + P.b - exp(log(N - x + P.b) - F / dF);
    }
    if (!(W.lb < xn && xn < W.hb)) xn = 0.5 * (W.lb + W.hb);
    if (fabs(xn - x) < kStop || it >= 40) return true;
    W.x = xn;
    return false;
  }
  if (M >= kMass) W.tL = t;
  else W.tH = t;
  double Dp = 0.0, mv = 0.0;
  if (!cl) {
    Dp += exp(t) / pe[0];
    mv += 1.0 / pe[0];
  }
  if (!cr) {
    Dp += exp(t) / -pe[1];
    mv += 1.0 / -pe[1];
  }
  Dp *= P.pm;
  if (it >= 40) return true;
  double tn;
  if (Dp > 0.0) {
    const double dt = (log(M) - log(kMass)) * M / Dp;
    if (fabs(dt) * mv < kStop) return true;
    tn = t + dt;
  } else {
    tn = 0.5 * (W.tL + W.tH);  // both ends clamped: raise the level
  }
  if (!(W.tL < tn && tn < W.tH)) tn = W.tL > -INFINITY ? 0.5 * (W.tL + W.tH) : t - fmax(1.0, fabs(t));
  W.t = tn;
  return false;
}

// the fix-up from the end pmfs (one site for both)
__device__ __forceinline__ void wide_finish(const Wide& W, double& lo, double& hi) {
  double pAB[2];
#pragma unroll 1
  for (int e = 0; e < 2; ++e) {
    const bool need = e == 0 || W.B != W.A;
    if (need) HPDI_CNT(5);
    pAB[e] = need ? fexp(g_of(W.P, e == 0 ? W.A : W.B)) * W.P.pm : pAB[0];
  }
  wide_fixup(W.P, W.A, W.B, W.M, pAB[0], pAB[1], lo, hi);
}

}  // namespace hpdi
}  // namespace mdfit
