// mdfit_hpdi.h — MDFIT-HPDI v2 on the device: the 68 % highest-probability
// window of the MAP predictive BetaBinomial(alpha, beta, N), the MAP counterpart
//  of numpyro.diagnostics.hpdi(obs / N, prob=0.68) over the
// reference's predictive draws (/root/reference/metadamage/fits.py:112-120,
// :260-261).
//
// Definition (oracle/mdfit_hpdi.c has the full statement and the point-by-point
// reference `hp_greedy`): the pmf is unimodal for phi > 2, so the shortest 68 %
// window grows from the mode by adding the more probable neighbour (a tie adds
// the lower one) until it holds >= 0.68.  Same spec as the oracle's `hp_window`:
//   * sd <= 40 points (round 6; 100 before), or the mode alone holds 0.68: that greedy, one point per
//     step through the ratio p(y+1)/p(y) -- `prep_position`, inline in K4a;
//   * otherwise ("wide" windows) Newton on the level t of
//     {y : ln p(y) >= ln p(m) + t} (or, when the window is clamped at 0 / N, on
//     its free end in a log variable), the window mass by Euler-Maclaurin over
//     exact end sums + 6-point Gauss-Legendre panels of the continuous pmf, then
//     the point-by-point fix-up that enforces the greedy's stopping rule and
//     level-set property -- `Wide`, a per-lane state machine run by K4b.
//   v2 (round 5): the same windows by a shorter path (oracle header): level
//   Newton in z = sqrt(-2t) on sqrt(2) erfinv(M), one-sided Newton on cloglog M,
//   moved root starts, and each iteration's mass = the previous one + the
//   strips the ends moved over, the Euler-Maclaurin ends' f, s doubling as the
//   Newton slopes and the fix-up's end pmfs: 40.6 -> 25.4 ln p per wide window.
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
#define MDFIT_HPDI_SIG_GREEDY 40.0
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
#define MDFIT_HPDI_ROOT_TOL 2.0
#endif
constexpr double kRootTol = MDFIT_HPDI_ROOT_TOL;  // counts: a window end's Newton root is settled
constexpr double kGLX[3] = {0.2386191860831969, 0.6612093864662645, 0.9324695142031521};
constexpr double kGLW[3] = {0.4679139345726910, 0.3607615730481386, 0.1713244923791704};
constexpr double kGL2X = 0.57735026918962576451;  // 1/sqrt(3)
constexpr double kGL3X = 0.77459666924148337704;  // sqrt(3/5)
constexpr double kGL3W0 = 0.88888888888888888889, kGL3W1 = 0.55555555555555555556;
constexpr double kS6 = 0.5;  // strips up to half the local scale: 6 nodes
constexpr double kZ68 = 0.99445788320975304;       // sqrt(2) erfinv(0.68)
constexpr double kCll68 = 0.13053189641996385;     // ln(-ln(1 - 0.68))
constexpr double kD68 = 0.48662348157070173;      // d erf(z / sqrt 2) / dz at kZ68
constexpr double kC2 = 0.49722894160487652;       // the inverse series: kZ68 / 2
constexpr double kC3 = 0.49631549382600754;       //   (2 kZ68^2 + 1) / 6

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

// What one mass evaluation leaves for the next level iteration (oracle:
// hp_mass_t): the window, its Euler-Maclaurin range [A1, B1] (the window less
// its exact heads), the integral over that range, the exact sums, f and s at A1
// and B1.
struct Memo {
  double A1, B1, I, tot, fA, sA, fB, sB;
  bool em;  // [A1, B1] summed by Euler-Maclaurin (else the window is all exact sums)
};

// Gauss-Legendre nodes of a strip between consecutive windows' ends (oracle:
// hp_strip_nodes): 0 empty, 2 / 3 / 6 by its width over the local scale,
// -1 too wide (recompute)
__device__ __forceinline__ int strip_nodes(const Pmf& P, double u0, double u1, double sd) {
  const double lo = fmin(u0, u1), hi = fmax(u0, u1), w = hi - lo;
  if (w == 0.0) return 0;
  const double l = fmin(sd, fmin(lo + P.a, P.N - hi + P.b));
  return w <= 0.02 * l ? 2 : (w <= 0.1 * l ? 3 : (w <= kS6 * l ? 6 : -1));
}

// sum_{y=A}^{B} p(y)/p(m) (oracle: hp_mass): exact within kK0 of the support
// ends and for short windows, Euler-Maclaurin elsewhere; the integral from
// Gauss-Legendre panels split at the mode, or -- when the previous iteration's
// window (mm on entry, `have`) has the same exact heads and both ends moved by
// narrow strips -- its integral plus the strips.  f, s at an unmoved range end
// are the previous ones.  (pA, pB) is the previous window; mm is updated for
// the next iteration.
__device__ __forceinline__ double wide_mass(const Pmf& P, double A, double B, double sd, bool have, double pA,
                                           double pB, Memo& mm) {
  const double N = P.N;
  const Memo& pv = mm;  // (read before mm is rewritten at the end)
  double A1 = A, B1 = B;
  if (A1 < kK0) A1 = fmin(kK0 - 1.0, B) + 1.0;
  if (B1 > N - kK0 && B1 >= A1) B1 = fmax(N - kK0 + 1.0, A1) - 1.0;
  const bool same = have && pv.em && ((A1 == A) == (pv.A1 == pA)) && (A1 == A || (A == pA && A1 == pv.A1)) &&
                    ((B1 == B) == (pv.B1 == pB)) && (B1 == B || (B == pB && B1 == pv.B1));
  const bool shortw = B1 >= A1 && B1 - A1 < 32.0;
  double tot = same ? pv.tot : 0.0;
  // up to three exact walks (left head, right head, the whole short window):
  // one evaluation site
  for (int w = 0; w < 3; ++w) {
    double ws = 0.0, we = -1.0;
    if (w == 0 && !same && A1 > A) {
      ws = A;
      we = A1 - 1.0;
    } else if (w == 1 && !same && B1 < B) {
      ws = B1 + 1.0;
      we = B;
    } else if (w == 2 && shortw) {
      ws = A1;
      we = B1;
    }
    if (we >= ws) {
      HPDI_CNT(10);
      tot += walk_sum(P, ws, we, g_of(P, ws));
    }
  }
  if (B1 < A1 || shortw) {
    mm.A1 = A1;
    mm.B1 = B1;
    mm.tot = tot;
    mm.em = false;
    return tot;
  }
#ifdef X_NOSTRIP
  const int nl = -1, nr = -1;
#else
  const int nl = same ? strip_nodes(P, A1, pv.A1, sd) : -1;
  const int nr = same ? strip_nodes(P, pv.B1, B1, sd) : -1;
#endif
  const bool strips = nl >= 0 && nr >= 0;
  const double c = fmin(fmax(P.m, A1), B1);
  double I = strips ? pv.I : 0.0;
  // The panels as ONE per-lane loop over "parts" -- q = 0..3 the full
  // computation's (part [A1, c] / [c, B1], its halves when near both support
  // ends), q = 4, 5 the strips [A1, pv.A1], [pv.B1, B1] (signed) -- in the
  // oracle's order: a wave issues the largest per-lane node count.
  double v0 = 0.0, dv = 0.0, acc = 0.0;
  bool lg = false, snl = false;
  int kp = 0, j = 0, nd = 0, np = 6, pi = strips ? 4 : 0;
  const int pe = strips ? 6 : 4;
  auto setup = [&](int q) -> bool {
    if (q >= 4) {
      const int n = q == 4 ? nl : nr;
      if (n == 0) return false;
      lg = false;
      v0 = q == 4 ? A1 : pv.B1;
      dv = (q == 4 ? pv.A1 : B1) - v0;
      kp = 1;
      np = n;
      return true;
    }
    const int part = q >> 1, sub = q & 1;
    const double u0 = part == 0 ? A1 : c, u1 = part == 0 ? c : B1;
    if (!(u1 > u0)) return false;
    const double L = u1 - u0;
    const bool nlg = (u0 + P.a) < L, nrg = (N - u1 + P.b) < L;
    double a0 = u0, a1 = u1;
    bool snl_ = nlg, snr = nrg;
    if (nlg && nrg) {
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
    const int k = lg ? (int)ceil((v1 - v0) / kLV) : (int)ceil((a1 - a0) / (kLX * sd));
    kp = k < 1 ? 1 : k;
    dv = (v1 - v0) / kp;
    np = 6;
    return true;
  };
  bool on = false;
  while (pi < pe && !(on = setup(pi))) ++pi;
  while (on) {
    const double w0 = v0 + dv * j, w1 = v0 + dv * (j + 1);
    const double h = 0.5 * (w1 - w0), cc = 0.5 * (w1 + w0);
    double gx, gw;
    if (np == 6) {
      gx = nd < 3 ? -kGLX[2 - nd] : kGLX[nd - 3];
      gw = kGLW[nd < 3 ? 2 - nd : nd - 3];
    } else if (np == 3) {
      gx = (nd - 1) * kGL3X;
      gw = nd == 1 ? kGL3W0 : kGL3W1;
    } else {
      gx = nd == 0 ? -kGL2X : kGL2X;
      gw = 1.0;
    }
    HPDI_CNT(2);
    const double v = cc + h * gx;
    const double ev = lg ? fexp(v) : 1.0;
    const double x = lg ? (snl ? ev - P.a : N + P.b - ev) : v;
    acc += gw * ev * fexp(g_of(P, x));
    if (++nd == np) {
      I += h * acc;
      acc = 0.0;
      nd = 0;
      if (++j == kp) {
        j = 0;
        on = false;
        while (++pi < pe && !(on = setup(pi))) {
        }
      }
    }
  }
  // Euler-Maclaurin ends: one site for both (an unmoved end: the previous values)
  double fA = pv.fA, sA = pv.sA, fB = pv.fB, sB = pv.sB;
#pragma unroll 1
  for (int e = 0; e < 2; ++e) {
    const bool reuse = same && (e == 0 ? A1 == pv.A1 : B1 == pv.B1);
    if (!reuse) {
      double sx;
      HPDI_CNT(3);
      const double fx = fexp(gfun<true>(P, e == 0 ? A1 : B1, sx));
      if (e == 0) {
        fA = fx;
        sA = sx;
      } else {
        fB = fx;
        sB = sx;
      }
    }
  }
  mm.A1 = A1;
  mm.B1 = B1;
  mm.tot = tot;
  mm.I = I;
  mm.fA = fA;
  mm.sA = sA;
  mm.fB = fB;
  mm.sB = sB;
  mm.em = true;
  return tot + I + 0.5 * (fA + fB) + (fB * sB - fA * sA) * (1.0 / 12.0);
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
  double sd, g0, gN;
  double t;             // two-sided: the level
  double tL, tH;        // two-sided: its bracket / one-sided: the free end's (lb, hb)
  double xe0, xe1;      // two-sided: the ends (root starts) / one-sided: xe0 = the free end x
  double sl, sr, dtp;   // two-sided: the ends' slopes, the last level step
  double A, B, M;       // the current window and its mass
  Memo mm;              // the last mass evaluation
  int one, it;
};

__device__ __forceinline__ void wide_start(Wide& W, const WideRec& r) {
  HPDI_CNT(8);
  load_pmf(W.P, r);
  const double N = W.P.N, m = W.P.m, sd = r.sd, mu = r.mu;
  W.sd = sd;
  // g(0), g(N) (one site) only when that end is within 4 tau of the mode
  const double tau = sqrt(sd * sd + (mu - m) * (mu - m));
#pragma unroll 1
  for (int e = 0; e < 2; ++e) {
    const bool inside = e == 0 ? m > 0.0 : m < N;
    const bool near = (e == 0 ? m : N - m) <= 4.0 * tau;
    if (inside && near) HPDI_CNT(0);
    const double g = inside ? (near ? g_of(W.P, e == 0 ? 0.0 : N) : -INFINITY) : 0.0;
    if (e == 0) W.g0 = g;
    else W.gN = g;
  }
  W.t = kT0;
  const bool L0 = m == 0.0 || W.g0 >= W.t, R0 = m == N || W.gN >= W.t;
  W.one = (L0 && !R0) ? 0 : ((R0 && !L0) ? 1 : -1);
  if (W.one >= 0) {
    W.xe0 = W.one == 0 ? fmax(mu, m + 1.0) : fmin(mu, m - 1.0);  // x
    W.tL = W.one == 0 ? m : 0.0;                                  // lb
    W.tH = W.one == 0 ? N : m;                                    // hb
  } else {
    W.tL = -INFINITY;
    W.tH = 0.0;
    W.xe0 = m - sd;  // the ends
    W.xe1 = m + sd;
  }
  W.sl = W.sr = W.dtp = 0.0;
  W.A = W.B = m;
  W.M = W.P.pm;
  W.mm.em = false;
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
    // the free ends' roots of g = t (oracle: hp_root), started from the
    // previous roots moved by the level step over their slopes: both ends'
    // Newton steps as ONE per-lane loop (end 0's steps, then end 1's), so a
    // wave issues the largest per-lane total
    const double xs0 = it > 0 && W.sl > 0.0 ? xe[0] + W.dtp / W.sl : xe[0];
    const double xs1 = it > 0 && W.sr > 0.0 ? xe[1] - W.dtp / W.sr : xe[1];
    int e = cl ? (cr ? 2 : 1) : 0;
    if (cl) xe[0] = 0.0;
    double rlo = 0.0, rhi = m, xr = 0.0;
    bool rising = true;
    int k = 0;
    auto start_end = [&](int ee) {
      rlo = ee == 0 ? 0.0 : m;
      rhi = ee == 0 ? m : N;
      rising = ee == 0;
      xr = fmin(fmax(ee == 0 ? xs0 : xs1, rlo), rhi);
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
    W.xe0 = xe[0];
    W.xe1 = xe[1];
    A = ceil(xe[0]);
    B = floor(xe[1]);
  } else {
    A = one == 0 ? 0.0 : ceil(W.xe0);
    B = one == 0 ? floor(W.xe0) : N;
  }
  const double M = wide_mass(P, A, B, W.sd, it > 0, W.A, W.B, W.mm) * P.pm;
  W.A = A;
  W.B = B;
  W.M = M;
  // after the mass: p at the free end (one-sided) or s at the free ends --
  // the Euler-Maclaurin ends' when those are the window's ends, else one
  // evaluation site
  const Memo& mm = W.mm;
  double pe0 = 0.0, pe1 = 0.0;
#pragma unroll 1
  for (int e = 0; e < 2; ++e) {
    const bool need = one >= 0 ? e == 0 : (e == 0 ? !cl : !cr);
    if (!need) continue;
    const bool atA = one >= 0 ? one == 1 : e == 0;  // the window end in question is A
    double v;
    if (mm.em && (atA ? mm.A1 == A : mm.B1 == B)) {
      v = one >= 0 ? (atA ? mm.fA : mm.fB) * P.pm : (atA ? mm.sA : mm.sB);
    } else {
      double sx;
      HPDI_CNT(4);
      const double gx = gfun<true>(P, e == 0 ? xe[0] : xe[1], sx);  // (one-sided: xe[0] = x)
      v = one >= 0 ? fexp(gx) * P.pm : sx;
    }
    if (e == 0) pe0 = v;
    else pe1 = v;
  }
  W.it = it + 1;
  if (one >= 0) {
    // Newton on the complementary log-log of M against ln(end + alpha) (resp.
    // ln(N - end + beta)): linear for a Gamma-like pmf near the clamped end and
    // in its exponential tail
    const double x = W.xe0;
    const double fx = pe0;
    const double Mc = fmin(M, 1.0 - 1e-16);
    const double Lc = -log1p(-Mc);
    const double F = log(Lc) - kCll68;
    const double jac = one == 0 ? x + P.a : N - x + P.b;
    const double dF = fx * jac / ((1.0 - Mc) * Lc);
    double xn;
    double& lb = W.tL;
    double& hb = W.tH;
    if (one == 0) {
      if (F > 0.0) hb = x;
      else lb = x;
      xn = exp(log(x + P.a) - F / dF) - P.a;
    } else {
      if (F > 0.0) lb = x;
      else hb = x;
      xn = N + P.b - exp(log(N - x + P.b) - F / dF);
    }
    if (!(lb < xn && xn < hb)) xn = 0.5 * (lb + hb);
    if (fabs(xn - x) < kStop || it >= 40) return true;
    W.xe0 = xn;
    return false;
  }
  if (M >= kMass) W.tL = t;
  else W.tH = t;
  double Dp = 0.0, mv = 0.0;
  if (!cl) {
    W.sl = pe0;
    Dp += exp(t) / pe0;
    mv += 1.0 / pe0;
  }
  if (!cr) {
    W.sr = -pe1;
    Dp += exp(t) / -pe1;
    mv += 1.0 / -pe1;
  }
  Dp *= P.pm;
  if (it >= 40) return true;
  double tn;
  if (Dp > 0.0) {
    // Newton in z = sqrt(-2t) on u(M) = sqrt(2) erfinv(M), which is z itself
    // for a Gaussian pmf -- u by its cubic Taylor series about 0.68 (within
    // +-0.3 z-units of it; beyond, the plain Newton step on ln M in t); the
    // stop: the ends would move < kStop counts
    const double z = sqrt(-2.0 * t);
    const double q = (M - kMass) / kD68;
    const double u = kZ68 + q * (1.0 + q * (kC2 + q * kC3));
    const double du = (1.0 + q * (2.0 * kC2 + q * 3.0 * kC3)) / kD68 * Dp * z;
    const double zn = fabs(q) < 0.3 ? z - (u - kZ68) / du : -1.0;
    const double step = zn > 0.0 ? -0.5 * zn * zn - t : (log(M) - log(kMass)) * M / Dp;
    if (fabs(step) * mv < kStop) return true;
    tn = t + step;
  } else {
    tn = 0.5 * (W.tL + W.tH);  // both ends clamped: raise the level
  }
  if (!(W.tL < tn && tn < W.tH)) tn = W.tL > -INFINITY ? 0.5 * (W.tL + W.tH) : t - fmax(1.0, fabs(t));
  W.dtp = tn - t;
  W.t = tn;
  return false;
}

// the fix-up from the end pmfs: the Euler-Maclaurin ends' when those are the
// window's ends, else one site for both
__device__ __forceinline__ void wide_finish(const Wide& W, double& lo, double& hi) {
  const Memo& mm = W.mm;
  double pA = 0.0, pB = 0.0;
#pragma unroll 1
  for (int e = 0; e < 2; ++e) {
    const bool need = e == 0 || W.B != W.A;
    const bool reuse = mm.em && (e == 0 ? mm.A1 == W.A : mm.B1 == W.B);
    if (need && !reuse) HPDI_CNT(5);
    const double v = !need ? pA : (reuse ? (e == 0 ? mm.fA : mm.fB) : fexp(g_of(W.P, e == 0 ? W.A : W.B))) * W.P.pm;
    if (e == 0) pA = v;
    else pB = v;
  }
  wide_fixup(W.P, W.A, W.B, W.M, pA, pB, lo, hi);
}

}  // namespace hpdi
}  // namespace mdfit
