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

constexpr double kMass = 0.68;
constexpr double kSigGreedy = 100.0;
constexpr double kT0 = -0.49447329849;  // -Z68^2 / 2
constexpr double kK0 = 16.0;
constexpr double kLV = 4.0;
constexpr double kLX = 2.5;
constexpr double kStop = 4.0;
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
// K4b: the wide-window state machine (oracle: hp_window's Newton branch)
// ---------------------------------------------------------------------------
// phases of the main machine
enum : int {
  W_G0 = 0, W_GN, W_DECIDE,
  W_ONE_TOP, W_ONE_FX,                         // one-sided Newton
  W_TWO_TOP, W_TWO_ROOTR, W_TWO_MASS, W_TWO_SL, W_TWO_SR,  // two-sided Newton
  W_FIX_A, W_FIX_B, W_FIX_WALK, W_DONE,
  // sub-machines (return to `ret`)
  W_ROOT, W_MASS_BEGIN, W_MASS_HR, W_MASS_MID, W_MASS_NODES, W_MASS_ENDA, W_MASS_ENDB,
  W_EXACT_WALK
};

struct Wide {
  Pmf P;
  double sd, mu, g0, gN, t, tL, tH, x, lb, hb, xl, xr, Dp, mv, M, A, B;
  int phase, ret, it, one, cl, cr;
  // root sub-machine
  double r_lo, r_hi, r_x;
  int r_it, r_rising, r_ret;
  // mass sub-machine
  double m_A1, m_B1, m_tot, m_I, m_c, m_e, fA, sA;
  double p_u0, p_u1, p_v0, p_v1, p_h, p_cm;
  int p_part, p_sub, p_j, p_k, p_i, p_nl, p_nr, m_ret, m_mode;
  // exact-walk sub-machine (sum_{y=ew_y..ew_end} p(y)/p(m))
  double ew_y, ew_end, ew_v, ew_s;
  int ew_ret;
  // fix-up
  double pA, pB, pl, pr;
  // the pending evaluation
  double req_x;
  int req_s;
  double res_g, res_s;
};

__device__ __forceinline__ void wide_load(Wide& W, const WideRec& r) {
  set_pmf(W.P, r.N, r.a, r.b, r.m, r.pm);
  const double z[4] = {r.m + r.a, r.m + 1.0, r.N - r.m + r.b, r.N - r.m + 1.0};
  Anchor* an[4] = {&W.P.Aa, &W.P.A1, &W.P.Bb, &W.P.B1};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    an[j]->z = z[j];
    an[j]->lz = r.lz[j];
    an[j]->iz = r.iz[j];
    an[j]->c = r.c[j];
  }
  W.sd = r.sd;
  W.mu = r.mu;
  W.phase = W_G0;
}

// the sub-part (p_part, p_sub) of the mass integral: bounds and variable
__device__ __forceinline__ bool part_setup(Wide& W) {
  // parts: 0 = [A1, c], 1 = [c, B1]; a part with both ends near a support end
  // splits at its midpoint into sub-parts 0 / 1 (oracle: hp_part)
  for (; W.p_part < 2; ++W.p_part, W.p_sub = 0) {
    const double u0 = W.p_part == 0 ? W.m_A1 : W.m_c;
    const double u1 = W.p_part == 0 ? W.m_c : W.m_B1;
    if (!(u1 > u0)) continue;
    const double L = u1 - u0;
    const bool nl = (u0 + W.P.a) < L, nr = (W.P.N - u1 + W.P.b) < L;
    double a0 = u0, a1 = u1;
    bool snl = nl, snr = nr;
    if (nl && nr) {
      const double cmid = 0.5 * (u0 + u1);
      const double L2 = cmid - u0;
      if (W.p_sub == 0) {
        a1 = cmid;
        snl = (u0 + W.P.a) < L2;
        snr = false;
      } else if (W.p_sub == 1) {
        a0 = cmid;
        snl = false;
        snr = (W.P.N - u1 + W.P.b) < L2;
      } else {
        continue;
      }
    } else if (W.p_sub > 0) {
      continue;
    }
    W.p_u0 = a0;
    W.p_u1 = a1;
    W.p_nl = snl;
    W.p_nr = snr;
    if (snl || snr) {
      W.p_v0 = snl ? flog(a0 + W.P.a) : flog(W.P.N - a1 + W.P.b);
      W.p_v1 = snl ? flog(a1 + W.P.a) : flog(W.P.N - a0 + W.P.b);
      const int k = (int)ceil((W.p_v1 - W.p_v0) / kLV);
      W.p_k = k < 1 ? 1 : k;
    } else {
      const int k = (int)ceil((a1 - a0) / (kLX * W.sd));
      W.p_k = k < 1 ? 1 : k;
    }
    W.p_j = 0;
    W.p_i = 0;
    return true;
  }
  return false;
}

// next quadrature node of the current sub-part -> req_x (and the weight *
// jacobian factor kept in p_h / p_cm); false when the part set is exhausted
__device__ __forceinline__ double node_x(Wide& W, double& wj) {
  const int i = W.p_i;
  const double gx = i < 3 ? -kGLX[2 - i] : kGLX[i - 3];
  const double gw = kGLW[i < 3 ? 2 - i : i - 3];
  const int k = W.p_k, j = W.p_j;
  if (W.p_nl || W.p_nr) {
    const double w0 = W.p_v0 + (W.p_v1 - W.p_v0) * j / k, w1 = W.p_v0 + (W.p_v1 - W.p_v0) * (j + 1) / k;
    const double h = 0.5 * (w1 - w0), c = 0.5 * (w1 + w0);
    const double v = c + h * gx;
    const double ev = exp(v);
    wj = gw * h * ev;
    return W.p_nl ? ev - W.P.a : W.P.N + W.P.b - ev;
  }
  const double L = W.p_u1 - W.p_u0;
  const double w0 = W.p_u0 + L * j / k, w1 = W.p_u0 + L * (j + 1) / k;
  const double h = 0.5 * (w1 - w0), c = 0.5 * (w1 + w0);
  wj = gw * h;
  return c + h * gx;
}

// Advance the machine (consuming the last evaluation when `have`) until it
// requests the next one (returns true) or finishes (returns false).
__device__ __forceinline__ bool wide_step(Wide& W, bool have) {
  const double N = W.P.N, m = W.P.m;
  for (int guard = 0; guard < 4096; ++guard) {
    switch (W.phase) {
      case W_G0:
        if (!have) {
          if (m > 0.0) { W.req_x = 0.0; W.req_s = 0; return true; }
          W.g0 = 0.0;
        } else {
          W.g0 = W.res_g;
          have = false;
        }
        W.phase = W_GN;
        break;
      case W_GN:
        if (!have) {
          if (m < N) { W.req_x = N; W.req_s = 0; return true; }
          W.gN = 0.0;
        } else {
          W.gN = W.res_g;
          have = false;
        }
        W.phase = W_DECIDE;
        break;
      case W_DECIDE:
        W.t = kT0;
        {
          const bool L0 = m == 0.0 || W.g0 >= W.t, R0 = m == N || W.gN >= W.t;
          W.one = (L0 && !R0) ? 0 : ((R0 && !L0) ? 1 : -1);
        }
        W.it = 0;
        if (W.one >= 0) {
          W.x = W.one == 0 ? fmax(W.mu, m + 1.0) : fmin(W.mu, m - 1.0);
          W.lb = W.one == 0 ? m : 0.0;
          W.hb = W.one == 0 ? N : m;
          W.phase = W_ONE_TOP;
        } else {
          W.tL = -INFINITY;
          W.tH = 0.0;
          W.xl = m - W.sd;
          W.xr = m + W.sd;
          W.phase = W_TWO_TOP;
        }
        break;
      // ---------------- one-sided: window [0, B] or [A, N] ----------------
      case W_ONE_TOP:
        W.A = W.one == 0 ? 0.0 : ceil(W.x);
        W.B = W.one == 0 ? floor(W.x) : N;
        W.m_ret = W_ONE_FX;
        W.phase = W_MASS_BEGIN;
        break;
      case W_ONE_FX:
        if (!have) {
          W.M = W.M * W.P.pm;  // mass() result (relative) -> absolute
          W.req_x = W.x;
          W.req_s = 0;
          return true;
        } else {
          have = false;
          const double fx = exp(W.res_g) * W.P.pm;
          const double Md = W.M;
          const double F = log(Md / (1.0 - Md)) - log(kMass / (1.0 - kMass));
          const double jac = W.one == 0 ? W.x + W.P.a : N - W.x + W.P.b;
          const double dF = fx * jac * (1.0 / Md + 1.0 / (1.0 - Md));
          double xn;
          if (W.one == 0) {
            if (F > 0.0) W.hb = W.x;
            else W.lb = W.x;
            xn = exp(log(W.x + W.P.a) - F / dF) - W.P.a;
          } else {
            if (F > 0.0) W.lb = W.x;
            else W.hb = W.x;
            xn = N + W.P.b - exp(log(N - W.x + W.P.b) - F / dF);
          }
          if (!(W.lb < xn && xn < W.hb)) xn = 0.5 * (W.lb + W.hb);
          if (fabs(xn - W.x) < fmax(kStop, 2e-5 * W.x) || W.it >= 40) {
            W.phase = W_FIX_A;
          } else {
            W.x = xn;
            W.it += 1;
            W.phase = W_ONE_TOP;
          }
        }
        break;
      // ---------------- two-sided: level-set Newton ------------------------
      case W_TWO_TOP:
        if (m == 0.0 || W.g0 >= W.t) {
          W.xl = 0.0;
          W.cl = 1;
          W.phase = W_TWO_ROOTR;
        } else {
          W.cl = 0;
          W.r_lo = 0.0;
          W.r_hi = m;
          W.r_x = fmin(fmax(W.xl, 0.0), m);
          W.r_rising = 1;
          W.r_it = 0;
          W.r_ret = W_TWO_ROOTR;
          W.phase = W_ROOT;
        }
        break;
      case W_TWO_ROOTR:
        if (!W.cl) W.xl = W.r_x;  // the left root (when it ran)
        if (m == N || W.gN >= W.t) {
          W.xr = N;
          W.cr = 1;
          W.phase = W_TWO_MASS;
        } else {
          W.cr = 0;
          W.r_lo = m;
          W.r_hi = N;
          W.r_x = fmin(fmax(W.xr, m), N);
          W.r_rising = 0;
          W.r_it = 0;
          W.r_ret = W_TWO_MASS;
          W.phase = W_ROOT;
        }
        break;
      case W_TWO_MASS:
        if (!W.cr) W.xr = W.r_x;
        W.A = ceil(W.xl);
        W.B = floor(W.xr);
        W.m_ret = W_TWO_SL;
        W.phase = W_MASS_BEGIN;
        break;
      case W_TWO_SL:
        if (!have) {
          W.M = W.M * W.P.pm;
          if (W.M >= kMass) W.tL = W.t;
          else W.tH = W.t;
          W.Dp = 0.0;
          W.mv = 0.0;
          if (!W.cl) { W.req_x = W.xl; W.req_s = 1; return true; }
        } else {
          have = false;
          const double sl = W.res_s;
          W.Dp += exp(W.t) / sl;
          W.mv += 1.0 / sl;
        }
        W.phase = W_TWO_SR;
        break;
      case W_TWO_SR:
        if (!have) {
          if (!W.cr) { W.req_x = W.xr; W.req_s = 1; return true; }
        } else {
          have = false;
          const double sr = -W.res_s;
          W.Dp += exp(W.t) / sr;
          W.mv += 1.0 / sr;
        }
        {
          W.Dp *= W.P.pm;
          bool stop = W.it >= 40;
          if (!stop) {
            double tn;
            if (W.Dp > 0.0) {
              const double dt = (log(W.M) - log(kMass)) * W.M / W.Dp;
              stop = fabs(dt) * W.mv < fmax(kStop, 2e-5 * W.A);
              tn = W.t + dt;
            } else {
              tn = 0.5 * (W.tL + W.tH);  // both ends clamped: raise the level
            }
            if (!stop) {
              if (!(W.tL < tn && tn < W.tH)) tn = W.tL > -INFINITY ? 0.5 * (W.tL + W.tH) : W.t - fmax(1.0, fabs(W.t));
              W.t = tn;
              W.it += 1;
            }
          }
          W.phase = stop ? W_FIX_A : W_TWO_TOP;
        }
        break;
      // ---------------- root sub-machine: g(x) = t on [r_lo, r_hi] ---------
      case W_ROOT:
        if (!have) {
          W.req_x = W.r_x;
          W.req_s = 1;
          return true;
        } else {
          have = false;
          const double gx = W.res_g - W.t;
          if (fabs(gx) < 1e-12) {
            W.phase = W.r_ret;
            break;
          }
          if ((gx < 0.0) == (W.r_rising != 0)) W.r_lo = W.r_x;
          else W.r_hi = W.r_x;
          const double sx = W.res_s;
          double xn = sx != 0.0 ? W.r_x - gx / sx : 0.5 * (W.r_lo + W.r_hi);
          if (!(W.r_lo < xn && xn < W.r_hi)) xn = 0.5 * (W.r_lo + W.r_hi);
          const bool conv = fabs(xn - W.r_x) < 0.05;
          W.r_x = xn;
          W.r_it += 1;
          if (conv || W.r_it >= 60) W.phase = W.r_ret;
        }
        break;
      // ---------------- mass sub-machine: sum_{A..B} p / p(m) ---------------
      case W_MASS_BEGIN:
        W.m_tot = 0.0;
        W.m_A1 = W.A;
        W.m_B1 = W.B;
        if (W.m_A1 < kK0) {
          W.m_e = fmin(kK0 - 1.0, W.B);
          W.ew_y = W.m_A1;
          W.ew_end = W.m_e;
          W.ew_ret = W_MASS_HR;
          W.m_mode = 1;  // A1 <- e + 1 on return
          W.phase = W_EXACT_WALK;
        } else {
          W.m_mode = 0;
          W.phase = W_MASS_HR;
        }
        break;
      case W_MASS_HR:
        if (W.m_mode == 1) {
          W.m_A1 = W.m_e + 1.0;
          W.m_mode = 0;
        }
        if (W.m_mode == 2) {  // back from the right head
          W.m_B1 = W.m_e - 1.0;
          W.m_mode = 0;
          W.phase = W_MASS_MID;
          break;
        }
        if (W.m_B1 > N - kK0 && W.m_B1 >= W.m_A1) {
          W.m_e = fmax(N - kK0 + 1.0, W.m_A1);
          W.ew_y = W.m_e;
          W.ew_end = W.m_B1;
          W.ew_ret = W_MASS_HR;
          W.m_mode = 2;
          W.phase = W_EXACT_WALK;
        } else {
          W.phase = W_MASS_MID;
        }
        break;
      case W_MASS_MID:
        if (W.m_mode == 3) {  // back from the short-window exact sum
          W.m_mode = 0;
          W.M = W.m_tot;
          W.phase = W.m_ret;
          break;
        }
        if (W.m_B1 < W.m_A1) {
          W.M = W.m_tot;
          W.phase = W.m_ret;
          break;
        }
        if (W.m_B1 - W.m_A1 < 32.0) {
          W.ew_y = W.m_A1;
          W.ew_end = W.m_B1;
          W.ew_ret = W_MASS_MID;
          W.m_mode = 3;
          W.phase = W_EXACT_WALK;
          break;
        }
        W.m_c = fmin(fmax(m, W.m_A1), W.m_B1);
        W.m_I = 0.0;
        W.p_part = 0;
        W.p_sub = 0;
        W.phase = part_setup(W) ? W_MASS_NODES : W_MASS_ENDA;
        break;
      case W_MASS_NODES: {
        double wj;
        if (!have) {
          W.req_x = node_x(W, wj);
          W.req_s = 0;
          return true;
        }
        have = false;
        (void)node_x(W, wj);
        W.m_I += wj * exp(W.res_g);
        if (++W.p_i == 6) {
          W.p_i = 0;
          if (++W.p_j == W.p_k) {
            ++W.p_sub;
            if (!part_setup(W)) W.phase = W_MASS_ENDA;
          }
        }
        break;
      }
      case W_MASS_ENDA:
        if (!have) {
          W.req_x = W.m_A1;
          W.req_s = 1;
          return true;
        }
        have = false;
        W.fA = exp(W.res_g);
        W.sA = W.res_s;
        W.phase = W_MASS_ENDB;
        break;
      case W_MASS_ENDB:
        if (!have) {
          W.req_x = W.m_B1;
          W.req_s = 1;
          return true;
        }
        have = false;
        {
          const double fB = exp(W.res_g), sB = W.res_s;
          W.M = W.m_tot + W.m_I + 0.5 * (W.fA + fB) + (fB * sB - W.fA * W.sA) * (1.0 / 12.0);
        }
        W.phase = W.m_ret;
        break;
      // ---------------- exact walk: m_tot += sum_{ew_y..ew_end} p/p(m) -------
      case W_EXACT_WALK:
        if (!have) {
          W.req_x = W.ew_y;
          W.req_s = 0;
          return true;
        }
        have = false;
        {
          double v = exp(W.res_g), s = 0.0;
          for (double y = W.ew_y; y <= W.ew_end; y += 1.0) {
            s += v;
            if (y < W.ew_end) v *= ratio(W.P, y);
          }
          W.m_tot += s;
        }
        W.phase = W.ew_ret;
        break;
      // ---------------- fix-up (oracle: hp_fixup) ----------------------------
      case W_FIX_A:
        if (!have) {
          W.req_x = W.A;
          W.req_s = 0;
          return true;
        }
        have = false;
        W.pA = exp(W.res_g) * W.P.pm;
        W.pB = W.pA;
        W.phase = W_FIX_B;
        break;
      case W_FIX_B:
        if (!have) {
          if (W.B != W.A) {
            W.req_x = W.B;
            W.req_s = 0;
            return true;
          }
        } else {
          have = false;
          W.pB = exp(W.res_g) * W.P.pm;
        }
        W.pl = W.A > 0.0 ? W.pA * rcp(ratio(W.P, W.A - 1.0)) : 0.0;
        W.pr = W.B < N ? W.pB * ratio(W.P, W.B) : 0.0;
        W.phase = W_FIX_WALK;
        break;
      case W_FIX_WALK: {
        double A = W.A, B = W.B, M = W.M, pA = W.pA, pB = W.pB, pl = W.pl, pr = W.pr;
        while (M < kMass && (pl > 0.0 || pr > 0.0)) {
          if (pl >= pr) {
            A -= 1.0;
            M += pl;
            pA = pl;
            pl = A > 0.0 ? pl * rcp(ratio(W.P, A - 1.0)) : 0.0;
          } else {
            B += 1.0;
            M += pr;
            pB = pr;
            pr = B < N ? pr * ratio(W.P, B) : 0.0;
          }
        }
        for (int g2 = 0; g2 < (1 << 24); ++g2) {
          const double pe = pB <= pA ? pB : pA;
          if (A < B && M - pe >= kMass) {
            if (pB <= pA) {
              M -= pB;
              pr = pB;
              B -= 1.0;
              pB = pB * rcp(ratio(W.P, B));
            } else {
              M -= pA;
              pl = pA;
              A += 1.0;
              pA = pA * ratio(W.P, A - 1.0);
            }
            continue;
          }
          const double pn = pl >= pr ? pl : pr;
          if (pn > pe) {
            if (pl >= pr) {
              A -= 1.0;
              M += pl;
              pA = pl;
              pl = A > 0.0 ? pl * rcp(ratio(W.P, A - 1.0)) : 0.0;
            } else {
              B += 1.0;
              M += pr;
              pB = pr;
              pr = B < N ? pr * ratio(W.P, B) : 0.0;
            }
            continue;
          }
          break;
        }
        W.A = A;
        W.B = B;
        W.phase = W_DONE;
        return false;
      }
      case W_DONE:
      default:
        return false;
    }
  }
  W.phase = W_DONE;  // (unreachable: a guard against a logic error looping)
  return false;
}

}  // namespace hpdi
}  // namespace mdfit
