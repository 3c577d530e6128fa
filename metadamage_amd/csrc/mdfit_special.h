// mdfit_special.h — FP64 lnGamma / digamma / trigamma for gfx950, fused.
//
// The fit needs, per beta-binomial point and per objective evaluation, the
// triple (lnGamma, psi, psi1) at six arguments (y+a, a, N-y+b, b, N+phi, phi).
// One call here returns all three from ONE log and ONE reciprocal of the
// (possibly shifted) argument (both hand-rolled below: the library log is a
// double-double routine ~3x longer, and the IEEE divide sequence is not
// needed where the result feeds a series):
//
//   x < 10:  shift by 10 with the product P(x) = prod_{j<10} (x+j) and its
//            first two derivatives (P'/P = sum 1/(x+j),
//            (P'/P)^2 - P''/P = sum 1/(x+j)^2), i.e. one more log and one
//            more reciprocal instead of ten of each;
//   x >= 10: Stirling / asymptotic series to O(x^-15).
//
// Accuracy (vs scipy, tests/test_special_*): |err| <= ~4e-15 * max(1, |f|).
#pragma once

#include <hip/hip_runtime.h>

namespace mdfit {

// FP64 reciprocal: v_rcp_f64 + two Newton steps (faithful, no IEEE div sequence).
// Measured on gfx950 (tools/micro/rcp_accuracy.hip, 2^28 log-uniform x):
// v_rcp_f64 alone is off by up to 2.1e8 ulp (~2^-25), one Newton step 10 ulp,
// two 0 (the correctly rounded 1/x).
__device__ __forceinline__ double rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  r = fma(fma(-x, r, 1.0), r, r);
  return r;
}
// One Newton step (<= 10 ulp): for reciprocals that only scale series
// corrections (lnGamma's Stirling terms, the shift sums of psi), where the
// relative error stays < 3e-15 of the function (lg3's fast form).
__device__ __forceinline__ double rcp1(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return fma(fma(-x, r, 1.0), r, r);
}

// Natural log, <= ~1 ulp (the classic reduction x = 2^e (1+f), 1+f in
// [sqrt(1/2), sqrt(2)), log(1+f) = f - hfsq + s (hfsq + R(s^2)), s = f/(2+f),
// R a degree-7 minimax polynomial in s^2 -- Cody & Waite / the fdlibm scheme).
// 0 -> -inf, +inf -> +inf, negative / NaN -> NaN.
__device__ __forceinline__ double flog(double x) {
#pragma clang fp contract(off)  // (every fusion explicit: the same bits in every inlined instance)
  constexpr double kLn2Hi = 6.93147180369123816490e-01;  // high 32 bits of ln 2
  constexpr double kLn2Lo = 1.90821492927058770002e-10;  // ln 2 - kLn2Hi
  constexpr double kSqrtHalf = 0.70710678118654752440;
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  int e = __builtin_amdgcn_frexp_exp(x);
  const bool lo = m < kSqrtHalf;
  m = lo ? m + m : m;
  e = lo ? e - 1 : e;
  const double f = m - 1.0;  // exact
  const double s = f * rcp(2.0 + f);
  const double z = s * s, w = z * z;
  const double t2 =
      z * fma(w, fma(w, fma(w, 1.479819860511658591e-01, 1.818357216161805012e-01),
                     2.857142874366239149e-01),
              6.666666666666735130e-01);
  const double R = fma(w, fma(w, fma(w, 1.531383769920937332e-01, 2.222219843214978396e-01),
                              3.999999999940941908e-01), t2);
  const double hfsq = 0.5 * f * f;
  const double de = (double)e;
  const double r = fma(de, kLn2Hi, -((hfsq - fma(s, hfsq + R, de * kLn2Lo)) - f));
  const bool normal = x > 0.0 && x < INFINITY;
  return normal ? r : (x == 0.0 ? -INFINITY : (x == INFINITY ? x : NAN));
}

#ifndef MDFIT_TLOG_NUTS
#define MDFIT_TLOG_NUTS 1  // the sampler's potential and WAIC: C3 chain + post ~7.0 -> 6.3 s (A/B)
#endif
}  // namespace mdfit
#include "mdfit_exptab.h"
#include "mdfit_logtab.h"
namespace mdfit {

// Natural log by table (the lnGamma family's logs: arguments >= 10, and the
// shift products), ~1 ulp for x away from 1: x = 2^e m, m in [1, 2), j = the
// top 8 mantissa bits, c_j = 1 + (2j+1)/512 the centre of its interval
// (mdfit_logtab.h: 1/c_j and ln c_j, one 16-B load); r = (m - c_j) / c_j with
// m - c_j exact and |r| <= 2^-9, ln(1 + r) by a degree-6 polynomial
// (truncation < 2^-66):  ln x = e ln2_hi + (ln c_j + (r + r^2 q(r) + e ln2_lo)).
// (ln c_j rounded to a double: <= 5.6e-17 absolute, a quarter ulp of ln x for
// x >= 10.)  ~20 VALU + one table load against flog's ~44 (its reciprocal,
// the degree-7 reduction, the special cases).  NOT for x near 1 where
// ln x ~ 0 (absolute, not relative, accuracy there): flog1p keeps flog.
// Inputs: finite and > 0 normal; kZero also 0 (-> -inf) and subnormals
// (pre-scaled) -- lnGamma's shift product, which is 0 at a = 0.
template <bool kZero = false>
__device__ __forceinline__ double flog_t(double x) {
#pragma clang fp contract(off)
  constexpr double kLn2Hi = 6.93147180369123816490e-01;
  constexpr double kLn2Lo = 1.90821492927058770002e-10;
  double xn = x;
  int eoff = 1023;
  if (kZero) {
    const bool sub = x < 2.2250738585072014e-308;
    xn = sub ? x * 0x1p60 : x;
    eoff = sub ? 1083 : 1023;
  }
  const uint32_t hw = (uint32_t)__double2hiint(xn);
  const int e = (int)(hw >> 20) - eoff;
  const int j = (int)((hw >> 12) & 255u);
  const double m = __hiloint2double((int)((hw & 0x000FFFFFu) | 0x3FF00000u), __double2loint(xn));
  const double2 t = *reinterpret_cast<const double2*>(&g_logtab[j][0]);  // (1/c, ln c)
  const double c = fma((double)(2 * j + 1), 1.0 / 512.0, 1.0);  // exact
  const double r = (m - c) * t.x;
  const double r2 = r * r;
  double q = fma(r, -1.0 / 6.0, 1.0 / 5.0);
  q = fma(r, q, -0.25);
  q = fma(r, q, 1.0 / 3.0);
  q = fma(r, q, -0.5);
  const double de = (double)e;
  // e ln2_hi is exact (ln2_hi has 21 trailing zero bits): one rounding at the
  // end, as fdlibm's, instead of two (~0.5 ulp typical instead of ~1)
  const double y = fma(de, kLn2Hi, t.y + (r + fma(r2, q, de * kLn2Lo)));
  return kZero ? (x > 0.0 ? y : -INFINITY) : y;
}

// log(1 + x), x > -1: Goldberg's correction log(u) * x / (u - 1), u = 1 + x.
__device__ __forceinline__ double flog1p(double x) {
#pragma clang fp contract(off)
  const double u = 1.0 + x;
  const double um1 = u - 1.0;
  return um1 == 0.0 ? x : flog(u) * (x * rcp(um1));
}

// exp(x), ~1 ulp: x = n ln2 + r (Cody-Waite, |r| <= ln2/2), e^r by a degree-12
// Taylor polynomial (|error| < 2e-17 on that range), 2^n by ldexp.  Saturates
// to 0 / +inf outside [-745, 709.8]; NaN passes through.
__device__ __forceinline__ double fexp(double x) {
  constexpr double kLog2e = 1.4426950408889634074;
  constexpr double kLn2Hi = 6.93147180369123816490e-01;
  constexpr double kLn2Lo = 1.90821492927058770002e-10;
  const double n = rint(x * kLog2e);
  const double r = fma(-n, kLn2Lo, fma(-n, kLn2Hi, x));
  double p = 1.0 / 479001600.0;
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  const double y = __builtin_amdgcn_ldexp(p, (int)fmax(fmin(n, 1100.0), -1100.0));
  return x < -745.2 ? 0.0 : (x > 709.8 ? INFINITY : y);
}

// exp(x) by table, ~1 ulp: x = (256 m + j) ln2 / 256 + r, |r| <= ln2 / 512,
// e^x = 2^m * 2^(j/256) * e^r with 2^(j/256) from mdfit_exptab.h (rounded
// binary64) and e^r = 1 + r + r^2 (1/2 + r (1/6 + r (1/24 + r / 120)))
// (truncation < 2^-66).  ln2_hi / 256 times the integer k is exact for |k| <
// 2^21.  ~20 VALU and one table load against the library exp's ~40.
// Saturates to 0 / +inf outside [-745.2, 709.78]; NaN passes through.
__device__ __forceinline__ double fexp_t(double x) {
#pragma clang fp contract(off)
  const double k = rint(x * 369.32986822047682);
  const int ki = (int)fmax(fmin(k, 262144.0), -262144.0);
  const double r = fma(-k, 1.90821492927058770002e-10 / 256.0,
                       fma(-k, 6.93147180369123816490e-01 / 256.0, x));
  double q = fma(r, 1.0 / 120.0, 1.0 / 24.0);
  q = fma(r, q, 1.0 / 6.0);
  q = fma(r, q, 0.5);
  const double p = fma(r * r, q, r);
  const double t = g_exptab[ki & 255];
  const double y = __builtin_amdgcn_ldexp(fma(t, p, t), ki >> 8);
  return x < -745.2 ? 0.0 : (x > 709.78 ? INFINITY : y);
}

struct LG3 {
  double l;  // lnGamma(x)
  double p;  // digamma(x)
  double q;  // trigamma(x)
};

// kTri = false: lnGamma and psi only (the sampler needs no Hessian).
// kTab: the fast form -- the logs by flog_t (the table) instead of flog, and
// the series' reciprocals (1/x of the Stirling terms, the shift sum's 1/P) by
// one Newton step (rcp1, <= 10 ulp: < 3e-15 of psi) -- for the sampler's
// potential and WAIC (MDFIT_TLOG_NUTS: C3 6.6 -> 6.1 s); the MAP fit, HPDI and
// record kernels keep the accurate form (the table log in the fit kernel was
// within +-1 % at C2 and 125k and spilled its PPL 2 layout: DESIGN.md §9).
template <bool kTri = true, bool kTab = false>
__device__ __forceinline__ LG3 lg3(double x) {
#pragma clang fp contract(off)  // (every fusion explicit: the same bits in every inlined instance)
  constexpr double kHalfLog2Pi = 0.91893853320467274178;  // 0.5 ln(2 pi)
  double P = 1.0, dP = 0.0, d2P = 0.0;
  double xs = x;
  const bool shift = x < 10.0;
  if (shift) {
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const double t = x + (double)j;
      if (kTri) d2P = fma(d2P, t, 2.0 * dP);
      dP = fma(dP, t, P);
      P = P * t;
    }
    xs = x + 10.0;
  }
  const double r = kTab ? rcp1(xs) : rcp(xs);
  const double r2 = r * r;
  const double lx = kTab ? flog_t(xs) : flog(xs);
  // lnGamma(xs) ~ (xs - 1/2) ln xs - xs + ln(2 pi)/2 + r (1/12 - r2 (1/360 - ...))
  double sl = fma(r2, -1.0 / 156.0, 691.0 / 360360.0);
  sl = fma(r2, -sl, 1.0 / 1188.0);
  sl = fma(r2, -sl, 1.0 / 1680.0);
  sl = fma(r2, -sl, 1.0 / 1260.0);
  sl = fma(r2, -sl, 1.0 / 360.0);
  sl = fma(r2, -sl, 1.0 / 12.0);
  double L = fma(r, sl, fma(xs - 0.5, lx, -xs) + kHalfLog2Pi);
  // psi(xs) ~ ln xs - r/2 - r2 (1/12 - r2 (1/120 - ...))
  double sp = fma(r2, -1.0 / 12.0, 691.0 / 32760.0);
  sp = fma(r2, -sp, 1.0 / 132.0);
  sp = fma(r2, -sp, 1.0 / 240.0);
  sp = fma(r2, -sp, 1.0 / 252.0);
  sp = fma(r2, -sp, 1.0 / 120.0);
  sp = fma(r2, -sp, 1.0 / 12.0);
  double Ps = fma(-r2, sp, fma(-0.5, r, lx));
  // psi1(xs) ~ r + r2/2 + r^3 (1/6 - r2 (1/30 - ...))
  double Q = 0.0;
  if (kTri) {
    double sq = fma(r2, -7.0 / 6.0, 691.0 / 2730.0);
    sq = fma(r2, -sq, 5.0 / 66.0);
    sq = fma(r2, -sq, 1.0 / 30.0);
    sq = fma(r2, -sq, 1.0 / 42.0);
    sq = fma(r2, -sq, 1.0 / 30.0);
    sq = fma(r2, -sq, 1.0 / 6.0);
    Q = fma(r * r2, sq, fma(0.5, r2, r));
  }
  if (shift) {
    const double iP = kTab ? rcp1(P) : rcp(P);
    const double s1 = dP * iP;          // sum 1/(x+j)
    L -= kTab ? flog_t<true>(P) : flog(P);
    Ps -= s1;
    if (kTri) Q += fma(s1, s1, -(d2P * iP));  // sum 1/(x+j)^2
  }
  return {L, Ps, Q};
}

// lnGamma alone (the unused psi is dead code after inlining)
__device__ __forceinline__ double lgam(double x) { return lg3<false>(x).l; }

// Stirling remainder lnGamma(z) - [(z - 1/2) ln z - z + ln(2 pi)/2], z >= 10
// (the series of lg3, O(z^-15))
__device__ __forceinline__ double stirling_rem(double z) {
#pragma clang fp contract(off)
  const double r = rcp(z), r2 = r * r;
  double sl = fma(r2, -1.0 / 156.0, 691.0 / 360360.0);
  sl = fma(r2, -sl, 1.0 / 1188.0);
  sl = fma(r2, -sl, 1.0 / 1680.0);
  sl = fma(r2, -sl, 1.0 / 1260.0);
  sl = fma(r2, -sl, 1.0 / 360.0);
  sl = fma(r2, -sl, 1.0 / 12.0);
  return r * sl;
}

// lnGamma(z + h) - lnGamma(z) for z, z + h > 0, without subtracting two large
// lnGamma values and without rounding the argument z + h (at z ~ 2e9 one ulp
// of it moves lnGamma by ~5e-6): in the Stirling range the leading terms are
// differenced analytically,
//   (z+h-1/2) ln(z+h) - (z+h) - (z-1/2) ln z + z = (z - 1/2 + h) log1p(h/z) + h (ln z - 1),
// so the rounding error scales with the difference, not with lnGamma ~ z ln z
// (one ulp of lnGamma(1e9) is ~4e-6); the remainders' difference is tiny.
// Below 10 the plain difference (small values, nothing to cancel).
__device__ __forceinline__ double lgdiff(double z, double h) {
#pragma clang fp contract(off)
  const double z1 = z + h;  // only for the branch test and the remainder
  if (z >= 10.0 && z1 >= 10.0) {
    const double t = flog1p(h * rcp(z));
    return fma(z - 0.5 + h, t, h * (flog(z) - 1.0)) + (stirling_rem(z1) - stirling_rem(z));
  }
  return lgam(z1) - lgam(z);
}

// ln[ Gamma(n+s) / (Gamma(n+1) Gamma(s)) ] = ln((s)_n / n!) for a count n >= 0
// and s > 0: the large lnGamma of the bigger of (n+1, s) is differenced
// against lnGamma(n+s) (lgdiff, with an exact step: s - 1 or the count n) and
// only the smaller one's lnGamma is subtracted, so the result carries
// rounding of the size of its own terms.
__device__ __forceinline__ double lrise(double n, double s) {
  if (n == 0.0) return 0.0;
  return s <= n + 1.0 ? lgdiff(n + 1.0, s - 1.0) - lgam(s) : lgdiff(s, n) - lgam(n + 1.0);
}

// Full beta-binomial log-pmf (numpyro BetaBinomial.log_prob with log C(N,y),
// fits.py:59,67,126-133) of one point at (D, phi):
//   log C(N,y) + lnB(y+a, N-y+b) - lnB(a, b) = R(y,a) + R(N-y,b) - R(N,phi),
// R = lrise, a = D phi, b = (1-D) phi.  Each R is O(s ln(n/s)), so the
// O(10)-sized result keeps ~1e-11 absolute accuracy even at N ~ 4e9, where the
// unnormalised form (a sum of lnGamma values ~1e11) would carry ~1e-5.
__device__ __forceinline__ double bb_logpmf_ab(double y, double N, double a, double b, double phi) {
  return (lrise(y, a) + lrise(N - y, b)) - lrise(N, phi);
}
__device__ __forceinline__ double bb_logpmf(double y, double N, double D, double phi) {
  return bb_logpmf_ab(y, N, D * phi, (1.0 - D) * phi, phi);
}

}  // namespace mdfit
