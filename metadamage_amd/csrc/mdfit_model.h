// mdfit_model.h — the per-point model, objective and Newton step shared by the
// fit kernels of mdfit.hip (MDFIT-MAP v1).
//
// model_PMD / model_null log densities of /root/reference/metadamage/fits.py:43-67
// (BetaBinomial log-pmf without the data-only log C(N,y)), their analytic
// gradient and Hessian in the unconstrained coordinates
// u = (logit q, logit A, c, log delta), and the projected, Hessian-modified
// Newton direction.  Same formulas as oracle/mdfit_oracle.c (written separately).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/mdfit.h"
#include "mdfit_special.h"

namespace mdfit {

constexpr int kNPos = MDFIT_NPOS;
constexpr int kNHalf = MDFIT_NHALF;
constexpr int kLD = MDFIT_LD;
constexpr int kNMM = MDFIT_NMM;

// u = (logit q, logit A, c, log delta): c on its own scale (see oracle).
constexpr double kULo[4] = {-25.0, -25.0, 0.0, -25.0};
constexpr double kUHi[4] = {25.0, 25.0, 0.999, 20.0};
constexpr double kEpsAct = 1e-8;
constexpr double kNoiseF = 1.4e-14;  // objective rounding scale (oracle: NOISE_F)
constexpr double kPgTol = 1e-6;      // exhausted line search + |proj. grad| below: converged (oracle: PG_TOL)
constexpr double kQuadK = 10.0;      // the quadratic-contraction stop of fit_kernel (oracle: QUAD_K)

// ---------------------------------------------------------------------------
// cross-lane sums inside aligned groups of G lanes (G = 2 ... 64)
// ---------------------------------------------------------------------------
// DPP move of a double (two 32-bit halves), all lanes active.
template <int Ctrl>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), Ctrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), Ctrl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// Every step pairs lanes by an involution (quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror, then xor 16 / xor 32) and adds two
// already-rounded values, so all G lanes end with bitwise-identical sums.  The
// leading empty asm makes `v` opaque: without it hipcc (fp-contract=fast)
// fuses the producer's multiply into the first add on THIS lane only
// (fma(a, b, partner) vs the partner's rounded a*b) and the lanes of one group
// drift apart in the last bit -- their Newton state machines then diverge.
template <int G>
__device__ __forceinline__ double gsum(double v) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "group size");
  asm volatile("" : "+v"(v));
  if (G >= 2) v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]  (xor 1)
  if (G >= 4) v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]  (xor 2)
  if (G >= 8) v += dpp<0x141>(v);  // row_half_mirror      (the other quad of the 8)
  if (G >= 16) v += dpp<0x140>(v); // row_mirror           (the other 8 of the row)
  if (G >= 32) v += __shfl_xor(v, 16, 64);
  if (G >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}

// opaque to the optimiser: a rounded value the compiler may not fuse into a
// later operation (keeps sums bitwise identical across lane layouts)
__device__ __forceinline__ double opaque(double v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ double clampd(double x, double lo, double hi) {
  return fmin(fmax(x, lo), hi);
}
__device__ __forceinline__ double logit(double p) { return flog(p) - flog1p(-p); }

// p = sigmoid(u), 1-p, ln p, ln(1-p) from one exp and one log1p
__device__ __forceinline__ void logit_parts(double u, double& p, double& omp, double& lp,
                                            double& l1mp) {
  const double e = exp(-fabs(u));
  const double r = rcp(1.0 + e);
  const double sp = flog1p(e);
  const bool pos = u >= 0.0;
  p = pos ? r : e * r;
  omp = pos ? e * r : r;
  lp = pos ? -sp : u - sp;
  l1mp = pos ? -(u + sp) : -sp;
}

// The value of the lane 16 away (lane ^ 16): rows 0 <-> 1 and 2 <-> 3 of the
// wave exchange, by v_permlane16_swap (gfx950; one swap per dword: with the
// same register as both operands, the even rows' copy ends up in the odd rows
// of the first result and the odd rows' in the even rows of the second).
__device__ __forceinline__ double xrow(double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const auto rl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto rh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const bool odd = (threadIdx.x & 16) != 0;
  return __hiloint2double((int)(odd ? rh[0] : rh[1]), (int)(odd ? rl[0] : rl[1]));
}

// Broadcast lane N of every 16-lane DPP row to the whole row (row_newbcast).
template <int N>
__device__ __forceinline__ double rowb(double v) {
  return dpp<0x150 + N>(v);
}

// Constrained parameters of one trial point u, computed once per trial
// instead of once per point evaluation; kept lean (registers).
struct Theta {
  double q, omq, iomq;  // q, 1-q, 1/(1-q)
  double A, JA;         // A and A(1-A) (PMD only)
  double c, iomc;       // c and 1/(1-c) (PMD only; c on its own scale)
  double delta, phi;
  double lprior;        // log prior at u (constants dropped)
};

// Row-collective: every lane of a W-lane row (W = 16: a DPP row; W = 8: one
// half of a DPP row) must be active and hold the same u and model (a row
// never spans two sub-fits).  The transcendental pieces are spread over the
// row -- lane 0: sigmoid / log-sigmoids of u0, lane 1: of u1, lane 2: exp(u3)
// and ln(1-c) -- one exp, one log1p and one reciprocal per lane instead of
// three of each, then broadcast (W = 8: from lane 0..2 or 8..10 of the DPP
// row, by half).  The result does not depend on W.
template <int W = 16>
__device__ __forceinline__ Theta make_theta(bool pmd, const double u[4]) {
  static_assert(W == 16 || W == 8, "row width");
  const int i = (int)(threadIdx.x & (W - 1));
  const bool hi8 = W == 8 && (threadIdx.x & 8);
  const double v = i == 0 ? u[0] : u[1];  // the logit this lane resolves (lanes 0, 1)
  const double e = exp(i < 2 ? -fabs(v) : u[3]);
  const double sp = flog1p(i < 2 ? e : -u[2]);  // ln(1 + e^-|v|), or ln(1-c) on lane 2
  const double rr = rcp(1.0 + e);
  const bool pos = v >= 0.0;
  const double p = pos ? rr : e * rr, omp = pos ? e * rr : rr;
  // ln p + 2 ln(1-p)  (fits.py:46-48: Beta(2, 3) prior up to a constant)
  const double lpp = (pos ? -sp : v - sp) + 2.0 * (pos ? -(v + sp) : -sp);
  auto bc = [=](double x, auto n) {
    constexpr int N = decltype(n)::value;
    if constexpr (W == 16) return rowb<N>(x);
    else return hi8 ? rowb<8 + N>(x) : rowb<N>(x);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  Theta th;
  th.q = bc(p, I0{});
  th.omq = bc(omp, I0{});
  const double lpq = bc(lpp, I0{});
  const double A = bc(p, I1{}), omA = bc(omp, I1{}), lpA = bc(lpp, I1{});
  th.delta = bc(e, I2{});
  const double l1mc = bc(sp, I2{});
  th.iomq = rcp(th.omq);
  th.phi = th.delta + 2.0;
  // ln q + 2 ln(1-q) - delta/1000  [+ ln A + 2 ln(1-A) + 8 ln(1-c)]  (fits.py:46-53)
  th.lprior = lpq - th.delta / 1000.0;
  if (pmd) {
    th.A = A;
    th.JA = A * omA;
    th.c = u[2];
    th.iomc = rcp(1.0 - th.c);
    th.lprior += lpA + 8.0 * l1mc;
  } else {
    th.A = th.JA = th.c = 0.0;
    th.iomc = 1.0;
  }
  return th;
}

// theta-space sums of one objective evaluation (before the chain rule):
// 0 ell, 1 mag, 2..5 G(q,A,c,phi), 6..15 H upper triangle
// (qq qA qc qphi AA Ac Aphi cc cphi phiphi)
constexpr int kNAcc = 16;

// x^k for 0 <= k < 16 by binary powering (3 squarings, 3 products): cheaper
// than exp(k ln x) and as accurate (a few rounding errors).
__device__ __forceinline__ double powk(double x, int k) {
  const double x2 = x * x, x4 = x2 * x2, x8 = x4 * x4;
  const double a = (k & 1) ? x : 1.0, b = (k & 2) ? x2 : 1.0;
  const double c = (k & 4) ? x4 : 1.0, d = (k & 8) ? x8 : 1.0;
  return (a * b) * (c * d);
}

// Per-lane point data of the current phase.
struct PointData {
  double y, N;
  int k;      // |z| - 1
  int valid;  // a real point (not a pad lane); ints, not bools: see fit_kernel
  int pmd;    // lane group fits model_PMD (else model_null)
};

// A point's D(z) and its derivatives at theta, and the beta-binomial
// parameters a = D phi, b = (1 - D) phi.
struct PointArgs {
  double D, Dq, DA, Dc, Dqq, DqA, omD, a, b;
};
__device__ __forceinline__ PointArgs point_args(const PointData& pd, const Theta& th) {
#pragma clang fp contract(off)  // (every fusion explicit: the same bits in both lane layouts)
  PointArgs r;
  if (pd.pmd) {
    const double kk = (double)pd.k;
    const double w = powk(th.omq, pd.k);  // (1-q)^k
    const double wq = w * th.iomq;        // (1-q)^(k-1)
    r.D = fma(th.A, w, th.c);
    r.DA = w;
    r.Dc = 1.0;
    r.Dq = pd.k >= 1 ? -th.A * kk * wq : 0.0;
    r.DqA = pd.k >= 1 ? -kk * wq : 0.0;
    r.Dqq = pd.k >= 2 ? th.A * kk * (kk - 1.0) * (wq * th.iomq) : 0.0;
  } else {
    r.D = th.q;
    r.Dq = 1.0;
    r.DA = r.Dc = r.Dqq = r.DqA = 0.0;
  }
  r.omD = 1.0 - r.D;
  r.a = r.D * th.phi;
  r.b = r.omD * th.phi;
  return r;
}

// One point's contribution at theta, ADDED to acc (same formulas as
// oracle/mdfit_oracle.c evaluate(); derivation in DESIGN.md §3), from the
// (lnGamma, psi, psi1) triples t1..t6 at y+a, N-y+b, N+phi, a, b, phi.
// Returns the point's log-likelihood (without log C(N,y)).
//
// accf (the polish phase of the fit, oracle: evaluate(accf = 1)): the value
// term is instead the full log-pmf in the cancellation-free form bb_logpmf_ab
// (the objective shifts by the constant sum log C(N,y)), and the rounding scale
// acc[1] the sum of its three |R| terms: F then resolves ~1e-10 instead of the
// ~1e-6 of a sum of ~N ln N-sized lnGamma values.  Gradient and Hessian terms
// are the same in both forms.
__device__ __forceinline__ double point_finish(const PointData& pd, const Theta& th, const PointArgs& pa,
                                              const LG3& t1, const LG3& t2, const LG3& t3, const LG3& t4,
                                              const LG3& t5, const LG3& t6, double acc[kNAcc], int accf = 0) {
#pragma clang fp contract(off)  // (every fusion explicit: the same bits in both lane layouts)
  const double D = pa.D, omD = pa.omD, a = pa.a, b = pa.b;
  const double phi = th.phi;
  const double la = t1.l - t4.l, Pa = t1.p - t4.p, Qa = t1.q - t4.q;
  double mag = fabs(t1.l) + fabs(t4.l);
  const double lb = t2.l - t5.l, Pb = t2.p - t5.p, Qb = t2.q - t5.q;
  mag += fabs(t2.l) + fabs(t5.l);
  const double lS = t3.l - t6.l, S = t6.p - t3.p, S1 = t6.q - t3.q;
  mag += fabs(t3.l) + fabs(t6.l);
  double ell = (la + lb) - lS;  // exact 0 when N = 0
  if (accf) {
    const double r1 = lrise(pd.y, a), r2 = lrise(pd.N - pd.y, b), r3 = lrise(pd.N, phi);
    ell = (r1 + r2) - r3;
    mag = (fabs(r1) + fabs(r2)) + fabs(r3);
  }
  const double Dq = pa.Dq, DA = pa.DA, Dc = pa.Dc, Dqq = pa.Dqq, DqA = pa.DqA;
  const double lD = phi * (Pa - Pb);
  const double lF = fma(D, Pa, fma(omD, Pb, S));
  const double lDD = (phi * phi) * (Qa + Qb);
  const double lDF = fma(phi, fma(D, Qa, -(omD * Qb)), Pa - Pb);
  const double lFF = fma(D * D, Qa, fma(omD * omD, Qb, S1));
  if (pd.valid) {
    const double lDDq = lDD * Dq, lDDA = lDD * DA;
    acc[0] += ell;
    acc[1] += mag;
    acc[2] = fma(lD, Dq, acc[2]);
    acc[3] = fma(lD, DA, acc[3]);
    acc[4] = fma(lD, Dc, acc[4]);
    acc[5] += lF;
    acc[6] = fma(lDDq, Dq, fma(lD, Dqq, acc[6]));
    acc[7] = fma(lDDq, DA, fma(lD, DqA, acc[7]));
    acc[8] = fma(lDDq, Dc, acc[8]);
    acc[9] = fma(lDF, Dq, acc[9]);
    acc[10] = fma(lDDA, DA, acc[10]);
    acc[11] = fma(lDDA, Dc, acc[11]);
    acc[12] = fma(lDF, DA, acc[12]);
    acc[13] = fma(lDD * Dc, Dc, acc[13]);
    acc[14] = fma(lDF, Dc, acc[14]);
    acc[15] += lFF;
  }
  return ell;
}

// a triple broadcast from lane N of every 16-lane DPP row
template <int N>
__device__ __forceinline__ LG3 rowb3(const LG3& t) {
  return {rowb<N>(t.l), rowb<N>(t.p), rowb<N>(t.q)};
}

// One point's contribution (point_finish): its lnGamma triples computed here.
//
// kRowPhi: the (lnGamma, psi, psi1) triple at phi is taken from lane 15 of
// the 16-lane row -- a pad lane (N = 0) whose lg3(N + phi) IS lg3(phi),
// bitwise -- so a point costs 5 lg3 instead of 6 (row-collective then: all
// lanes active, lane 15 of every row a pad holding the row's phi).
// null_row (wave-uniform; kRowPhi only): every row fits model_null, where a =
// q phi and b = (1-q) phi are the same at every point of the row, and the pad
// lane's lg3(y + a), lg3(N - y + b) ARE lg3(a), lg3(b), bitwise: broadcast
// from it, 3 lg3 per point instead of 5.
// whole_pair (wave-uniform; kRowPhi only): every 32-lane slot holds one
// all-position fit, rows z > 0 and z < 0 at the same |z| lane by lane, so a
// lane and its partner 16 away have the same a and b: the even row computes
// lg3(a), the odd row lg3(b), and they exchange (xrow): 4 lg3 instead of 5.
template <bool kRowPhi = false>
__device__ __forceinline__ double point_accum(const PointData& pd, const Theta& th, double acc[kNAcc],
                                              int accf = 0, bool null_row = false, bool whole_pair = false) {
  const PointArgs pa = point_args(pd, th);
  const LG3 t3 = lg3<true>(pd.N + th.phi);
  const LG3 t6 = kRowPhi ? rowb3<15>(t3) : lg3<true>(th.phi);
  const LG3 t1 = lg3<true>(pd.y + pa.a);
  const LG3 t2 = lg3<true>(pd.N - pd.y + pa.b);
  LG3 t4, t5;
  if (kRowPhi && null_row) {
    t4 = rowb3<15>(t1);
    t5 = rowb3<15>(t2);
  } else if (kRowPhi && whole_pair) {
    const bool odd = (threadIdx.x & 16) != 0;
    const LG3 mine = lg3<true>(odd ? pa.b : pa.a);
    const LG3 other = {xrow(mine.l), xrow(mine.p), xrow(mine.q)};
    t4 = odd ? other : mine;
    t5 = odd ? mine : other;
  } else {
    t4 = lg3<true>(pa.a);
    t5 = lg3<true>(pa.b);
  }
  return point_finish(pd, th, pa, t1, t2, t3, t4, t5, t6, acc, accf);
}

// Pointwise log-likelihood of one point at a mode for the record assembly
// (waic_i = -2 ell_i, fits.py:126-172): the full log-pmf including log C(N,y)
// -- what numpyro's log_likelihood returns -- in the cancellation-free form
// bb_logpmf.  (The fit objective drops the data-only log C(N,y); it cancels in
// n_sigma / asymmetry, but without it ell_i is ~ -N H(y/N) ~ 1e8 and a 1-ulp
// lnGamma difference becomes ~1e-4 of a small WAIC-difference statistic.)
__device__ __forceinline__ double point_ell(double y, double N, double D, double phi) {
  return bb_logpmf(y, N, D, phi);
}

// Objective in u-space from the group sums (oracle: evaluate(), chain rule
// part).  H is the packed upper triangle in acc order: qq qA qc qphi AA Ac
// Aphi cc cphi phiphi.
struct Eval {
  double F, mag;
  double g[4];
  double H[10];
};

__device__ __forceinline__ int hidx(int j, int m) {  // packed index, j <= m
  return j == 0 ? m : (j == 1 ? 3 + m : (j == 2 ? 5 + m : 9));
}

__device__ __forceinline__ void finish_eval(bool pmd, const Theta& th, const double s[kNAcc],
                                            Eval& e) {
  const double q = th.q, A = th.A, c = th.c, delta = th.delta;
  const double J[4] = {q * th.omq, th.JA, 1.0, delta};
  const double J2[4] = {J[0] * (1.0 - 2.0 * q), th.JA * (1.0 - 2.0 * A), 0.0, delta};
  const double gp[4] = {1.0 - 3.0 * q, pmd ? 1.0 - 3.0 * A : 0.0, pmd ? -8.0 * th.iomc : 0.0,
                        -delta / 1000.0};
  const double hp[4] = {-3.0 * J[0], pmd ? -3.0 * th.JA : 0.0,
                        pmd ? -8.0 * th.iomc * th.iomc : 0.0, -delta / 1000.0};
  const bool infeasible = pmd && (A + c >= 1.0);
  e.F = infeasible ? INFINITY : -(s[0] + th.lprior);
  e.mag = s[1];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool fixed = !pmd && (j == 1 || j == 2);
    e.g[j] = fixed ? 0.0 : -(J[j] * s[2 + j] + gp[j]);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int m = j; m < 4; ++m) {
      const int k = hidx(j, m);
      double h = J[j] * s[6 + k] * J[m];
      if (j == m) h += J2[j] * s[2 + j] + hp[j];
      const bool fixed = !pmd && (j == 1 || j == 2 || m == 1 || m == 2);
      e.H[k] = fixed ? 0.0 : -h;
    }
  }
}

__device__ __forceinline__ double maxabs4(const double v[4]) {
  return fmax(fmax(fabs(v[0]), fabs(v[1])), fmax(fabs(v[2]), fabs(v[3])));
}

// projected-gradient size (oracle: pgnorm): 0 for a variable held on its bound
__device__ __forceinline__ double pgnorm(const double u[4], const double g[4]) {
  double m = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) m = fmax(m, fabs(u[j] - clampd(u[j] - g[j], kULo[j], kUHi[j])));
  return m;
}

// the projected-gradient direction P(u - g) - u scaled to max-norm 1 (the
// gradient fallback of fit_kernel; oracle: pg_direction); false when it vanishes
__device__ __forceinline__ bool pg_direction(const double u[4], const double g[4], double d[4]) {
  double p[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) p[j] = clampd(u[j] - g[j], kULo[j], kUHi[j]) - u[j];
  const double mx = maxabs4(p);
  if (!(mx > 0.0)) return false;
#pragma unroll
  for (int j = 0; j < 4; ++j) d[j] = p[j] / mx;
  return true;
}

constexpr double kEpsBind[4] = {1e-3, 1e-3, 1e-4, 1e-3};

// 1/sqrt(x), x > 0: v_rsq_f64 + two Newton steps (no IEEE sqrt sequence)
__device__ __forceinline__ double rsqrt_nr(double x) {
  double r = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  r = r * fma(-hx * r, r, 1.5);
  r = r * fma(-hx * r, r, 1.5);
  return r;
}

// Cholesky of the free block of H + mu*I (fixed / bound rows -> identity);
// returns the first non-positive pivot's index (-1: positive definite).
// Packed lower triangle L (same index as H), iL = 1 / diag(L).
__device__ __forceinline__ int chol4(const bool fr[4], const double H[10], double mu, double L[10],
                                     double iL[4]) {
  int jf = -1;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int m = 0; m <= j; ++m) {
      double s;
      if (!fr[j] || !fr[m]) s = (j == m) ? 1.0 : 0.0;
      else s = H[hidx(m, j)] + ((j == m) ? mu : 0.0);
#pragma unroll
      for (int p = 0; p < m; ++p) s = fma(-L[hidx(p, j)], L[hidx(p, m)], s);  // explicit: the same rounding in every instance
      if (j == m) {
        if (!(s > 0.0) && jf < 0) jf = j;
        const double sp = fmax(s, 1e-300);
        const double il = rsqrt_nr(sp);  // 1/L_jj, then L_jj = s/L_jj
        L[hidx(j, j)] = sp * il;
        iL[j] = il;
      } else {
        L[hidx(m, j)] = s * iL[m];  // L(j,m) stored at packed (m,j)
      }
    }
  }
  return jf;
}

// Projected, Hessian-modified Newton direction with a Bertsekas binding set
// (oracle: direction()): variables within eps of a bound and pushed outward
// step onto the bound and leave the Newton system.
// w = pgnorm(u, g) (the fixed coordinates of model_null have g = 0 and sit
// inside the box, so they add nothing to it).
__device__ __forceinline__ void free_set(bool pmd, const double u[4], const double g[4], const double H[10],
                                         double w, bool fr[4], double dbind[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool fixed = !pmd && (j == 1 || j == 2);
    const double eps = fmin(kEpsBind[j], w);
    const double dlo = u[j] - kULo[j], dhi = kUHi[j] - u[j];
    const bool atlo = dlo <= eps, athi = dhi <= eps;
    // on / next to a box bound and not pulled inward by more than kEpsAct --
    // unless, with positive curvature, its own Newton step g/H stops short of
    // the bound (an interior optimum just inside it)
    const double hjj = H[hidx(j, j)];
    const bool bind = (atlo && g[j] > -kEpsAct && (hjj <= 0.0 || g[j] + kEpsAct > hjj * dlo)) ||
                      (athi && g[j] < kEpsAct && (hjj <= 0.0 || -g[j] + kEpsAct > hjj * dhi));
    dbind[j] = (bind && !fixed) ? (atlo ? kULo[j] : kUHi[j]) - u[j] : 0.0;
    fr[j] = !(fixed || bind);
  }
}

// Returns true when the free block of H is indefinite (the Cholesky needed a
// shift): the saddle escape's trigger (oracle: direction()).  With want_nc and
// an indefinite H, d is instead a direction of non-positive curvature (the
// saddle escape; oracle: nc_direction): the unshifted Cholesky's first
// non-positive pivot s_j with the rows above it gives z = (-L^-T l, 1, 0..),
// z'Hz = s_j <= 0, scaled to max-norm 1 and signed downhill.
//
// G: the lanes that hold this fit's (replicated) state -- an aligned group.
// An indefinite H is shifted by mu_a = 1e-10 scale x 10^(a-1) for the first a
// = 1, 2, ... whose Cholesky succeeds (oracle: direction(), the same mu by the
// same repeated products); the group's lanes try attempts 1..G at once, lane k
// attempt k+1 (one Cholesky's latency instead of up to G in a row), and take
// the step from the lane of the first success; past G the rest of the
// sequence runs replicated, as before (rare: ~1 % of shifted systems at G = 8).
template <int G>
__device__ __forceinline__ bool newton_dir(bool pmd, const double u[4], const double g[4],
                                           const double H[10], double w, double d[4], bool want_nc = false) {
  bool fr[4];
  double dbind[4];
  free_set(pmd, u, g, H, w, fr, dbind);
  double L[10], iL[4];
  const int jf = chol4(fr, H, 0.0, L, iL);  // plain Newton: the common case
  const bool indef = jf >= 0;
  if (want_nc && indef) {
    double z[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) z[j] = j == jf ? 1.0 : 0.0;
#pragma unroll
    for (int p = 2; p >= 0; --p) {
      if (p < jf) {
        double s = 0.0;
#pragma unroll
        for (int k = p + 1; k < 4; ++k) s += k <= jf ? L[hidx(p, k)] * z[k] : 0.0;  // L(k,p)
        z[p] = -s * iL[p];
      }
    }
    const double mx = maxabs4(z);
    const double gz = g[0] * z[0] + g[1] * z[1] + g[2] * z[2] + g[3] * z[3];
    const double sg = gz > 0.0 ? -1.0 : 1.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = sg * z[j] / mx;
    return true;
  }
  bool ok = !indef;
  // the solve with the accepted factor: every lane of a group that needed a
  // shift solves with its own attempt's factor, then takes the winner's step
  int src = -1;  // >= 0: the lane (absolute) whose step this lane takes
  if (__any(!ok)) {
    double sc = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (fr[j]) sc = fmax(sc, fabs(H[hidx(j, j)]));
    if (sc == 0.0) sc = 1.0;
    const int kl = (int)(threadIdx.x & (G - 1));
    const int gbase = (int)(threadIdx.x & ~(G - 1));
    double mu = 1e-10 * sc;
#pragma unroll
    for (int i = 1; i < G; ++i) mu = i <= kl ? mu * 10.0 : mu;  // attempt kl + 1
    double L2[10], iL2[4];
    // (mu opaque: a product the compiler may not fuse into the Cholesky's
    // diagonal add -- it would round differently in the parallel and the
    // sequential instance, and the two layouts reach them at different attempts)
    const bool ok2 = !ok && chol4(fr, H, opaque(mu), L2, iL2) < 0;
    const unsigned long long gm = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << gbase;
    const unsigned long long okm = __ballot(ok2) & gm;
    if (!ok) {
      if (okm != 0ull) {
        ok = true;
        src = __ffsll(okm) - 1;
#pragma unroll
        for (int j = 0; j < 10; ++j) L[j] = L2[j];
#pragma unroll
        for (int j = 0; j < 4; ++j) iL[j] = iL2[j];
      } else {  // attempts G+1 .. 39, replicated on the group's lanes
        mu = 1e-10 * sc;
#pragma unroll 1
        for (int i = 1; i < G; ++i) mu *= 10.0;  // attempt G
        mu *= 10.0;
        for (int attempt = G + 1; attempt < 40 && !ok; ++attempt, mu *= 10.0) ok = chol4(fr, H, opaque(mu), L, iL) < 0;
      }
    }
  }
  if (!ok) {
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = (fr[j] && isfinite(g[j])) ? -g[j] : 0.0;
  } else {
    double z[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // L z = -g (free rows)
      double s = fr[j] ? -g[j] : 0.0;
#pragma unroll
      for (int p = 0; p < j; ++p) s = fma(-L[hidx(p, j)], z[p], s);
      z[j] = s * iL[j];
    }
#pragma unroll
    for (int j = 3; j >= 0; --j) {  // L^T d = z
      double s = z[j];
#pragma unroll
      for (int p = j + 1; p < 4; ++p) s = fma(-L[hidx(j, p)], d[p], s);
      d[j] = s * iL[j];
    }
  }
  if (__any(src >= 0)) {
    const int from = src >= 0 ? src : (int)threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = __shfl(d[j], from, 64);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (!fr[j]) d[j] = dbind[j];
  const double mx = maxabs4(d);
  if (mx > 4.0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] *= 4.0 / mx;
  }
  return indef;
}


// ---------------------------------------------------------------------------
// record pieces shared by the MAP and sampling assembly kernels (one wave per
// taxon, counts staged in LDS)
// ---------------------------------------------------------------------------
// sums (fits.py:272-283) into the record s_rec.  Wave-collective.
__device__ __forceinline__ void record_sums(int lane, const double* s_y, const double* s_N, double* s_rec) {
  {
    const double v = lane < kNPos ? 1.0 : 0.0;
    const double fw = lane < kNHalf ? 1.0 : 0.0;
    const int pi = lane < kNPos ? lane : 0;
    const double yv = v * s_y[pi], nv = v * s_N[pi];
    const double nf = gsum<64>(fw * nv), nt = gsum<64>(nv);
    const double yf = gsum<64>(fw * yv), yt = gsum<64>(yv);
    if (lane == 0) {
      s_rec[MDFIT_F_N_Z1_FORWARD] = s_N[0];
      s_rec[MDFIT_F_N_Z1_REVERSE] = s_N[kNHalf];
      s_rec[MDFIT_F_N_SUM_FORWARD] = nf;
      s_rec[MDFIT_F_N_SUM_REVERSE] = nt - nf;
      s_rec[MDFIT_F_N_SUM_TOTAL] = nt;
      s_rec[MDFIT_F_Y_SUM_FORWARD] = yf;
      s_rec[MDFIT_F_Y_SUM_REVERSE] = yt - yf;
      s_rec[MDFIT_F_Y_SUM_TOTAL] = yt;
    }
  }
}

// noise (fits.py:359-376) of the mismatch counts s_mm[30][12] into the record
// s_rec (NaN without them); s_tmp: 64 doubles of LDS scratch.  Wave-collective
// (one 64-lane block).
__device__ __forceinline__ void record_noise(int lane, const uint32_t* s_mm, bool has_mm, double* s_rec,
                                             double* s_tmp) {
  {
    // mismatch column j = lane % 12 (AC AG AT CA CG CT GA GC GT TA TC TG), rows
    // i = lane / 12 + 5k (k < 6) on lanes 0..59: 6 rows per lane instead of 30
    // (shorter dependency chains); CT is NaN on rows 0..14, GA on rows 15..29.
    constexpr int kG = 5, kRows = kNPos / kG;
    const int j = lane % kNMM, g = lane / kNMM;
    const bool own = lane < kNMM * kG && has_mm;
    const int gi = own ? g : 0;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int i = gi + kG * k;
      const bool nanned = (j == 5 && i < kNHalf) || (j == 6 && i >= kNHalf);
      if (!nanned) s += (double)s_mm[i * kNMM + j];
    }
    // column sums (exact: integer-valued doubles) through LDS
    s_tmp[lane] = own ? s : 0.0;
    __syncthreads();
    double sc = 0.0;
#pragma unroll
    for (int gg = 0; gg < kG; ++gg) sc += s_tmp[j + kNMM * gg];
    __syncthreads();
    const double m = sc / ((j == 5 || j == 6) ? (double)kNHalf : (double)kNPos);  // nanmean
    double sa[3] = {0, 0, 0}, ca[3] = {0, 0, 0};
    double xs[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int i = gi + kG * k;
      const bool nanned = (j == 5 && i < kNHalf) || (j == 6 && i >= kNHalf);
      const double x = (double)s_mm[i * kNMM + j] / m;
      const bool use = own && !nanned && !isnan(x);
      xs[k] = use ? x : NAN;
      if (use) {
        const int h = i < kNHalf ? 1 : 2;
        sa[0] += x;
        ca[0] += 1.0;
        sa[h] += x;
        ca[h] += 1.0;
      }
    }
    double mean[3], cq[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      cq[q] = gsum<64>(ca[q]);
      mean[q] = gsum<64>(sa[q]) / cq[q];
    }
    double ss[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int i = gi + kG * k;
      const double x = xs[k];
      if (!isnan(x)) {
        const int h = i < kNHalf ? 1 : 2;
        ss[0] += (x - mean[0]) * (x - mean[0]);
        ss[h] += (x - mean[h]) * (x - mean[h]);
      }
    }
    double nz[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) nz[q] = cq[q] > 0.0 ? sqrt(gsum<64>(ss[q]) / cq[q]) : NAN;
    if (lane == 0) {
      const bool have = has_mm;
      s_rec[MDFIT_F_NORMALIZED_NOISE] = have ? nz[0] : NAN;
      s_rec[MDFIT_F_NORMALIZED_NOISE_FORWARD] = have ? nz[1] : NAN;
      s_rec[MDFIT_F_NORMALIZED_NOISE_REVERSE] = have ? nz[2] : NAN;
    }
  }
}

__device__ __forceinline__ void record_sums_noise(int lane, const double* s_y, const double* s_N,
                                                  const uint32_t* s_mm, bool has_mm, double* s_rec,
                                                  double* s_tmp) {
  record_sums(lane, s_y, s_N, s_rec);
  record_noise(lane, s_mm, has_mm, s_rec, s_tmp);
}

}  // namespace mdfit
