// mdfit.hip — MI355X (gfx950) batched per-TaxID damage fit + C-ABI (include/mdfit.h).
//
// Replaces the per-taxon NUTS loop of /root/reference/metadamage/fits.py
// (compute_fits :709-730 -> fit_single_group_without_timeout :428-469) with one
// stream-ordered launch over a dense count tensor.  Inference mode:
// MDFIT-MAP v1 — the mode of model_PMD / model_null
// (fits.py:43-67) found by projected, Hessian-modified Newton in unconstrained
// coordinates, followed by the record assembly of compute_fit_results
// (fits.py:230-295), add_assymetry_results_to_fit_results (:298-356) and
// add_noise_estimates (:359-376).
//
// Work decomposition: ONE WAVEFRONT PER TAXON (64-thread workgroups, so the
// hardware dispatcher load-balances taxa whose Newton iteration counts differ).
//   phase A: lanes 0-31  = model_PMD on all 30 points  (lane = point, 30,31 pad)
//            lanes 32-63 = model_null on all 30 points
//   phase B: lanes 0-15  = PMD on forward  z=1..15     (fits.py:311-312)
//            lanes 16-31 = PMD on reverse  z=-1..-15   (fits.py:333-334)
//            lanes 32-47 = null on forward, lanes 48-63 = null on reverse
// Each lane group runs its own Newton state machine in lock-step with the
// others (a wave-uniform loop, per-group "done" masks); the per-point
// log-likelihood, gradient and Hessian contributions are summed over the group
// with cross-lane butterflies.  Counts are staged in LDS once per taxon.
// Everything is FP64 (the reference enables x64, fits.py:32).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/mdfit.h"
#include "mdfit_special.h"

namespace mdfit {

constexpr int kNPos = MDFIT_NPOS;
constexpr int kNHalf = MDFIT_NHALF;
constexpr int kLD = MDFIT_LD;
constexpr int kNMM = MDFIT_NMM;
constexpr double kZ68 = 0.994457883209753;  // Phi^-1(0.84)

// u = (logit q, logit A, c, log delta): c on its own scale (see oracle).
__constant__ double kULo[4] = {-25.0, -25.0, 0.0, -25.0};
__constant__ double kUHi[4] = {25.0, 25.0, 0.999, 20.0};
constexpr double kEpsAct = 1e-8;
constexpr double kNoiseF = 1.4e-14;  // objective rounding scale (oracle: NOISE_F)

// ---------------------------------------------------------------------------
// cross-lane sums inside aligned groups of G lanes (G = 16 or 32)
// ---------------------------------------------------------------------------
// The leading empty asm makes `v` opaque: without it hipcc (fp-contract=fast)
// fuses the producer's multiply into the first butterfly add on THIS lane only
// (fma(a, b, partner) vs partner's rounded a*b), so lanes of one group end up
// with sums that differ in the last bit and their Newton state machines drift
// apart.  With both operands already rounded every step is a commutative add
// and all G lanes hold bitwise-identical sums.
template <int G>
__device__ __forceinline__ double gsum(double v) {
  asm volatile("" : "+v"(v));
#pragma unroll
  for (int m = G / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

__device__ __forceinline__ double softplus(double x) {
  return fmax(x, 0.0) + log1p(exp(-fabs(x)));
}
__device__ __forceinline__ double sigm(double u) { return 1.0 / (1.0 + exp(-u)); }
__device__ __forceinline__ double clampd(double x, double lo, double hi) {
  return fmin(fmax(x, lo), hi);
}
__device__ __forceinline__ double logit(double p) { return log(p) - log1p(-p); }

// theta-space sums of one objective evaluation (before the chain rule):
// 0 ell, 1 mag, 2..5 G(q,A,c,phi), 6..15 H upper triangle
// (qq qA qc qphi AA Ac Aphi cc cphi phiphi)
constexpr int kNAcc = 16;

// Per-lane point data of the current phase.
struct PointData {
  double y, N;
  int k;       // |z| - 1
  bool valid;  // a real point (not a pad lane)
  bool pmd;    // lane group fits model_PMD (else model_null)
};

// One point's contribution at u (identical formulas to oracle/mdfit_oracle.c
// evaluate(); see DESIGN.md §3 for the derivation).
__device__ __forceinline__ void point_eval(const PointData& pd, const double u[4],
                                           double acc[kNAcc], double& ell_out) {
  const double l1mq = -softplus(u[0]);  // ln(1-q)
  const double q = sigm(u[0]);
  double D, Dq, DA, Dc, Dqq, DqA;
  if (pd.pmd) {
    const double A = sigm(u[1]);
    const double c = u[2];
    const double kk = (double)pd.k;
    const double wq = exp((kk - 1.0) * l1mq);  // (1-q)^(k-1)
    const double w = exp(kk * l1mq);
    D = fma(A, w, c);
    DA = w;
    Dc = 1.0;
    Dq = pd.k >= 1 ? -A * kk * wq : 0.0;
    DqA = pd.k >= 1 ? -kk * wq : 0.0;
    Dqq = pd.k >= 2 ? A * kk * (kk - 1.0) * exp((kk - 2.0) * l1mq) : 0.0;
  } else {
    D = q;
    Dq = 1.0;
    DA = Dc = Dqq = DqA = 0.0;
  }
  const double phi = exp(u[3]) + 2.0;
  const double omD = 1.0 - D;
  const double a = D * phi, b = omD * phi;
  const LG3 t1 = lg3(pd.y + a);
  const LG3 t2 = lg3(pd.N - pd.y + b);
  const LG3 t3 = lg3(pd.N + phi);
  const LG3 t4 = lg3(a);
  const LG3 t5 = lg3(b);
  const LG3 t6 = lg3(phi);
  const double ell = (t1.l - t4.l) + (t2.l - t5.l) - (t3.l - t6.l);  // exact 0 when N = 0
  const double mag = fabs(t1.l) + fabs(t2.l) + fabs(t3.l) + fabs(t4.l) + fabs(t5.l) + fabs(t6.l);
  const double Pa = t1.p - t4.p, Pb = t2.p - t5.p, S = t6.p - t3.p;
  const double Qa = t1.q - t4.q, Qb = t2.q - t5.q, S1 = t6.q - t3.q;
  const double lD = phi * (Pa - Pb);
  const double lF = D * Pa + omD * Pb + S;
  const double lDD = phi * phi * (Qa + Qb);
  const double lDF = (Pa - Pb) + phi * (D * Qa - omD * Qb);
  const double lFF = D * D * Qa + omD * omD * Qb + S1;
  const double w = pd.valid ? 1.0 : 0.0;
  ell_out = ell;
  acc[0] = w * ell;
  acc[1] = w * mag;
  acc[2] = w * lD * Dq;
  acc[3] = w * lD * DA;
  acc[4] = w * lD * Dc;
  acc[5] = w * lF;
  acc[6] = w * (lDD * Dq * Dq + lD * Dqq);
  acc[7] = w * (lDD * Dq * DA + lD * DqA);
  acc[8] = w * (lDD * Dq * Dc);
  acc[9] = w * (lDF * Dq);
  acc[10] = w * (lDD * DA * DA);
  acc[11] = w * (lDD * DA * Dc);
  acc[12] = w * (lDF * DA);
  acc[13] = w * (lDD * Dc * Dc);
  acc[14] = w * (lDF * Dc);
  acc[15] = w * lFF;
}

// Objective in u-space from the group sums (oracle: evaluate(), chain rule part).
struct Eval {
  double F, mag;
  double g[4];
  double H[4][4];
};

__device__ __forceinline__ void finish_eval(bool pmd, const double u[4], const double s[kNAcc],
                                            Eval& e) {
  const double q = sigm(u[0]), omq = sigm(-u[0]);
  const double A = pmd ? sigm(u[1]) : 0.0, omA = pmd ? sigm(-u[1]) : 1.0;
  const double c = pmd ? u[2] : 0.0, omc = 1.0 - c;
  const double delta = exp(u[3]);
  const double G[4] = {s[2], s[3], s[4], s[5]};
  double Hh[4][4];
  Hh[0][0] = s[6];
  Hh[0][1] = Hh[1][0] = s[7];
  Hh[0][2] = Hh[2][0] = s[8];
  Hh[0][3] = Hh[3][0] = s[9];
  Hh[1][1] = s[10];
  Hh[1][2] = Hh[2][1] = s[11];
  Hh[1][3] = Hh[3][1] = s[12];
  Hh[2][2] = s[13];
  Hh[2][3] = Hh[3][2] = s[14];
  Hh[3][3] = s[15];
  const double J[4] = {q * omq, A * omA, 1.0, delta};
  const double J2[4] = {q * omq * (omq - q), A * omA * (omA - A), 0.0, delta};
  double lp = -softplus(-u[0]) - 2.0 * softplus(u[0]) - delta / 1000.0;
  double gp[4] = {1.0 - 3.0 * q, 0.0, 0.0, -delta / 1000.0};
  double hp[4] = {-3.0 * q * omq, 0.0, 0.0, -delta / 1000.0};
  if (pmd) {
    lp += -softplus(-u[1]) - 2.0 * softplus(u[1]) + 8.0 * log1p(-c);
    gp[1] = 1.0 - 3.0 * A;
    hp[1] = -3.0 * A * omA;
    gp[2] = -8.0 / omc;
    hp[2] = -8.0 / (omc * omc);
  }
  const bool infeasible = pmd && (A + c >= 1.0);
  e.F = infeasible ? INFINITY : -(s[0] + lp);
  e.mag = s[1];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    e.g[j] = -(J[j] * G[j] + gp[j]);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      double h = J[j] * Hh[j][m] * J[m];
      if (j == m) h += J2[j] * G[j] + hp[j];
      e.H[j][m] = -h;
    }
  }
  if (!pmd) {
#pragma unroll
    for (int j = 1; j <= 2; ++j) {
      e.g[j] = 0.0;
#pragma unroll
      for (int m = 0; m < 4; ++m) e.H[j][m] = e.H[m][j] = 0.0;
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

__constant__ double kEpsBind[4] = {1e-3, 1e-3, 1e-4, 1e-3};

// Projected, Hessian-modified Newton direction with a Bertsekas binding set
// (oracle: direction()): variables within eps of a bound and pushed outward
// step onto the bound and leave the Newton system.
__device__ void newton_dir(bool pmd, const double u[4], const double g[4], const double H[4][4],
                           double d[4]) {
  bool fr[4];
  double dbind[4];
  double w = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool fixed = !pmd && (j == 1 || j == 2);
    if (!fixed) w = fmax(w, fabs(u[j] - clampd(u[j] - g[j], kULo[j], kUHi[j])));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bool fixed = !pmd && (j == 1 || j == 2);
    const double eps = fmin(kEpsBind[j], w);
    const bool atlo = u[j] - kULo[j] <= eps, athi = kUHi[j] - u[j] <= eps;
    // on / next to a box bound and not pulled inward by more than kEpsAct
    const bool bind = (atlo && g[j] > -kEpsAct) || (athi && g[j] < kEpsAct);
    dbind[j] = (bind && !fixed) ? (atlo ? kULo[j] : kUHi[j]) - u[j] : 0.0;
    fr[j] = !(fixed || bind);
  }
  double sc = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (fr[j]) sc = fmax(sc, fabs(H[j][j]));
  if (sc == 0.0) sc = 1.0;
  double Lc[4][4];
  double mu = 0.0;
  bool ok = false;
  for (int attempt = 0; attempt < 40 && !ok; ++attempt) {
    ok = true;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if (m > j) continue;
        double s;
        if (!fr[j] || !fr[m]) s = (j == m) ? 1.0 : 0.0;
        else s = H[j][m] + ((j == m) ? mu : 0.0);
#pragma unroll
        for (int p = 0; p < 4; ++p)
          if (p < m) s -= Lc[j][p] * Lc[m][p];
        if (j == m) {
          if (!(s > 0.0)) ok = false;
          Lc[j][j] = sqrt(fmax(s, 1e-300));
        } else {
          Lc[j][m] = s / Lc[m][m];
        }
      }
    }
    if (!ok) mu = (mu == 0.0) ? 1e-10 * sc : mu * 10.0;
  }
  double rhs[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) rhs[j] = fr[j] ? -g[j] : 0.0;
  if (!ok) {
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] = isfinite(rhs[j]) ? rhs[j] : 0.0;
  } else {
    double z[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      double s = rhs[j];
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (p < j) s -= Lc[j][p] * z[p];
      z[j] = s / Lc[j][j];
    }
#pragma unroll
    for (int j = 3; j >= 0; --j) {
      double s = z[j];
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (p > j) s -= Lc[p][j] * d[p];
      d[j] = s / Lc[j][j];
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (!fr[j]) d[j] = dbind[j];
  const double mx = maxabs4(d);
  if (mx > 4.0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) d[j] *= 4.0 / mx;
  }
}

#ifdef MDFIT_TRACE
// debug-only build (-DMDFIT_TRACE): per-iteration trace of one taxon's fits
__device__ double* g_trace = nullptr;
__device__ int64_t g_trace_taxon = -1;
__device__ int g_trace_phase = 0;
#endif

// Result of one group's fit, replicated on every lane of the group.
struct FitOut {
  double u[4];
  double F;
  double ell;  // this lane's point log-likelihood at the returned mode
  int evals;
  int status;
};

// Run the per-group Newton state machines of one phase to completion.
// Must be called from wave-uniform control flow by all 64 lanes.
template <int G>
__device__ FitOut run_fits(const PointData& pd, const double u0[4], int max_iter, double tol) {
  FitOut o;
  double u[4], ut[4], d[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = ut[j] = u0[j];
  Eval cur;
  cur.F = INFINITY;
  cur.mag = 0.0;
  double ell_cur = 0.0;
  double t = 1.0;
  int evals = 0, status = MDFIT_MAXITER;
  bool first = true, done = false;
  while (__any(!done)) {
    double acc[kNAcc], ell;
    point_eval(pd, ut, acc, ell);
#pragma unroll
    for (int i = 0; i < kNAcc; ++i) acc[i] = gsum<G>(acc[i]);
    if (!done) {
      Eval tr;
      finish_eval(pd.pmd, ut, acc, tr);
      ++evals;
      bool accept;
      if (first) {
        accept = true;
        first = false;
        if (!isfinite(tr.F)) {
          done = true;
          status = MDFIT_NONFINITE;
        }
      } else {
        accept = isfinite(tr.F) &&
                 (tr.F < cur.F ||
                  (tr.F <= cur.F + kNoiseF * (cur.mag + fabs(cur.F)) &&
                   pgnorm(ut, tr.g) < pgnorm(u, cur.g)));
      }
      if (accept) {
#pragma unroll
        for (int j = 0; j < 4; ++j) u[j] = ut[j];
        cur = tr;
        ell_cur = ell;
        if (!done) {
          newton_dir(pd.pmd, u, cur.g, cur.H, d);
          t = 1.0;
          if (maxabs4(d) <= tol) {
            done = true;
            status = MDFIT_OK;
          }
        }
      } else {
        t *= 0.5;
        if (t < 1e-12) {
          done = true;
          status = maxabs4(d) <= 1e-5 ? MDFIT_OK : MDFIT_MAXITER;
        }
      }
      if (!done && evals >= max_iter) {
        done = true;
        status = MDFIT_MAXITER;
      }
      if (!done) {
#pragma unroll
        for (int j = 0; j < 4; ++j) ut[j] = clampd(u[j] + t * d[j], kULo[j], kUHi[j]);
      }
#ifdef MDFIT_TRACE
      if (g_trace != nullptr && (int64_t)blockIdx.x == g_trace_taxon && evals <= 200) {
        const int grp = G == 32 ? (threadIdx.x >> 5) : 2 + (threadIdx.x >> 4);
        double* r = g_trace + ((int64_t)grp * 200 + (evals - 1)) * 64;
        r[32 + (threadIdx.x % G)] = ell;
        r[16 + (threadIdx.x % G) % 16] = ut[0];
      }
      if (g_trace != nullptr && (int64_t)blockIdx.x == g_trace_taxon && (threadIdx.x % G) == 0 &&
          evals <= 200) {
        const int grp = G == 32 ? (threadIdx.x >> 5) : 2 + (threadIdx.x >> 4);
        double* r = g_trace + ((int64_t)grp * 200 + (evals - 1)) * 64;
        r[0] = tr.F; r[1] = cur.F; r[2] = accept; r[3] = t; r[4] = maxabs4(d);
        r[5] = maxabs4(tr.g); r[6] = maxabs4(cur.g); r[7] = cur.mag; r[8] = done; r[9] = status;
        for (int j = 0; j < 4; ++j) { r[10 + j] = u[j]; }
        r[14] = d[0]; r[15] = d[3];
      }
#endif
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) o.u[j] = u[j];
  o.F = cur.F;
  o.ell = ell_cur;
  o.evals = evals;
  o.status = status;
  return o;
}

// Initial point of MDFIT-MAP v1 (oracle: init_u) from group sums of the
// pooled ratios r(S) = (sum y + 0.5) / (sum N + 1).
template <int G>
__device__ void init_point(const PointData& pd, double u0[4]) {
  const double v = pd.valid ? 1.0 : 0.0;
  const double yall = gsum<G>(v * pd.y), nall = gsum<G>(v * pd.N);
  const double m1 = (pd.valid && pd.k == 0) ? 1.0 : 0.0;
  const double m2 = (pd.valid && pd.k == 1) ? 1.0 : 0.0;
  const double mt = (pd.valid && pd.k >= 9) ? 1.0 : 0.0;
  const double y1 = gsum<G>(m1 * pd.y), n1 = gsum<G>(m1 * pd.N);
  const double y2 = gsum<G>(m2 * pd.y), n2 = gsum<G>(m2 * pd.N);
  const double yt = gsum<G>(mt * pd.y), nt = gsum<G>(mt * pd.N);
  u0[3] = log(100.0);
  if (!pd.pmd) {
    u0[0] = logit(clampd((yall + 0.5) / (nall + 1.0), 1e-4, 0.9));
    u0[1] = u0[2] = 0.0;
    return;
  }
  const double c0 = clampd((yt + 0.5) / (nt + 1.0), 1e-4, 0.3);
  const double r1 = (y1 + 0.5) / (n1 + 1.0);
  const double r2 = (y2 + 0.5) / (n2 + 1.0);
  const double A0 = clampd(r1 - c0, 1e-3, 0.9 * (1.0 - c0));
  double q0 = 1.0 / 3.0;
  if (r1 - c0 > 1e-3) q0 = clampd(1.0 - (r2 - c0) / (r1 - c0), 0.05, 0.95);
  u0[0] = logit(q0);
  u0[1] = logit(A0);
  u0[2] = c0;
}

// MAP predictive summary of one point (oracle: predict()).
__device__ __forceinline__ void predict(double A, double q, double c, double phi, int k, double N,
                                        double o[3]) {
  if (N == 0.0) {
    o[0] = o[1] = o[2] = NAN;
    return;
  }
  double D = fma(A, pow(1.0 - q, (double)k), c);
  D = fmin(D, 1.0);
  const double sd = sqrt(D * (1.0 - D) * (phi + N) / (N * (phi + 1.0)));
  o[0] = D;
  o[1] = clampd(D - kZ68 * sd, 0.0, 1.0);
  o[2] = clampd(D + kZ68 * sd, 0.0, 1.0);
}

// n_sigma (fits.py:194-201) over the valid lanes of G-lane groups from each
// lane's waic difference d and waic values.
template <int G>
__device__ __forceinline__ double nsigma_group(bool valid, double lP, double lN, double n) {
  const double v = valid ? 1.0 : 0.0;
  const double d = v * ((-2.0 * lP) - (-2.0 * lN));
  const double md = gsum<G>(d) / n;
  const double wP = gsum<G>(v * (-2.0 * lP));
  const double wN = gsum<G>(v * (-2.0 * lN));
  const double dd = v * (d - md);
  const double var = gsum<G>(dd * dd) / n;
  return (wN - wP) / sqrt(n * var);
}

// Lane -> point maps of the two phases (see the header comment).
__device__ __forceinline__ PointData phase_a_point(int lane, const double* s_y, const double* s_N) {
  PointData pd;
  const int p = lane & 31;
  pd.valid = p < kNPos;
  const int pi = pd.valid ? p : 0;
  pd.y = s_y[pi];
  pd.N = s_N[pi];
  pd.k = pi < kNHalf ? pi : pi - kNHalf;
  pd.pmd = lane < 32;
  return pd;
}

__device__ __forceinline__ PointData phase_b_point(int lane, const double* s_y, const double* s_N) {
  PointData pd;
  const int row = lane >> 4, p = lane & 15;
  const bool rev = row & 1;
  pd.valid = p < kNHalf;
  const int pi = (pd.valid ? p : 0) + (rev ? kNHalf : 0);
  pd.y = s_y[pi];
  pd.N = s_N[pi];
  pd.k = pd.valid ? p : 0;
  pd.pmd = lane < 32;
  return pd;
}

constexpr int kBlock = 64;  // one wave = one taxon

__global__ __launch_bounds__(kBlock) void fit_map_kernel(
    const uint32_t* __restrict__ gy, const uint32_t* __restrict__ gN,
    const uint32_t* __restrict__ gmm, int64_t n_taxa, int max_iter, double tol,
    double* __restrict__ out, float* __restrict__ pred, int32_t* __restrict__ status) {
  __shared__ double s_y[kLD], s_N[kLD];
  __shared__ uint32_t s_mm[kNPos * kNMM];
  __shared__ double s_rec[MDFIT_NOUT];

  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  if (t >= n_taxa) return;

  // ---- stage counts (coalesced 128-B rows) --------------------------------
  if (lane < kLD) {
    s_y[lane] = (double)gy[t * kLD + lane];
    s_N[lane] = (double)gN[t * kLD + lane];
  }
  if (gmm != nullptr) {
    for (int i = lane; i < kNPos * kNMM; i += kBlock) s_mm[i] = gmm[t * (kNPos * kNMM) + i];
  }
  for (int i = lane; i < MDFIT_NOUT; i += kBlock) s_rec[i] = 0.0;
  __syncthreads();

  // invalid input (y > N) -> status 3, NaN record (oracle: fit_taxon)
  const bool bad_lane = lane < kNPos && s_y[lane] > s_N[lane];
  if (__any(bad_lane)) {
    for (int i = lane; i < MDFIT_NOUT; i += kBlock) out[t * MDFIT_NOUT + i] = NAN;
    if (pred != nullptr)
      for (int i = lane; i < MDFIT_NPRED * kNPos; i += kBlock)
        pred[t * (MDFIT_NPRED * kNPos) + i] = NAN;
    if (lane == 0) status[t] = MDFIT_INVALID;
    return;
  }

  int st = MDFIT_OK;
  // ======================= phase A: PMD-all | null-all =======================
  double ellPall;  // lane p < 30: PMD-all pointwise log-lik at the mode
  {
    const PointData pd = phase_a_point(lane, s_y, s_N);
    double u0[4];
    init_point<32>(pd, u0);
    const FitOut f = run_fits<32>(pd, u0, max_iter, tol);
    ellPall = f.ell;
    const double q = sigm(f.u[0]);
    const double A = pd.pmd ? sigm(f.u[1]) : 0.0;
    const double c = pd.pmd ? f.u[2] : 0.0;
    const double phi = exp(f.u[3]) + 2.0;
    // diagnostics: sub-fit 0 (PMD-all) from lane 0, sub-fit 1 (null-all) from lane 32
    if (lane == 0 || lane == 32) {
      double* dg = s_rec + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * (lane == 0 ? 0 : 1);
      dg[0] = q;
      dg[1] = A;
      dg[2] = c;
      dg[3] = phi;
      dg[4] = f.F;
      dg[5] = (double)f.evals;
      dg[6] = (double)f.status;
    }
    const int stA = max(__shfl(f.status, 0), __shfl(f.status, 32));
    st = max(st, stA);
    // predictions from PMD-all (fits.py:442-446 median + hpdi per position)
    double pr[3];
    predict(A, q, c, phi, pd.k, pd.N, pr);
    if (lane < kNPos && pred != nullptr) {
#pragma unroll
      for (int r = 0; r < 3; ++r) pred[t * (MDFIT_NPRED * kNPos) + r * kNPos + lane] = (float)pr[r];
    }
    if (lane == 0) {
      s_rec[MDFIT_F_D_MAX] = pr[0];  // fits.py:249-250
      s_rec[MDFIT_F_D_MAX_LOWER_HPDI] = pr[1];
      s_rec[MDFIT_F_D_MAX_UPPER_HPDI] = pr[2];
      s_rec[MDFIT_F_Q_MEAN] = q;
      s_rec[MDFIT_F_CONCENTRATION_MEAN] = phi;
      s_rec[MDFIT_F_D_MAX_MARGINALIZED_MEAN] = A + c;
    }
    // n_sigma (fits.py:252) : PMD lane p vs null lane p+32
    const double ellN = __shfl_xor(f.ell, 32);
    const double ns = nsigma_group<32>(pd.valid, f.ell, ellN, (double)kNPos);
    if (lane == 0) s_rec[MDFIT_F_N_SIGMA] = ns;
  }

  // ================ phase B: PMD-fwd | PMD-rev | null-fwd | null-rev =========
  {
    const int row = lane >> 4, p = lane & 15;
    const PointData pd = phase_b_point(lane, s_y, s_N);
    double u0[4];
    init_point<16>(pd, u0);
    const FitOut f = run_fits<16>(pd, u0, max_iter, tol);
    const double q = sigm(f.u[0]);
    const double A = pd.pmd ? sigm(f.u[1]) : 0.0;
    const double c = pd.pmd ? f.u[2] : 0.0;
    const double phi = exp(f.u[3]) + 2.0;
    if (p == 0) {  // lanes 0, 16, 32, 48 -> sub-fits 2, 3, 4, 5
      double* dg = s_rec + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * (2 + row);
      dg[0] = q;
      dg[1] = A;
      dg[2] = c;
      dg[3] = phi;
      dg[4] = f.F;
      dg[5] = (double)f.evals;
      dg[6] = (double)f.status;
    }
    const int stB = max(max(__shfl(f.status, 0), __shfl(f.status, 16)),
                        max(__shfl(f.status, 32), __shfl(f.status, 48)));
    st = max(st, stB);
    // n_sigma_forward / _reverse (fits.py:317-320, 339-342): PMD row vs null row (+32)
    const double ellN = __shfl_xor(f.ell, 32);
    const double ns = nsigma_group<16>(pd.valid, f.ell, ellN, (double)kNHalf);
    // D_max_forward / _reverse: predictive median at data_forward[0]
    // (fits.py:322-327; the reverse one is evaluated on data_forward, :343-348)
    double pr[3];
    predict(A, q, c, phi, 0, s_N[0], pr);
    if (lane == 0) {
      s_rec[MDFIT_F_N_SIGMA_FORWARD] = ns;
      s_rec[MDFIT_F_D_MAX_FORWARD] = pr[0];
      s_rec[MDFIT_F_Q_MEAN_FORWARD] = q;
    }
    if (lane == 16) {
      s_rec[MDFIT_F_N_SIGMA_REVERSE] = ns;
      s_rec[MDFIT_F_D_MAX_REVERSE] = pr[0];
      s_rec[MDFIT_F_Q_MEAN_REVERSE] = q;
    }
    // asymmetry (fits.py:352-356, 204-227): PMD-all vs concat(PMD-fwd, PMD-rev);
    // point p of the concatenation lives on lane p (p < 15) or lane p + 1.
    const int src = lane < kNHalf ? lane : lane + 1;
    const double ellFR = __shfl(f.ell, src & 63);
    const bool vA = lane < kNPos;
    const double v = vA ? 1.0 : 0.0;
    const double dC = v * ((-2.0 * ellPall) - (-2.0 * ellFR));
    const double md = gsum<64>(dC) / kNPos;
    const double wC = gsum<64>(v * (-2.0 * ellPall));
    const double wFR = gsum<64>(v * (-2.0 * ellFR));
    const double dd = v * (dC - md);
    const double var = gsum<64>(dd * dd) / kNPos;
    if (lane == 0) s_rec[MDFIT_F_ASYMMETRY] = (wFR - wC) / sqrt(kNPos * var);
  }

  // ==================== sums (fits.py:272-283) ===============================
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

  // ==================== noise (fits.py:359-376) ==============================
  {
    // lane j < 12 owns mismatch column j (AC AG AT CA CG CT GA GC GT TA TC TG);
    // CT is NaN on rows 0..14, GA on rows 15..29.
    const int j = lane < kNMM ? lane : 0;
    const bool own = lane < kNMM && gmm != nullptr;
    double s = 0.0, cnt = 0.0;
    for (int i = 0; i < kNPos; ++i) {
      const bool nanned = (j == 5 && i < kNHalf) || (j == 6 && i >= kNHalf);
      if (!nanned) {
        s += (double)s_mm[i * kNMM + j];
        cnt += 1.0;
      }
    }
    const double m = s / cnt;
    double sa[3] = {0, 0, 0}, ca[3] = {0, 0, 0};
    for (int i = 0; i < kNPos; ++i) {
      const bool nanned = (j == 5 && i < kNHalf) || (j == 6 && i >= kNHalf);
      const double x = (double)s_mm[i * kNMM + j] / m;
      if (own && !nanned && !isnan(x)) {
        const int h = i < kNHalf ? 1 : 2;
        sa[0] += x;
        ca[0] += 1.0;
        sa[h] += x;
        ca[h] += 1.0;
      }
    }
    double mean[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) mean[r] = gsum<16>(sa[r]) / gsum<16>(ca[r]);
    double ss[3] = {0, 0, 0};
    for (int i = 0; i < kNPos; ++i) {
      const bool nanned = (j == 5 && i < kNHalf) || (j == 6 && i >= kNHalf);
      const double x = (double)s_mm[i * kNMM + j] / m;
      if (own && !nanned && !isnan(x)) {
        const int h = i < kNHalf ? 1 : 2;
        ss[0] += (x - mean[0]) * (x - mean[0]);
        ss[h] += (x - mean[h]) * (x - mean[h]);
      }
    }
    double nz[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const double c = gsum<16>(ca[r]);
      nz[r] = c > 0.0 ? sqrt(gsum<16>(ss[r]) / c) : NAN;
    }
    if (lane == 0) {
      const bool have = gmm != nullptr;
      s_rec[MDFIT_F_NORMALIZED_NOISE] = have ? nz[0] : NAN;
      s_rec[MDFIT_F_NORMALIZED_NOISE_FORWARD] = have ? nz[1] : NAN;
      s_rec[MDFIT_F_NORMALIZED_NOISE_REVERSE] = have ? nz[2] : NAN;
    }
  }

  __syncthreads();
  for (int i = lane; i < MDFIT_NOUT; i += kBlock) out[t * MDFIT_NOUT + i] = s_rec[i];
  if (lane == 0) status[t] = st;
}

// ---------------------------------------------------------------------------
// parity / roofline helper kernels
// ---------------------------------------------------------------------------
__global__ void special_kernel(const double* __restrict__ x, int64_t n, double* __restrict__ o) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const LG3 r = lg3(x[i]);
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
  const LG3 c0 = lg3(m + 1.0), c1 = lg3(k + 1.0), c2 = lg3(m - k + 1.0);
  const LG3 t1 = lg3(k + al), t2 = lg3(m - k + be), t3 = lg3(m + al + be);
  const LG3 t4 = lg3(al), t5 = lg3(be), t6 = lg3(al + be);
  o[i] = (c0.l - c1.l - c2.l) + (t1.l + t2.l - t3.l) - (t4.l + t5.l - t6.l);
  if (g != nullptr) {
    const double ps = t6.p - t3.p;
    g[2 * i + 0] = t1.p - t4.p + ps;
    g[2 * i + 1] = t2.p - t5.p + ps;
  }
}

// Register-only throughput probe: each lane evaluates point_eval `iters`
// times on a representative argument mix (a needs the small-x shift, the
// others do not — as in typical fits).
__global__ __launch_bounds__(kBlock) void peak_probe_kernel(int iters, double* __restrict__ sink) {
  const int lane = threadIdx.x;
  PointData pd;
  pd.valid = true;
  pd.pmd = true;
  pd.k = lane % kNHalf;
  pd.N = 1.0e5 + 1000.0 * lane;
  pd.y = 0.01 * pd.N;
  double u[4] = {-0.5, -3.0, -4.5, 6.0};
  double accum = 0.0;
  for (int it = 0; it < iters; ++it) {
    double acc[kNAcc], ell;
    point_eval(pd, u, acc, ell);
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < kNAcc; ++i) s += acc[i];
    accum += s;
    u[0] += 1e-9 * s;  // loop-carried dependence: no hoisting
  }
  sink[(int64_t)blockIdx.x * kBlock + lane] = accum;
}

// Objective / gradient / Hessian of one sub-fit at a given u, evaluated with
// exactly the lane layout and code of the fit kernel (parity tests of the
// objective itself).  One wave per item.
__global__ __launch_bounds__(kBlock) void objective_kernel(
    const int32_t* __restrict__ model, const int32_t* __restrict__ subset,
    const uint32_t* __restrict__ gy, const uint32_t* __restrict__ gN, const double* __restrict__ gu,
    int64_t n, double* __restrict__ F, double* __restrict__ g, double* __restrict__ H,
    double* __restrict__ ell_out) {
  __shared__ double s_y[kLD], s_N[kLD];
  const int lane = threadIdx.x;
  const int64_t i = blockIdx.x;
  if (i >= n) return;
  if (lane < kLD) {
    s_y[lane] = (double)gy[i * kLD + lane];
    s_N[lane] = (double)gN[i * kLD + lane];
  }
  __syncthreads();
  const int m = model[i], sub = subset[i];
  double u[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = gu[i * 4 + j];
  double acc[kNAcc], ell;
  Eval e;
  int lead, point;
  bool mine;
  if (sub == 0) {
    const PointData pd = phase_a_point(lane, s_y, s_N);
    point_eval(pd, u, acc, ell);
#pragma unroll
    for (int k = 0; k < kNAcc; ++k) acc[k] = gsum<32>(acc[k]);
    finish_eval(pd.pmd, u, acc, e);
    lead = m == 0 ? 0 : 32;
    mine = (lane >> 5) == (lead >> 5) && pd.valid;
    point = lane & 31;
  } else {
    const PointData pd = phase_b_point(lane, s_y, s_N);
    point_eval(pd, u, acc, ell);
#pragma unroll
    for (int k = 0; k < kNAcc; ++k) acc[k] = gsum<16>(acc[k]);
    finish_eval(pd.pmd, u, acc, e);
    lead = 16 * ((m == 0 ? 0 : 2) + (sub == 2 ? 1 : 0));
    mine = (lane >> 4) == (lead >> 4) && pd.valid;
    point = (lane & 15) + (sub == 2 ? kNHalf : 0);
  }
  if (lane < kNPos) ell_out[i * kNPos + lane] = 0.0;
  __syncthreads();
  if (mine) ell_out[i * kNPos + point] = ell;
  if (lane == lead) {
    F[i] = e.F;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      g[i * 4 + j] = e.g[j];
#pragma unroll
      for (int k = 0; k < 4; ++k) H[i * 16 + 4 * j + k] = e.H[j][k];
    }
  }
}

}  // namespace mdfit

// ===========================================================================
// C-ABI
// ===========================================================================
namespace {
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
}  // namespace

extern "C" {

void mdfit_default_opts(mdfit_opts* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->mode = MDFIT_MODE_MAP;
  o->max_iter = 200;
  o->tol_step = 1e-9;
  o->seed = 0;
  o->num_warmup = 500;
  o->num_samples = 1000;
}

int64_t mdfit_workspace_bytes(void) { return 256; }

int mdfit_fit_batch(const uint32_t* y, const uint32_t* N, const uint32_t* mm, int64_t n_taxa,
                    const mdfit_opts* opts, double* out, float* pred, int32_t* status,
                    void* workspace, void* hip_stream) {
  (void)workspace;
  if (n_taxa < 0) return set_err(MDFIT_E_ARG, "n_taxa < 0");
  if (n_taxa == 0) return 0;
  if (!y || !N || !out || !status) return set_err(MDFIT_E_ARG, "null required pointer");
  mdfit_opts o;
  mdfit_default_opts(&o);
  if (opts) o = *opts;
  if (o.mode != MDFIT_MODE_MAP) return set_err(MDFIT_E_ARG, "unsupported mode");
  if (o.max_iter < 1) return set_err(MDFIT_E_ARG, "max_iter < 1");
  if (n_taxa > (int64_t)0x7fffffff) return set_err(MDFIT_E_ARG, "n_taxa exceeds grid limit");
  hipStream_t s = (hipStream_t)hip_stream;
  hipLaunchKernelGGL(mdfit::fit_map_kernel, dim3((unsigned)n_taxa), dim3(mdfit::kBlock), 0, s, y,
                     N, mm, n_taxa, o.max_iter, o.tol_step, out, pred, status);
  return check_launch("fit_map_kernel");
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

int mdfit_special(const double* x, int64_t n, double* out3, void* hip_stream) {
  if (n < 0 || (n > 0 && (!x || !out3))) return set_err(MDFIT_E_ARG, "bad arguments");
  if (n == 0) return 0;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(mdfit::special_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)hip_stream,
                     x, n, out3);
  return check_launch("special_kernel");
}

int mdfit_peak_probe(int64_t n_waves, int32_t iters, double* sink, void* hip_stream) {
  if (n_waves <= 0 || iters <= 0 || !sink) return set_err(MDFIT_E_ARG, "bad arguments");
  hipLaunchKernelGGL(mdfit::peak_probe_kernel, dim3((unsigned)n_waves), dim3(mdfit::kBlock), 0,
                     (hipStream_t)hip_stream, iters, sink);
  return check_launch("peak_probe_kernel");
}

int mdfit_objective(const int32_t* model, const int32_t* subset, const uint32_t* y,
                    const uint32_t* N, const double* u, int64_t n, double* F, double* g,
                    double* H, double* ell, void* hip_stream) {
  if (n < 0 || (n > 0 && (!model || !subset || !y || !N || !u || !F || !g || !H || !ell)))
    return set_err(MDFIT_E_ARG, "bad arguments");
  if (n == 0) return 0;
  hipLaunchKernelGGL(mdfit::objective_kernel, dim3((unsigned)n), dim3(mdfit::kBlock), 0,
                     (hipStream_t)hip_stream, model, subset, y, N, u, n, F, g, H, ell);
  return check_launch("objective_kernel");
}

#ifdef MDFIT_TRACE
int mdfit_set_trace(double* buf, int64_t taxon) {
  hipMemcpyToSymbol(HIP_SYMBOL(mdfit::g_trace), &buf, sizeof(buf));
  hipMemcpyToSymbol(HIP_SYMBOL(mdfit::g_trace_taxon), &taxon, sizeof(taxon));
  return 0;
}
#endif

const char* mdfit_last_error(void) { return g_err; }

int mdfit_abi_version(void) { return MDFIT_ABI_VERSION; }

}  // extern "C"
