/*
 * mdfit_oracle.c — CPU ORACLE (test infrastructure only).
 *
 * Plain-C FP64 restatement of the per-taxon damage fit that the HIP kernel in
 * metadamage_amd/csrc/mdfit.hip implements.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library; the product path never
 * does.  It is written independently of the kernel (scalar loops over points,
 * libm lgamma, textbook digamma/trigamma) so that a kernel bug cannot hide in
 * shared code.
 *
 * What it restates (reference = /root/reference/metadamage):
 *   model_PMD                    fits.py:43-59   (priors, D(z), BetaBinomial)
 *   model_null                   fits.py:62-67
 *   BetaBinomial log-pmf         numpyro ^0.4.1 (pyproject.toml:17), same
 *                                formula as scipy.stats.betabinom.logpmf
 *   group_to_numpyro_data        fits.py:398-419 (dense [30] layout, z implicit)
 *   get_lppd_and_waic            fits.py:147-172 (one "sample" = the mode)
 *   compute_n_sigma              fits.py:194-201
 *   compute_assymmetry_...       fits.py:204-227
 *   compute_fit_results          fits.py:230-295 (record assembly)
 *   add_assymetry_results_...    fits.py:298-356 (fwd/rev sub-fits; the
 *                                D_max_reverse-on-data_forward quirk, :343-348)
 *   add_noise_estimates          fits.py:359-376
 *
 * The inference is the build-defined MAP mode "MDFIT-MAP v1.1" (DESIGN.md §3):
 * the reference only samples with NUTS (fits.py:382-387), so the MAP spec is
 * ours; parity of the MAP optimum itself is pinned against an independent
 * scipy optimiser (tests/golden/make_golden_scipy.py), and the WAIC /
 * n_sigma / asymmetry / noise / packing formulas against the reference's own
 * functions (tests/golden/make_golden_reference.py).
 */
/* lgamma_r / lgammal_r: the reentrant forms (plain lgamma writes the global
 * signgam, a cache line every OpenMP thread then fights over: the oracle ran
 * 1.6x faster on 8 threads than on 1 with it) */
#define _DEFAULT_SOURCE 1
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mdfit.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#define NPOS 30
#define NHALF 15

/* ---------------------------------------------------------------------------
 * special functions (oracle versions: libm lgamma, recurrence + asymptotic
 * series for digamma / trigamma)
 * ------------------------------------------------------------------------- */
static double o_lgamma(double x) {
  int sg;
  return lgamma_r(x, &sg);
}
static long double o_lgammal(long double x) {
  int sg;
  return lgammal_r(x, &sg);
}

static double o_digamma(double x) {
  double acc = 0.0;
  while (x < 12.0) {
    acc -= 1.0 / x;
    x += 1.0;
  }
  double r = 1.0 / x, r2 = r * r;
  /* psi(x) ~ ln x - 1/(2x) - sum B_2k / (2k x^2k) */
  double s = r2 * (1.0 / 12 -
             r2 * (1.0 / 120 -
             r2 * (1.0 / 252 -
             r2 * (1.0 / 240 -
             r2 * (1.0 / 132 -
             r2 * (691.0 / 32760 -
             r2 * (1.0 / 12)))))));
  return acc + log(x) - 0.5 * r - s;
}

static double o_trigamma(double x) {
  double acc = 0.0;
  while (x < 12.0) {
    acc += 1.0 / (x * x);
    x += 1.0;
  }
  double r = 1.0 / x, r2 = r * r;
  /* psi1(x) ~ 1/x + 1/(2x^2) + sum B_2k / x^(2k+1) */
  double s = r * r2 * (1.0 / 6 -
             r2 * (1.0 / 30 -
             r2 * (1.0 / 42 -
             r2 * (1.0 / 30 -
             r2 * (5.0 / 66 -
             r2 * (691.0 / 2730 -
             r2 * (7.0 / 6)))))));
  return acc + r + 0.5 * r2 + s;
}

void oracle_special(const double* x, int64_t n, double* out3) {
  for (int64_t i = 0; i < n; i++) {
    out3[3 * i + 0] = o_lgamma(x[i]);
    out3[3 * i + 1] = o_digamma(x[i]);
    out3[3 * i + 2] = o_trigamma(x[i]);
  }
}

/* numpyro BetaBinomial.log_prob incl. the binomial coefficient */
void oracle_betabinom_logpmf(const double* y, const double* N, const double* a,
                             const double* b, int64_t n, double* out,
                             double* grad) {
  for (int64_t i = 0; i < n; i++) {
    double k = y[i], m = N[i];
    double lc = o_lgamma(m + 1) - o_lgamma(k + 1) - o_lgamma(m - k + 1);
    double lb1 = o_lgamma(k + a[i]) + o_lgamma(m - k + b[i]) - o_lgamma(m + a[i] + b[i]);
    double lb0 = o_lgamma(a[i]) + o_lgamma(b[i]) - o_lgamma(a[i] + b[i]);
    out[i] = lc + lb1 - lb0;
    if (grad) {
      double ps = o_digamma(a[i] + b[i]) - o_digamma(m + a[i] + b[i]);
      grad[2 * i + 0] = o_digamma(k + a[i]) - o_digamma(a[i]) + ps;
      grad[2 * i + 1] = o_digamma(m - k + b[i]) - o_digamma(b[i]) + ps;
    }
  }
}

/* ---------------------------------------------------------------------------
 * model pieces
 * ------------------------------------------------------------------------- */
enum { M_PMD = 0, M_NULL = 1 };
enum { P_Q = 0, P_A = 1, P_C = 2, P_D = 3 }; /* u-space parameter slots */

/* u = (logit q, logit A, c, log delta); c is optimised on its own scale so a
 * background rate that the data do not support lands exactly on c = 0 (the
 * mode of its Beta(1,9) prior) in one projected step instead of an
 * exponentially slow walk down logit c. */
static const double U_LO[4] = {-25.0, -25.0, 0.0, -25.0};
static const double U_HI[4] = {25.0, 25.0, 0.999, 20.0};
#define EPS_ACT 1e-8
/* rounding scale of the objective: a trial whose F is within NOISE_F*(sum |lnGamma| + |F|)
 * of the current one is accepted when it lowers the projected gradient */
#define NOISE_F 1.4e-14
/* projected-gradient size below which an exhausted line search counts as converged */
#define PG_TOL 1e-6

static double softplus(double x) { return (x > 0 ? x : 0.0) + log1p(exp(-fabs(x))); }
static double sigm(double u) { return 1.0 / (1.0 + exp(-u)); }

typedef struct {
  double F;        /* objective  -(sum ell_i + log prior)            */
  double g[4];     /* dF/du                                          */
  double H[4][4];  /* d2F/du2                                        */
  double mag;      /* sum |lgamma terms| (noise scale of F)          */
  double ell[NPOS];/* pointwise log-likelihood (without log C(N,y));
                    * the full log-pmf in the polish phase             */
} evalres;

static long double lrise_l(long double n, long double s);

/* absolute position |z| - 1 of dense column i */
static int kpos(int i) { return i < NHALF ? i : i - NHALF; }

/* Evaluate the objective at u for the points i in [lo, hi).
 *
 * accf = 0: F = -(sum_i ell_i + ln p) with ell_i the beta-binomial log-pmf
 * without the data-only log C(N,y), as a sum of six lnGamma values per point
 * (each ~N ln N: at N ~ 1e7 the sum carries ~1e-6 of rounding).
 * accf = 1 (the polish phase of fit_one): ell_i is the full log-pmf in the
 * cancellation-free form R(y,a) + R(N-y,b) - R(N,phi) (bb_logpmf_full, below;
 * F shifts by the constant sum log C(N,y)), so F resolves differences of
 * ~1e-10 and the line search can follow a flat valley to its optimum.  The
 * gradient and Hessian are the same in both forms. */
static void evaluate(int model, const uint32_t* y, const uint32_t* N, int lo,
                     int hi, const double u[4], evalres* r, int accf) {
  double q = sigm(u[P_Q]);
  double omq = sigm(-u[P_Q]);
  double l1mq = -softplus(u[P_Q]); /* ln(1-q) */
  double A = 0, omA = 1, c = 0, omc = 1;
  if (model == M_PMD) {
    A = sigm(u[P_A]);
    omA = sigm(-u[P_A]);
    c = u[P_C];
    omc = 1.0 - c;
  }
  double delta = exp(u[P_D]);
  double phi = delta + 2.0;

  double G[4] = {0, 0, 0, 0};
  double Hh[4][4];
  memset(Hh, 0, sizeof(Hh));
  double L = 0.0, mag = 0.0;
  int infeasible = (model == M_PMD) && (A + c >= 1.0);

  for (int i = lo; i < hi && !infeasible; i++) {
    int k = kpos(i);
    double yy = (double)y[i], NN = (double)N[i];
    double D, Dq = 0, DA = 0, Dc = 0, Dqq = 0, DqA = 0;
    if (model == M_PMD) {
      double w = exp(k * l1mq);
      D = A * w + c;
      DA = w;
      Dc = 1.0;
      if (k >= 1) {
        double wq = exp((k - 1) * l1mq); /* (1-q)^(k-1) */
        Dq = -A * k * wq;
        DqA = -k * wq;
        if (k >= 2) Dqq = A * k * (k - 1) * exp((k - 2) * l1mq);
      }
    } else {
      D = q;
      Dq = 1.0;
    }
    double omD = 1.0 - D;
    double a = D * phi, b = omD * phi;
    double t1 = o_lgamma(yy + a), t2 = o_lgamma(NN - yy + b), t3 = o_lgamma(NN + phi);
    double t4 = o_lgamma(a), t5 = o_lgamma(b), t6 = o_lgamma(phi);
    double ell = (t1 - t4) + (t2 - t5) - (t3 - t6); /* exact 0 when N = 0 */
    if (accf) {
      long double r1 = lrise_l(yy, a), r2 = lrise_l(NN - yy, b), r3 = lrise_l(NN, phi);
      ell = (double)(r1 + r2 - r3);
      mag += (double)(fabsl(r1) + fabsl(r2) + fabsl(r3));
    } else {
      mag += fabs(t1) + fabs(t2) + fabs(t3) + fabs(t4) + fabs(t5) + fabs(t6);
    }
    r->ell[i] = ell;
    L += ell;
    double Pa = o_digamma(yy + a) - o_digamma(a);
    double Pb = o_digamma(NN - yy + b) - o_digamma(b);
    double S = o_digamma(phi) - o_digamma(NN + phi);
    double Qa = o_trigamma(yy + a) - o_trigamma(a);
    double Qb = o_trigamma(NN - yy + b) - o_trigamma(b);
    double S1 = o_trigamma(phi) - o_trigamma(NN + phi);
    double lD = phi * (Pa - Pb);
    double lF = D * Pa + omD * Pb + S;
    double lDD = phi * phi * (Qa + Qb);
    double lDF = (Pa - Pb) + phi * (D * Qa - omD * Qb);
    double lFF = D * D * Qa + omD * omD * Qb + S1;
    double dD[3] = {Dq, DA, Dc};
    for (int j = 0; j < 3; j++) {
      G[j] += lD * dD[j];
      for (int m = 0; m < 3; m++) Hh[j][m] += lDD * dD[j] * dD[m];
      Hh[j][3] += lDF * dD[j];
    }
    Hh[P_Q][P_Q] += lD * Dqq;
    Hh[P_Q][P_A] += lD * DqA;
    Hh[P_A][P_Q] += lD * DqA;
    G[3] += lF;
    Hh[3][3] += lFF;
  }
  if (infeasible) {
    r->F = INFINITY;
    r->mag = 0;
    for (int j = 0; j < 4; j++) {
      r->g[j] = 0;
      for (int m = 0; m < 4; m++) r->H[j][m] = 0;
    }
    return;
  }
  for (int j = 0; j < 3; j++) Hh[3][j] = Hh[j][3];

  /* chain rule to u-space: theta = (q, A, c, phi), dtheta/du = J, d2theta/du2 = J2 */
  double J[4] = {q * omq, A * omA, 1.0, delta};
  double J2[4] = {q * omq * (omq - q), A * omA * (omA - A), 0.0, delta};
  /* log prior (constants dropped): ln q + 2 ln(1-q) [+ ln A + 2 ln(1-A) + 8 ln(1-c)] - delta/1000 */
  double lq = -softplus(-u[P_Q]);
  double lp = lq + 2.0 * l1mq - delta / 1000.0;
  double gp[4] = {1.0 - 3.0 * q, 0, 0, -delta / 1000.0};
  double hp[4] = {-3.0 * q * omq, 0, 0, -delta / 1000.0};
  if (model == M_PMD) {
    lp += -softplus(-u[P_A]) + 2.0 * (-softplus(u[P_A])) + 8.0 * log1p(-c);
    gp[P_A] = 1.0 - 3.0 * A;
    hp[P_A] = -3.0 * A * omA;
    gp[P_C] = -8.0 / omc;
    hp[P_C] = -8.0 / (omc * omc);
  }
  r->F = -(L + lp);
  r->mag = mag;
  for (int j = 0; j < 4; j++) {
    r->g[j] = -(J[j] * G[j] + gp[j]);
    for (int m = 0; m < 4; m++) {
      double h = J[j] * Hh[j][m] * J[m];
      if (j == m) h += J2[j] * G[j] + hp[j];
      r->H[j][m] = -h;
    }
  }
  if (model == M_NULL) { /* A, c are not parameters of model_null */
    for (int j = 1; j <= 2; j++) {
      r->g[j] = 0;
      for (int m = 0; m < 4; m++) r->H[j][m] = r->H[m][j] = 0;
    }
  }
}

/* pooled ratio (sum y + 0.5) / (sum N + 1) over points i in [lo,hi) with
 * kmin <= |z|-1 <= kmax */
static double pooled(const uint32_t* y, const uint32_t* N, int lo, int hi,
                     int kmin, int kmax) {
  double sy = 0, sn = 0;
  for (int i = lo; i < hi; i++) {
    int k = kpos(i);
    if (k >= kmin && k <= kmax) {
      sy += y[i];
      sn += N[i];
    }
  }
  return (sy + 0.5) / (sn + 1.0);
}

static double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
static double logit(double p) { return log(p) - log1p(-p); }

static void init_u(int model, const uint32_t* y, const uint32_t* N, int lo,
                   int hi, double u[4]) {
  u[P_A] = 0;
  u[P_C] = 0;
  u[P_D] = log(100.0);
  if (model == M_NULL) {
    u[P_Q] = logit(clampd(pooled(y, N, lo, hi, 0, 99), 1e-4, 0.9));
    return;
  }
  double c0 = clampd(pooled(y, N, lo, hi, 9, 99), 1e-4, 0.3);
  double r1 = pooled(y, N, lo, hi, 0, 0);
  double r2 = pooled(y, N, lo, hi, 1, 1);
  double A0 = clampd(r1 - c0, 1e-3, 0.9 * (1.0 - c0));
  double q0 = 1.0 / 3.0;
  if (r1 - c0 > 1e-3) q0 = clampd(1.0 - (r2 - c0) / (r1 - c0), 0.05, 0.95);
  u[P_Q] = logit(q0);
  u[P_A] = logit(A0);
  u[P_C] = c0;
}

static double maxabs4(const double v[4]) {
  double m = 0;
  for (int j = 0; j < 4; j++)
    if (fabs(v[j]) > m) m = fabs(v[j]);
  return m;
}

/* projected, Hessian-modified Newton direction (Bertsekas-style binding set):
 * a variable within eps of a bound whose gradient pushes it outward is moved
 * onto the bound (d = bound - u) and removed from the Newton system; the
 * others take the (Hessian-modified) Newton step of the reduced system. */
static const double EPS_BIND[4] = {1e-3, 1e-3, 1e-4, 1e-3};
/* the quadratic-contraction stop of fit_one (MDFIT-MAP v1.1) */
#define QUAD_K 10.0

static void free_set(int model, const double u[4], const double g[4], double H[4][4], int fr[4],
                     double dbind[4]) {
  double w = 0; /* projected-gradient size */
  for (int j = 0; j < 4; j++) {
    if (model == M_NULL && (j == P_A || j == P_C)) continue;
    double pg = fabs(u[j] - clampd(u[j] - g[j], U_LO[j], U_HI[j]));
    if (pg > w) w = pg;
  }
  for (int j = 0; j < 4; j++) {
    int fixed = (model == M_NULL && (j == P_A || j == P_C));
    double eps = EPS_BIND[j] < w ? EPS_BIND[j] : w;
    double dlo = u[j] - U_LO[j], dhi = U_HI[j] - u[j];
    int atlo = dlo <= eps, athi = dhi <= eps;
    /* a variable on (or next to) its box bound stays there unless the
     * objective pulls it inward by more than EPS_ACT -- or, next to the bound
     * with positive curvature, unless its own Newton step g/H stops short of
     * the bound (an interior optimum just inside it) */
    double hjj = H[j][j];
    int bind = (atlo && g[j] > -EPS_ACT && (hjj <= 0 || g[j] + EPS_ACT > hjj * dlo)) ||
               (athi && g[j] < EPS_ACT && (hjj <= 0 || -g[j] + EPS_ACT > hjj * dhi));
    dbind[j] = (bind && !fixed) ? (atlo ? U_LO[j] : U_HI[j]) - u[j] : 0.0;
    fr[j] = !(fixed || bind);
  }
}

/* returns 1 when the free block of H is not positive definite (the Cholesky
 * needed a shift) */
static int direction(int model, const double u[4], const double g[4], double H[4][4], double d[4]) {
  int fr[4];
  double dbind[4];
  free_set(model, u, g, H, fr, dbind);
  double sc = 0;
  for (int j = 0; j < 4; j++)
    if (fr[j] && fabs(H[j][j]) > sc) sc = fabs(H[j][j]);
  if (sc == 0) sc = 1.0;
  double mu = 0.0;
  double Lc[4][4];
  int ok = 0;
  for (int attempt = 0; attempt < 40; attempt++) {
    ok = 1;
    for (int j = 0; j < 4 && ok; j++) {
      for (int m = 0; m <= j; m++) {
        double s;
        if (!fr[j] || !fr[m]) s = (j == m) ? 1.0 : 0.0;
        else s = H[j][m] + ((j == m) ? mu : 0.0);
        for (int p = 0; p < m; p++) s -= Lc[j][p] * Lc[m][p];
        if (j == m) {
          if (!(s > 0)) { ok = 0; break; }
          Lc[j][j] = sqrt(s);
        } else {
          Lc[j][m] = s / Lc[m][m];
        }
      }
    }
    if (ok) break;
    mu = (mu == 0.0) ? 1e-10 * sc : mu * 10.0;
  }
  double rhs[4], z[4];
  for (int j = 0; j < 4; j++) rhs[j] = fr[j] ? -g[j] : 0.0;
  if (!ok) { /* no usable curvature (non-finite Hessian): steepest descent */
    for (int j = 0; j < 4; j++) d[j] = isfinite(rhs[j]) ? rhs[j] : 0.0;
    goto cap;
  }
  for (int j = 0; j < 4; j++) {
    double s = rhs[j];
    for (int p = 0; p < j; p++) s -= Lc[j][p] * z[p];
    z[j] = s / Lc[j][j];
  }
  for (int j = 3; j >= 0; j--) {
    double s = z[j];
    for (int p = j + 1; p < 4; p++) s -= Lc[p][j] * d[p];
    d[j] = s / Lc[j][j];
  }
cap:;
  for (int j = 0; j < 4; j++)
    if (!fr[j]) d[j] = dbind[j];
  double mx = 0;
  for (int j = 0; j < 4; j++)
    if (fabs(d[j]) > mx) mx = fabs(d[j]);
  if (mx > 4.0)
    for (int j = 0; j < 4; j++) d[j] *= 4.0 / mx;
  return mu > 0.0 || !ok;
}

/* a direction of non-positive curvature of the free block of H (the saddle
 * escape of fit_one): the unshifted Cholesky's first non-positive pivot s_j
 * with the computed rows above it gives z = (-L^-T l, 1, 0..), z'Hz = s_j <= 0;
 * scaled to max-norm 1 and signed downhill.  Returns 0 if H is positive
 * definite on the free set. */
static int nc_direction(int model, const double u[4], const double g[4], double H[4][4], double v[4]) {
  int fr[4];
  double dbind[4], L[4][4] = {{0}};
  free_set(model, u, g, H, fr, dbind);
  int jf = -1;
  for (int j = 0; j < 4 && jf < 0; j++) {
    for (int m = 0; m <= j; m++) {
      double s = (!fr[j] || !fr[m]) ? (j == m ? 1.0 : 0.0) : H[j][m];
      for (int p = 0; p < m; p++) s -= L[j][p] * L[m][p];
      if (j == m) {
        if (!(s > 0)) {
          jf = j;
          break;
        }
        L[j][j] = sqrt(s);
      } else {
        L[j][m] = s / L[m][m];
      }
    }
  }
  if (jf < 0) return 0;
  double z[4] = {0, 0, 0, 0};
  z[jf] = 1.0;
  for (int p = jf - 1; p >= 0; p--) {
    double s = 0;
    for (int k = p + 1; k <= jf; k++) s += L[k][p] * z[k];
    z[p] = -s / L[p][p];
  }
  const double mx = maxabs4(z);
  double gz = 0;
  for (int j = 0; j < 4; j++) gz += g[j] * z[j];
  const double sg = gz > 0 ? -1.0 : 1.0;
  for (int j = 0; j < 4; j++) v[j] = sg * z[j] / mx;
  return 1;
}

/* projected-gradient size max_j |u_j - clamp(u_j - g_j)|: the stationarity
 * measure of a box-constrained problem (0 for a variable held on its bound) */
static double pgnorm(const double u[4], const double g[4]) {
  double m = 0;
  for (int j = 0; j < 4; j++) {
    double v = fabs(u[j] - clampd(u[j] - g[j], U_LO[j], U_HI[j]));
    if (v > m) m = v;
  }
  return m;
}

/* the projected-gradient direction P(u - g) - u scaled to max-norm 1 (the
 * gradient fallback below); 0 when the projected gradient vanishes */
static int pg_direction(const double u[4], const double g[4], double v[4]) {
  double p[4];
  for (int j = 0; j < 4; j++) p[j] = clampd(u[j] - g[j], U_LO[j], U_HI[j]) - u[j];
  const double mx = maxabs4(p);
  if (!(mx > 0)) return 0;
  for (int j = 0; j < 4; j++) v[j] = p[j] / mx;
  return 1;
}


typedef struct {
  double u[4];
  evalres r;
  int evals;
  int status;
  int polished; /* the fit entered the polish phase */
} fitres;

#include <stdio.h>
static int g_trace = 0; /* debugging aid: print every evaluation of fit_one */
void oracle_set_trace(int on) { g_trace = on; }

/* u0 == NULL: the data-driven initial point (init_u); else start at u0 */
static void fit_one(int model, const uint32_t* y, const uint32_t* N, int lo,
                    int hi, int max_iter, double tol, const double* u0, fitres* out) {
  double u[4], d[4], ut[4], t = 1.0;
  evalres cur, tr;
  if (u0) memcpy(u, u0, sizeof(u));
  else init_u(model, y, N, lo, hi, u);
  int accf = 0; /* the polish phase (below): F in the cancellation-free form */
  evaluate(model, y, N, lo, hi, u, &cur, accf);
  int evals = 1, status = MDFIT_MAXITER;
  if (!isfinite(cur.F)) {
    status = MDFIT_NONFINITE;
    goto done;
  }
  int indef = direction(model, u, cur.g, cur.H, d);
  if (maxabs4(d) <= tol) {
    status = MDFIT_OK;
    goto done;
  }
  int rescued = 0, relax = 0; /* the flat-tail rescue (below): once per fit */
  int nc = 0, n_nc = 0, st_exh = MDFIT_MAXITER; /* the saddle escape (below) */
  int grad = 0, n_grad = 0;                       /* the gradient fallback (below): up to 8 times per fit */
  while (evals < max_iter) {
    for (int j = 0; j < 4; j++) ut[j] = clampd(u[j] + t * d[j], U_LO[j], U_HI[j]);
    evaluate(model, y, N, lo, hi, ut, &tr, accf);
    evals++;
    /* (in the polish phase mag is the sum of the |R| terms of the cancellation-free form) */
    const double noise = NOISE_F * (cur.mag + fabs(cur.F));
    const int was_relax = relax;
    int acc = isfinite(tr.F) &&
              (nc ? tr.F < cur.F - noise
                  : (tr.F < cur.F ||
                     (tr.F <= cur.F + noise && (relax || pgnorm(ut, tr.g) < pgnorm(u, cur.g)))));
    relax = 0;
    if (g_trace)
      printf("%d trF=%.12f curF=%.12f acc=%d t=%.3g |d|=%.3e |gt|=%.3e |gc|=%.3e u=[%.10f %.10f %.10f %.10f] d=[%.3e %.3e %.3e %.3e]\n",
             evals, tr.F, cur.F, acc, t, maxabs4(d), maxabs4(tr.g), maxabs4(cur.g), u[0], u[1], u[2], u[3], d[0], d[1], d[2], d[3]);
    if (acc) {
      /* the step just taken: a full Newton step (not a backtracked, escape,
       * gradient-fallback or flat-tail-rescue step), and its size */
      const int newton_step = !nc && !grad && !was_relax && t == 1.0;
      const double dprev = t * maxabs4(d);
      memcpy(u, ut, sizeof(u));
      cur = tr;
      indef = direction(model, u, cur.g, cur.H, d);
      nc = grad = 0;
      t = 1.0;
      const double dn = maxabs4(d);
      if (dn <= tol) {
        status = MDFIT_OK;
        break;
      }
      /* MDFIT-MAP v1.1: converged by quadratic contraction.  After a full Newton
       * step, a positive-definite Newton system whose next step satisfies
       * QUAD_K |d|^2 <= tol and |d| <= QUAD_K |d_prev|^2 (the quadratic regime
       * observed) is taken WITHOUT evaluating its end point: the error left
       * after it is O(|d|^2) <= tol, what the |d| <= tol stop would have
       * confirmed with one more evaluation (~0.8 evaluations per sub-fit). */
      if (newton_step && !indef && QUAD_K * dn * dn <= tol && dn <= QUAD_K * dprev * dprev) {
        for (int j = 0; j < 4; j++) u[j] = clampd(u[j] + d[j], U_LO[j], U_HI[j]);
        status = MDFIT_OK;
        break;
      }
    } else if (nc) { /* the escape step finds no decrease beyond F's rounding */
      t *= 0.5;
      if (t < (grad ? 1e-6 : 1e-3)) {
        /* no decrease beyond F's rounding along the projected gradient either,
         * for steps down to 1e-6: optimal to F's resolution (the boundary fits
         * at c -> 0 whose curvature in c grows by ~1e7 within 1e-6 of the bound) */
        if (grad) {
          status = MDFIT_OK;
          break;
        }
        /* the gradient fallback: a fit that ends here unconverged (an escape
         * direction or the Newton step pushing a variable that sits on its
         * bound outward, while the gradient pulls it inward -- every clamped
         * trial then raises F) tries (up to 8 times per fit) the projected-gradient direction
         * P(u - g) - u, re-evaluating at u first as the kernel does, with the
         * escape's strict acceptance, halving to 1e-6 */
        if (st_exh != MDFIT_OK && n_grad < 8 && evals < max_iter) {
          evaluate(model, y, N, lo, hi, u, &tr, accf);
          evals++;
          n_grad++;
          if (pg_direction(u, tr.g, d)) {
            grad = 1;
            t = 1.0;
            continue;
          }
        }
        status = st_exh;
        break;
      }
    } else {
      t *= 0.5;
      /* the polish phase: once the backtracking step's predicted decrease
       * t |g.d| is below F's rounding scale (the sum of ~N ln N-sized lnGamma
       * values), F can no longer judge the trials -- in a flat valley the
       * stopping point would depend on the rounding path.  Once per fit:
       * re-evaluate at u with F in the cancellation-free form (an evaluation;
       * same g, H, hence the same d) and restart the line search at t = 1; the
       * fit keeps that form to its end. */
      double gdc = 0;
      for (int j = 0; j < 4; j++) gdc += cur.g[j] * d[j];
      const int unresolved = t * fabs(gdc) <= noise;
      if (!accf && evals < max_iter && (t < 1e-12 || unresolved)) {
        accf = 1;
        evaluate(model, y, N, lo, hi, u, &cur, accf);
        evals++;
        indef = direction(model, u, cur.g, cur.H, d);
        t = 1.0;
        continue;
      }
      /* exhausted: t below 1e-12, or (polish phase) the predicted decrease
       * below even the cancellation-free F's rounding -- where noise-level
       * "decreases" would otherwise be accepted at ever smaller steps (a saddle
       * whose shifted Newton step is ~0 then never exhausts the search) */
      if (t < 1e-12 || (accf && unresolved)) { /* line search exhausted */
        /* the flat tail of log delta (phi -> 2): the Newton step heads down a
         * tail in which F changes below its rounding scale, so the stopping
         * point would depend on the rounding path.  Once per fit: jump log delta
         * onto its lower bound (the limit of that walk; accepted within F's
         * rounding scale) and continue from there. */
        if (!rescued && u[P_D] < 0.0 && d[P_D] < 0.0 && u[P_D] > U_LO[P_D]) {
          rescued = relax = 1;
          for (int j = 0; j < 4; j++) d[j] = j == P_D ? U_LO[P_D] - u[P_D] : 0.0;
          t = 1.0;
          continue;
        }
        /* numerically at the optimum when the step, the projected gradient or
         * the step's predicted decrease |g.d| is below F's resolution */
        double gd = 0;
        for (int j = 0; j < 4; j++) gd += cur.g[j] * d[j];
        st_exh = (maxabs4(d) <= 1e-5 || pgnorm(u, cur.g) <= PG_TOL || fabs(gd) <= noise) ? MDFIT_OK : MDFIT_MAXITER;
        /* the saddle escape: at a point whose Hessian is indefinite on the free
         * set (flat valleys of q, A, c), the shifted Newton step is ~0 and the
         * line search stalls although F still falls along the negative
         * curvature.  Up to 4 times per fit: re-evaluate at u (an evaluation,
         * as the kernel does: it keeps no H), step along nc_direction from t = 1
         * halving to 1e-3, accepting only a decrease beyond F's rounding. */
        if (indef && n_nc < 4 && evals < max_iter) {
          evaluate(model, y, N, lo, hi, u, &tr, accf);
          evals++;
          if (nc_direction(model, u, tr.g, tr.H, d)) {
            n_nc++;
            nc = 1;
            t = 1.0;
            continue;
          }
        }
        if (st_exh != MDFIT_OK && n_grad < 8 && evals < max_iter) { /* the gradient fallback (above) */
          evaluate(model, y, N, lo, hi, u, &tr, accf);
          evals++;
          n_grad++;
          if (pg_direction(u, tr.g, d)) {
            nc = grad = 1;
            t = 1.0;
            continue;
          }
        }
        status = st_exh;
        break;
      }
    }
  }
done:
  memcpy(out->u, u, sizeof(u));
  out->r = cur;
  out->evals = evals;
  out->status = status;
  out->polished = accf;
}

/* ---- pointwise log-likelihood at a mode (fits.py:126-133) -----------------
 * The record's WAIC statistics use the full beta-binomial log-pmf (numpyro's
 * log_likelihood, log C(N,y) included), computed in long double as
 *   R(y, a) + R(N-y, b) - R(N, phi),  R(n, s) = lnG(n+s) - lnG(n+1) - lnG(s),
 * where each R is formed without subtracting two large lnGamma values and
 * without rounding a sum like n + s (at n ~ 2e9 one ulp of the argument moves
 * lnGamma by ~5e-6): lnG(z + h) - lnG(z) for z, z + h >= 8 is the difference
 * of the Stirling expansions taken term by term -- the leading terms as
 * (z - 1/2 + h) log1p(h/z) + h (ln z - 1), then the Bernoulli series
 * B_2k/(2k(2k-1) x^(2k-1)) to k = 9.  The plain sum of lnGamma values (~1e11
 * at N = 4e9) would carry ~1e-5 absolute error into an O(10) result.
 * (Restated from the math, not from the kernel; the kernel's bb_logpmf is
 * the same decomposition in double.)  Checked against mpmath at 40 digits
 * (tests/test_oracle_golden.py). */
static long double lgdiff_l(long double z, long double h) {
  if (z >= 8.0L && z + h >= 8.0L) {
    static const long double bern[9] = {1.0L / 12, -1.0L / 360, 1.0L / 1260, -1.0L / 1680, 1.0L / 1188,
                                        -691.0L / 360360, 1.0L / 156, -3617.0L / 122400,
                                        43867.0L / 244188};
    long double t = log1pl(h / z);
    long double s = (z - 0.5L + h) * t + h * (logl(z) - 1.0L);
    long double r1 = 1.0L / (z + h), r2 = 1.0L / z, p1 = r1, p2 = r2;
    for (int k = 0; k < 9; k++) {
      s += bern[k] * (p1 - p2);
      p1 *= r1 * r1;
      p2 *= r2 * r2;
    }
    return s;
  }
  return o_lgammal(z + h) - o_lgammal(z);
}

static long double lrise_l(long double n, long double s) {
  if (n == 0.0L) return 0.0L;
  return s <= n + 1.0L ? lgdiff_l(n + 1.0L, s - 1.0L) - o_lgammal(s) : lgdiff_l(s, n) - o_lgammal(n + 1.0L);
}

static double bb_logpmf_full(double y, double N, double D, double phi) {
  long double a = (long double)D * phi, b = (1.0L - (long double)D) * phi;
  return (double)(lrise_l(y, a) + lrise_l(N - y, b) - lrise_l(N, phi));
}

/* the full pointwise log-pmf of sub-fit points [lo, hi) at its mode u */
static void mode_ell(int model, const uint32_t* y, const uint32_t* N, int lo, int hi,
                     const double u[4], double* ell) {
  double q = sigm(u[P_Q]), phi = exp(u[P_D]) + 2.0;
  double A = model == M_PMD ? sigm(u[P_A]) : 0.0, c = model == M_PMD ? u[P_C] : 0.0;
  for (int i = lo; i < hi; i++) {
    double D = model == M_PMD ? A * pow(1.0 - q, kpos(i)) + c : q;
    ell[i] = bb_logpmf_full((double)y[i], (double)N[i], D, phi);
  }
}

/* the same on arrays (alpha, beta given: phi = alpha + beta), for tests */
void oracle_bb_logpmf_full(const double* y, const double* N, const double* a, const double* b, int64_t n,
                           double* out) {
  for (int64_t i = 0; i < n; i++)
    out[i] = (double)(lrise_l(y[i], a[i]) + lrise_l(N[i] - y[i], b[i]) - lrise_l(N[i], (long double)(a[i] + b[i])));
}

/* n_sigma of fits.py:194-201 with one posterior "sample" (the mode):
 * lppd_i = ell_i, pWAIC_i = 0, waic_i = -2 ell_i (fits.py:147-172) */
static double n_sigma(const double* lP, const double* lN, int n) {
  double d[NPOS], md = 0, wP = 0, wN = 0;
  for (int i = 0; i < n; i++) {
    d[i] = (-2.0 * lP[i]) - (-2.0 * lN[i]);
    md += d[i];
    wP += -2.0 * lP[i];
    wN += -2.0 * lN[i];
  }
  md /= n;
  double v = 0;
  for (int i = 0; i < n; i++) v += (d[i] - md) * (d[i] - md);
  v /= n;
  return (wN - wP) / sqrt(n * v);
}

/* compute_assymmetry_combined_vs_forwardreverse, fits.py:204-227 */
static double asymmetry(const double* lC, const double* lF, const double* lR) {
  double d[NPOS], md = 0, wC = 0, wFR = 0;
  for (int i = 0; i < NPOS; i++) {
    double fr = (i < NHALF) ? lF[i] : lR[i];
    d[i] = (-2.0 * lC[i]) - (-2.0 * fr);
    md += d[i];
    wC += -2.0 * lC[i];
    wFR += -2.0 * fr;
  }
  md /= NPOS;
  double v = 0;
  for (int i = 0; i < NPOS; i++) v += (d[i] - md) * (d[i] - md);
  v /= NPOS;
  return (wFR - wC) / sqrt(NPOS * v);
}

/* add_noise_estimates, fits.py:359-376: columns AC AG AT CA CG CT GA GC GT TA TC TG */
static void noise(const uint32_t* mm, double out3[3]) {
  double X[NPOS][12];
  int valid[NPOS][12];
  for (int j = 0; j < 12; j++) {
    double s = 0;
    int cnt = 0;
    for (int i = 0; i < NPOS; i++) {
      int nanned = (j == 5 && i < NHALF) || (j == 6 && i >= NHALF);
      valid[i][j] = !nanned;
      if (!nanned) {
        s += mm[i * 12 + j];
        cnt++;
      }
    }
    double m = s / cnt;
    for (int i = 0; i < NPOS; i++) {
      X[i][j] = mm[i * 12 + j] / m;
      if (valid[i][j] && isnan(X[i][j])) valid[i][j] = 0;
    }
  }
  int ranges[3][2] = {{0, NPOS}, {0, NHALF}, {NHALF, NPOS}};
  for (int r = 0; r < 3; r++) {
    double s = 0;
    int cnt = 0;
    for (int i = ranges[r][0]; i < ranges[r][1]; i++)
      for (int j = 0; j < 12; j++)
        if (valid[i][j]) {
          s += X[i][j];
          cnt++;
        }
    if (cnt == 0) {
      out3[r] = NAN;
      continue;
    }
    double mean = s / cnt, v = 0;
    for (int i = ranges[r][0]; i < ranges[r][1]; i++)
      for (int j = 0; j < 12; j++)
        if (valid[i][j]) v += (X[i][j] - mean) * (X[i][j] - mean);
    out3[r] = sqrt(v / cnt);
  }
}

#include "mdfit_hpdi.c"

/* MAP predictive summary at point i (fits.py:112-120 with the mode as the one
 * posterior sample): median := D(z); HPDI := the 68 % window [lo, hi] / N of
 * BetaBinomial(D phi, (1-D) phi, N) (MDFIT-HPDI v2, mdfit_hpdi.c); NaN when
 * N = 0 (the reference divides 0 draws by N = 0, fits.py:115).  want_hpdi = 0:
 * the median only (D_max_forward / _reverse). */
/* tests may switch the HPDI off (oracle_set_hpdi(0)) to check the other
 * columns of a large batch quickly; the HPDI columns are then NaN */
static int g_hpdi_on = 1;
void oracle_set_hpdi(int on) { g_hpdi_on = on != 0; }

static void predict(double A, double q, double c, double phi, int k, double N,
                    double o[3], int want_hpdi) {
  if (N == 0) {
    o[0] = o[1] = o[2] = NAN;
    return;
  }
  double D = A * pow(1.0 - q, k) + c;
  if (D > 1.0) D = 1.0;
  o[0] = D;
  o[1] = o[2] = NAN;
  if (want_hpdi && g_hpdi_on) {
    double lo, hi;
    hp_window(N, D * phi, (1.0 - D) * phi, &lo, &hi);
    o[1] = lo / N;
    o[2] = hi / N;
  }
}

static void fit_taxon(const uint32_t* y, const uint32_t* N, const uint32_t* mm,
                      const mdfit_opts* o, double* out, float* pred, int32_t* status) {
  for (int j = 0; j < MDFIT_NOUT; j++) out[j] = 0.0;
  for (int i = 0; i < NPOS; i++)
    if (y[i] > N[i]) {
      for (int j = 0; j < MDFIT_NOUT; j++) out[j] = NAN;
      if (pred)
        for (int j = 0; j < 3 * NPOS; j++) pred[j] = NAN;
      *status = MDFIT_INVALID;
      return;
    }
  static const int models[6] = {M_PMD, M_NULL, M_PMD, M_PMD, M_NULL, M_NULL};
  static const int los[6] = {0, 0, 0, NHALF, 0, NHALF};
  static const int his[6] = {NPOS, NPOS, NHALF, NPOS, NHALF, NPOS};
  fitres f[6];
  int st = MDFIT_OK;
  for (int s = 0; s < 6; s++) {
    /* MDFIT-MAP v1 warm start: the forward / reverse sub-fits start from the
     * all-position mode of the same model when that fit converged */
    const double* u0 = NULL;
    if (s >= 2) {
      const fitres* base = &f[models[s] == M_PMD ? 0 : 1];
      if (base->status == MDFIT_OK) u0 = base->u;
    }
    fit_one(models[s], y, N, los[s], his[s], o->max_iter, o->tol_step, u0, &f[s]);
    if (f[s].status > st) st = f[s].status;
    double* dg = out + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * s;
    dg[0] = sigm(f[s].u[P_Q]);
    dg[1] = models[s] == M_PMD ? sigm(f[s].u[P_A]) : 0.0;
    dg[2] = models[s] == M_PMD ? f[s].u[P_C] : 0.0;
    dg[3] = exp(f[s].u[P_D]) + 2.0;
    dg[4] = f[s].r.F;
    dg[5] = f[s].evals;
    dg[6] = f[s].status;
    dg[7] = f[s].polished;
  }
  double p[3];
  /* PMD-all: predictions + D_max (fits.py:249-261: median / HPDI at z = +1) */
  double qa = out[MDFIT_F_DIAG + 0], Aa = out[MDFIT_F_DIAG + 1];
  double ca = out[MDFIT_F_DIAG + 2], pa = out[MDFIT_F_DIAG + 3];
  for (int i = 0; i < NPOS; i++) {
    predict(Aa, qa, ca, pa, kpos(i), (double)N[i], p, 1);
    if (pred)
      for (int r = 0; r < 3; r++) pred[r * NPOS + i] = (float)p[r];
    if (i == 0) {
      out[MDFIT_F_D_MAX] = p[0];
      out[MDFIT_F_D_MAX_LOWER_HPDI] = p[1];
      out[MDFIT_F_D_MAX_UPPER_HPDI] = p[2];
    }
  }
  /* pointwise full log-pmf of every sub-fit at its mode (the WAIC inputs) */
  double ell[6][NPOS];
  for (int s = 0; s < 6; s++) mode_ell(models[s], y, N, los[s], his[s], f[s].u, ell[s]);
  out[MDFIT_F_N_SIGMA] = n_sigma(ell[0], ell[1], NPOS);
  out[MDFIT_F_Q_MEAN] = qa;
  out[MDFIT_F_CONCENTRATION_MEAN] = pa;
  out[MDFIT_F_D_MAX_MARGINALIZED_MEAN] = Aa + ca;
  double nf = 0, nr = 0, yf = 0, yr = 0;
  for (int i = 0; i < NHALF; i++) {
    nf += N[i];
    yf += y[i];
    nr += N[NHALF + i];
    yr += y[NHALF + i];
  }
  out[MDFIT_F_N_Z1_FORWARD] = N[0];
  out[MDFIT_F_N_Z1_REVERSE] = N[NHALF];
  out[MDFIT_F_N_SUM_FORWARD] = nf;
  out[MDFIT_F_N_SUM_REVERSE] = nr;
  out[MDFIT_F_N_SUM_TOTAL] = nf + nr;
  out[MDFIT_F_Y_SUM_FORWARD] = yf;
  out[MDFIT_F_Y_SUM_REVERSE] = yr;
  out[MDFIT_F_Y_SUM_TOTAL] = yf + yr;
  /* forward (fits.py:311-329) */
  out[MDFIT_F_N_SIGMA_FORWARD] = n_sigma(ell[2], ell[4], NHALF);
  {
    const double* dg = out + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * 2;
    predict(dg[1], dg[0], dg[2], dg[3], 0, (double)N[0], p, 0);
    out[MDFIT_F_D_MAX_FORWARD] = p[0];
    out[MDFIT_F_Q_MEAN_FORWARD] = dg[0];
  }
  /* reverse (fits.py:333-350); D_max_reverse evaluated on data_forward (:343-348) */
  out[MDFIT_F_N_SIGMA_REVERSE] =
      n_sigma(ell[3] + NHALF, ell[5] + NHALF, NHALF);
  {
    const double* dg = out + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * 3;
    predict(dg[1], dg[0], dg[2], dg[3], 0, (double)N[0], p, 0);
    out[MDFIT_F_D_MAX_REVERSE] = p[0];
    out[MDFIT_F_Q_MEAN_REVERSE] = dg[0];
  }
  out[MDFIT_F_ASYMMETRY] = asymmetry(ell[0], ell[2], ell[3]);
  if (mm) {
    double nz[3];
    noise(mm, nz);
    out[MDFIT_F_NORMALIZED_NOISE] = nz[0];
    out[MDFIT_F_NORMALIZED_NOISE_FORWARD] = nz[1];
    out[MDFIT_F_NORMALIZED_NOISE_REVERSE] = nz[2];
  } else {
    out[MDFIT_F_NORMALIZED_NOISE] = out[MDFIT_F_NORMALIZED_NOISE_FORWARD] =
        out[MDFIT_F_NORMALIZED_NOISE_REVERSE] = NAN;
  }
  *status = st;
}

/* Host-pointer batch fit: same layout as mdfit_fit_batch.  OpenMP over taxa;
 * n_threads <= 0 -> OpenMP default. */
int oracle_fit_batch(const uint32_t* y, const uint32_t* N, const uint32_t* mm,
                     int64_t n_taxa, const mdfit_opts* opts, double* out,
                     float* pred, int32_t* status, int n_threads) {
  mdfit_opts o;
  memset(&o, 0, sizeof(o));
  o.max_iter = 200;
  o.tol_step = 1e-9;
  if (opts) o = *opts;
#ifdef _OPENMP
  int nt = n_threads > 0 ? n_threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 4) num_threads(nt)
#endif
  for (int64_t t = 0; t < n_taxa; t++) {
    fit_taxon(y + t * MDFIT_LD, N + t * MDFIT_LD,
              mm ? mm + t * NPOS * MDFIT_NMM : NULL, &o, out + t * MDFIT_NOUT,
              pred ? pred + t * MDFIT_NPRED * NPOS : NULL, status + t);
  }
  return 0;
}

/* Objective / gradient / Hessian at u for one sub-fit (scipy cross-checks).
 * model 0 = PMD, 1 = null; subset 0 = all, 1 = fwd, 2 = rev. */
void oracle_objective(int model, int subset, const uint32_t* y, const uint32_t* N,
                      const double* u, double* F, double* g4, double* H16,
                      double* ell30) {
  int lo = subset == 2 ? NHALF : 0, hi = subset == 1 ? NHALF : NPOS;
  evalres r;
  memset(&r, 0, sizeof(r));
  evaluate(model, y, N, lo, hi, u, &r, 0);
  *F = r.F;
  for (int j = 0; j < 4; j++) {
    g4[j] = r.g[j];
    for (int m = 0; m < 4; m++) H16[4 * j + m] = r.H[j][m];
  }
  if (ell30)
    for (int i = 0; i < NPOS; i++) ell30[i] = (i >= lo && i < hi) ? r.ell[i] : 0.0;
}

/* One sub-fit from u0 (NULL: the spec's initial point); returns u*, F*, evals, status. */
void oracle_fit_subfit(int model, int subset, const uint32_t* y, const uint32_t* N,
                       int max_iter, double tol, const double* u0, double* u4, double* F,
                       int32_t* evals, int32_t* status) {
  int lo = subset == 2 ? NHALF : 0, hi = subset == 1 ? NHALF : NPOS;
  fitres f;
  fit_one(model, y, N, lo, hi, max_iter, tol, u0, &f);
  for (int j = 0; j < 4; j++) u4[j] = f.u[j];
  *F = f.r.F;
  *evals = f.evals;
  *status = f.status;
}

/* Initial point of the spec (for tests). */
void oracle_init_u(int model, int subset, const uint32_t* y, const uint32_t* N, double* u4) {
  int lo = subset == 2 ? NHALF : 0, hi = subset == 1 ? NHALF : NPOS;
  init_u(model, y, N, lo, hi, u4);
}

/* the sampling mode (MDFIT-NUTS v1) */
#include "mdfit_nuts.c"
