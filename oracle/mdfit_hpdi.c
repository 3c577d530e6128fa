/*
 * mdfit_hpdi.c — CPU ORACLE (test infrastructure only; included by
 * mdfit_oracle.c).
 *
 * MDFIT-HPDI v1: the 68 % highest-probability window of the MAP predictive
 * BetaBinomial(alpha, beta, N) -- the MAP counterpart of the
 * reference's numpyro.diagnostics.hpdi(obs / N, prob=0.68) over the predictive
 * draws (/root/reference/metadamage/fits.py:112-120, :260-261), whose
 * population limit is the shortest window holding 68 % of the mass.
 *
 * Definition.  The pmf is unimodal (phi = alpha + beta > 2: the sign of
 * p(y+1) - p(y) is that of (alpha-1)(N-y) - (beta-1)(y+1), linear in y), so the
 * shortest 68 % window is grown greedily: start at the mode, add the more
 * probable neighbour (a tie adds the lower one) until the window holds >= 0.68.
 * The result is the integer window [lo, hi]; the reported bounds are lo/N, hi/N.
 *
 * Two ways to the same window:
 *   hp_greedy  -- the definition, point by point (p(y+1) = p(y) R(y));
 *   hp_window  -- the spec the kernel implements: the greedy when the
 *                 predictive sd is <= 100 points (or the mode alone holds 68 %),
 *                 otherwise a Newton iteration on the level set
 *                 {y : ln p(y) >= ln p(m) + t} (two-sided), or on the window end
 *                 when the window is clamped at 0 or N (one-sided), with the
 *                 window mass from Euler-Maclaurin (exact sums within 16 points
 *                 of the support ends, 6-point Gauss-Legendre panels of the
 *                 continuous pmf in x or, near a support end, in ln(x + alpha)
 *                 / ln(N - x + beta)); then a point-by-point fix-up of the
 *                 window from that mass: add the more probable neighbour while
 *                 the mass is < 0.68, drop the less probable end while the rest
 *                 still holds 0.68 (exactly the greedy's stopping rule).
 * The oracle evaluates ln p with long-double lgammal; the kernel with the
 * cancellation-free lnGamma differences of mdfit_special.h.
 */

#define HP_MASS 0.68
#ifndef HP_SIG_GREEDY
#define HP_SIG_GREEDY 100.0 /* sd (counts) up to which the greedy itself runs */
#endif
#define HP_T0 (-0.49447329849) /* -Z68^2 / 2: the Gaussian 68 % level */
#define HP_K0 16               /* exact sums this close to a support end */
#define HP_LV 4.0              /* max panel length in a log variable */
#define HP_LX 2.5              /* max linear panel length, in units of sd */
#define HP_STOP 16.0           /* Newton stops when the ends would move < this (counts): the
                                * exact fix-up walk (~20 instructions a count) finishes */

static const double HP_GLX[3] = {0.2386191860831969, 0.6612093864662645, 0.9324695142031521};
static const double HP_GLW[3] = {0.4679139345726910, 0.3607615730481386, 0.1713244923791704};

typedef struct {
  double N, a, b, m;
  double pm; /* p(m) */
} hpd_t;

/* p(y+1) / p(y) */
static long double hp_R(const hpd_t* P, double y) {
  return ((long double)(P->N - y) * (y + P->a)) / ((long double)(y + 1.0) * (P->N - y - 1.0 + P->b));
}

/* ln p(x) - ln p(m) of the continuous extension (long double lgamma) */
static double hp_g(const hpd_t* P, double x) {
  long double N = P->N, a = P->a, b = P->b, m = P->m, X = x;
  long double r = (o_lgammal(X + a) - o_lgammal(m + a)) - (o_lgammal(X + 1.0L) - o_lgammal(m + 1.0L)) +
                  (o_lgammal(N - X + b) - o_lgammal(N - m + b)) - (o_lgammal(N - X + 1.0L) - o_lgammal(N - m + 1.0L));
  return (double)r;
}

/* d/dx ln p(x) */
static double hp_s(const hpd_t* P, double x) {
  return o_digamma(x + P->a) - o_digamma(x + 1.0) - o_digamma(P->N - x + P->b) + o_digamma(P->N - x + 1.0);
}

static double hp_f(const hpd_t* P, double x) { return exp(hp_g(P, x)); } /* p(x) / p(m) */

static double hp_mode(double N, double a, double b) {
  double y0 = ((a - 1.0) * N - (b - 1.0)) / (a + b - 2.0);
  double m = ceil(y0);
  return m < 0.0 ? 0.0 : (m > N ? N : m);
}

/* the definition: greedy from the mode */
static void hp_greedy(const hpd_t* P, double* lo, double* hi) {
  double A = P->m, B = P->m, N = P->N;
  long double pm = P->pm, M = pm;
  long double pl = A > 0 ? pm / hp_R(P, A - 1) : 0.0L;
  long double pr = B < N ? pm * hp_R(P, B) : 0.0L;
  while (M < HP_MASS && (pl > 0 || pr > 0)) {
    if (pl >= pr) {
      A -= 1;
      M += pl;
      pl = A > 0 ? pl / hp_R(P, A - 1) : 0.0L;
    } else {
      B += 1;
      M += pr;
      pr = B < N ? pr * hp_R(P, B) : 0.0L;
    }
  }
  *lo = A;
  *hi = B;
}

/* sum_{y=A}^{B} p(y)/p(m) by the recurrence */
static double hp_exact_sum(const hpd_t* P, double A, double B) {
  long double v = hp_f(P, A), s = 0.0L;
  for (double y = A; y <= B; y += 1.0) {
    s += v;
    if (y < B) v *= hp_R(P, y);
  }
  return (double)s;
}

/* int_{u0}^{u1} p(x)/p(m) dx over one part with a fixed variable */
static double hp_part(const hpd_t* P, double u0, double u1, double sd) {
  const double N = P->N, a = P->a, b = P->b;
  const double L = u1 - u0;
  const int nl = (u0 + a) < L, nr = (N - u1 + b) < L;
  if (nl && nr) {
    const double c = 0.5 * (u0 + u1);
    return hp_part(P, u0, c, sd) + hp_part(P, c, u1, sd);
  }
  double I = 0.0;
  if (nl || nr) {
    const double v0 = nl ? log(u0 + a) : log(N - u1 + b);
    const double v1 = nl ? log(u1 + a) : log(N - u0 + b);
    int k = (int)ceil((v1 - v0) / HP_LV);
    if (k < 1) k = 1;
    for (int j = 0; j < k; j++) {
      const double w0 = v0 + (v1 - v0) * j / k, w1 = v0 + (v1 - v0) * (j + 1) / k;
      const double h = 0.5 * (w1 - w0), c = 0.5 * (w1 + w0);
      for (int i = 0; i < 6; i++) {
        const double v = c + h * (i < 3 ? -HP_GLX[2 - i] : HP_GLX[i - 3]);
        const double wgt = HP_GLW[i < 3 ? 2 - i : i - 3];
        const double ev = exp(v);
        const double x = nl ? ev - a : N + b - ev;
        I += wgt * h * hp_f(P, x) * ev;
      }
    }
  } else {
    int k = (int)ceil(L / (HP_LX * sd));
    if (k < 1) k = 1;
    for (int j = 0; j < k; j++) {
      const double w0 = u0 + L * j / k, w1 = u0 + L * (j + 1) / k;
      const double h = 0.5 * (w1 - w0), c = 0.5 * (w1 + w0);
      for (int i = 0; i < 6; i++) {
        const double x = c + h * (i < 3 ? -HP_GLX[2 - i] : HP_GLX[i - 3]);
        I += HP_GLW[i < 3 ? 2 - i : i - 3] * h * hp_f(P, x);
      }
    }
  }
  return I;
}

/* sum_{y=A}^{B} p(y)/p(m): exact within HP_K0 of the support ends and for
 * short windows, Euler-Maclaurin elsewhere (integral split at the mode +
 * (f(A)+f(B))/2 + (f'(B)-f'(A))/12) */
static double hp_mass(const hpd_t* P, double A, double B, double sd) {
  const double N = P->N;
  double tot = 0.0, A1 = A, B1 = B;
  if (A1 < HP_K0) {
    const double e = fmin(HP_K0 - 1, B);
    tot += hp_exact_sum(P, A1, e);
    A1 = e + 1;
  }
  if (B1 > N - HP_K0 && B1 >= A1) {
    const double s0 = fmax(N - HP_K0 + 1, A1);
    tot += hp_exact_sum(P, s0, B1);
    B1 = s0 - 1;
  }
  if (B1 < A1) return tot;
  if (B1 - A1 < 32) return tot + hp_exact_sum(P, A1, B1);
  const double c = fmin(fmax(P->m, A1), B1);
  double I = 0.0;
  if (c > A1) I += hp_part(P, A1, c, sd);
  if (B1 > c) I += hp_part(P, c, B1, sd);
  const double fA = hp_f(P, A1), fB = hp_f(P, B1);
  const double dA = fA * hp_s(P, A1), dB = fB * hp_s(P, B1);
  return tot + I + 0.5 * (fA + fB) + (dB - dA) / 12.0;
}

/* x in [lo, hi] with g(x) = t (g monotone there; rising = g - t < 0 at lo):
 * safeguarded Newton */
static double hp_root(const hpd_t* P, double t, double lo, double hi, double x0, int rising) {
  double x = fmin(fmax(x0, lo), hi);
  for (int it = 0; it < 60; it++) {
    const double gx = hp_g(P, x) - t;
    if (fabs(gx) < 1e-12) return x;
    if ((gx < 0) == (rising != 0)) lo = x;
    else hi = x;
    const double sx = hp_s(P, x);
    double xn = sx != 0.0 ? x - gx / sx : 0.5 * (lo + hi);
    if (!(lo < xn && xn < hi)) xn = 0.5 * (lo + hi);
    if (fabs(xn - x) < 0.05) return xn;
    x = xn;
  }
  return x;
}

/* window [A, B] holding mass M (absolute) -> the greedy's window */
static void hp_fixup(const hpd_t* P, double A, double B, long double M, double* lo, double* hi) {
  const double N = P->N;
  long double pA = (long double)hp_f(P, A) * P->pm;
  long double pB = B != A ? (long double)hp_f(P, B) * P->pm : pA;
  long double pl = A > 0 ? pA / hp_R(P, A - 1) : 0.0L;
  long double pr = B < N ? pB * hp_R(P, B) : 0.0L;
  while (M < HP_MASS && (pl > 0 || pr > 0)) {
    if (pl >= pr) {
      A -= 1;
      M += pl;
      pA = pl;
      pl = A > 0 ? pl / hp_R(P, A - 1) : 0.0L;
    } else {
      B += 1;
      M += pr;
      pB = pr;
      pr = B < N ? pr * hp_R(P, B) : 0.0L;
    }
  }
  /* then: drop the less probable end while the rest holds the mass (a tie:
   * the upper end, which the greedy adds last); when it cannot be dropped
   * but a neighbour outside is more probable than it (the window is not a
   * level set -- a nearly flat pmf), add that neighbour: the next pass drops
   * the end, so the window slides toward the level set */
  for (;;) {
    const long double pe = pB <= pA ? pB : pA;
    if (A < B && M - pe >= HP_MASS) {
      if (pB <= pA) {
        M -= pB;
        pr = pB;
        B -= 1;
        pB = pB / hp_R(P, B);
      } else {
        M -= pA;
        pl = pA;
        A += 1;
        pA = pA * hp_R(P, A - 1);
      }
      continue;
    }
    const long double pn = pl >= pr ? pl : pr;
    if (pn > pe) {
      if (pl >= pr) {
        A -= 1;
        M += pl;
        pA = pl;
        pl = A > 0 ? pl / hp_R(P, A - 1) : 0.0L;
      } else {
        B += 1;
        M += pr;
        pB = pr;
        pr = B < N ? pr * hp_R(P, B) : 0.0L;
      }
      continue;
    }
    break;
  }
  *lo = A;
  *hi = B;
}

static void hp_setup(hpd_t* P, double N, double a, double b) {
  P->N = N;
  P->a = a;
  P->b = b;
  P->m = hp_mode(N, a, b);
  P->pm = exp((double)(lrise_l(P->m, a) + lrise_l(N - P->m, b) - lrise_l(N, (long double)a + b)));
}

/* MDFIT-HPDI v1 (see the header): window of BetaBinomial(a, b, N), N >= 1 */
static void hp_window(double N, double a, double b, double* lo, double* hi) {
  if (!(a > 0.0)) {
    *lo = *hi = 0.0;
    return;
  }
  if (!(b > 0.0)) {
    *lo = *hi = N;
    return;
  }
  hpd_t P;
  hp_setup(&P, N, a, b);
  const double phi = a + b, m = P.m;
  const double sd = sqrt(N * a * b * (phi + N) / (phi * phi * (phi + 1.0)));
  if (sd <= HP_SIG_GREEDY || P.pm >= HP_MASS) {
    hp_greedy(&P, lo, hi);
    return;
  }
  const double mu = N * a / phi;
  /* g(0), g(N) only when that support end is within 4 tau of the mode (tau^2 =
   * sd^2 + (mean - mode)^2): beyond, the 68 % window (inside mode +- 2.4 tau,
   * Gauss's inequality) never reaches it */
  const double tau = sqrt(sd * sd + (mu - m) * (mu - m));
  const double g0 = m > 0 ? (m <= 4.0 * tau ? hp_g(&P, 0.0) : -INFINITY) : 0.0;
  const double gN = m < N ? (N - m <= 4.0 * tau ? hp_g(&P, N) : -INFINITY) : 0.0;
  double A, B;
  long double M;
  double t = HP_T0;
  /* one-sided when exactly one end is clamped at the start level (both
   * clamped: a near-flat pmf -- the level Newton below raises t) */
  const int L0 = m == 0 || g0 >= t, R0 = m == N || gN >= t;
  const int one = (L0 && !R0) ? 0 : ((R0 && !L0) ? 1 : -1);
  if (one >= 0) {
    /* window [0, B] (one = 0) or [A, N] (one = 1): Newton on the free end in
     * w = ln(end + alpha) (resp. ln(N - end + beta)) for logit(M) */
    double x = one == 0 ? fmax(mu, m + 1.0) : fmin(mu, m - 1.0);
    double lb = one == 0 ? m : 0.0, hb = one == 0 ? N : m;
    const double Lt = log(HP_MASS / (1.0 - HP_MASS));
    for (int it = 0;; it++) {
      A = one == 0 ? 0.0 : ceil(x);
      B = one == 0 ? floor(x) : N;
      M = (long double)hp_mass(&P, A, B, sd) * P.pm;
      const double Md = (double)M;
      const double fx = hp_f(&P, x) * P.pm;
      const double F = log(Md / (1.0 - Md)) - Lt;
      const double jac = one == 0 ? x + a : N - x + b;
      const double dF = fx * jac * (1.0 / Md + 1.0 / (1.0 - Md));
      double xn;
      if (one == 0) {
        if (F > 0) hb = x;
        else lb = x;
        xn = exp(log(x + a) - F / dF) - a;
      } else {
        if (F > 0) lb = x;
        else hb = x;
        xn = N + b - exp(log(N - x + b) - F / dF);
      }
      if (!(lb < xn && xn < hb)) xn = 0.5 * (lb + hb);
      if (fabs(xn - x) < HP_STOP || it >= 40) break;
      x = xn;
    }
  } else {
    double tL = -INFINITY, tH = 0.0;
    double xl = m - sd, xr = m + sd;
    for (int it = 0;; it++) {
      int cl, cr;
      if (m == 0 || g0 >= t) {
        xl = 0.0;
        cl = 1;
      } else {
        xl = hp_root(&P, t, 0.0, m, xl, 1);
        cl = 0;
      }
      if (m == N || gN >= t) {
        xr = N;
        cr = 1;
      } else {
        xr = hp_root(&P, t, m, N, xr, 0);
        cr = 0;
      }
      A = ceil(xl);
      B = floor(xr);
      M = (long double)hp_mass(&P, A, B, sd) * P.pm;
      if (M >= HP_MASS) tL = t;
      else tH = t;
      double Dp = 0.0, mv = 0.0;
      if (!cl) {
        const double sl = hp_s(&P, xl);
        Dp += exp(t) / sl;
        mv += 1.0 / sl;
      }
      if (!cr) {
        const double sr = -hp_s(&P, xr);
        Dp += exp(t) / sr;
        mv += 1.0 / sr;
      }
      Dp *= P.pm;
      if (it >= 40) break;
      double tn;
      if (Dp > 0.0) {
        const double Md = (double)M;
        const double dt = (log(Md) - log(HP_MASS)) * Md / Dp;
        if (fabs(dt) * mv < HP_STOP) break;
        tn = t + dt;
      } else {
        tn = 0.5 * (tL + tH); /* both ends clamped: all the mass, raise the level */
      }
      if (!(tL < tn && tn < tH)) tn = tL > -INFINITY ? 0.5 * (tL + tH) : t - fmax(1.0, fabs(t));
      t = tn;
    }
  }
  hp_fixup(&P, A, B, M, lo, hi);
}

/* batch entry points for tests: mode 0 = the spec (hp_window), 1 = greedy */
void oracle_hpdi68(const double* N, const double* a, const double* b, int64_t n, int mode, double* lo,
                   double* hi) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int64_t i = 0; i < n; i++) {
    if (!(N[i] > 0)) {
      lo[i] = hi[i] = NAN;
      continue;
    }
    if (mode == 0) {
      hp_window(N[i], a[i], b[i], lo + i, hi + i);
    } else if (!(a[i] > 0)) {
      lo[i] = hi[i] = 0.0;
    } else if (!(b[i] > 0)) {
      lo[i] = hi[i] = N[i];
    } else {
      hpd_t P;
      hp_setup(&P, N[i], a[i], b[i]);
      hp_greedy(&P, lo + i, hi + i);
    }
  }
}
