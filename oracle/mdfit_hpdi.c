/*
 * mdfit_hpdi.c — CPU ORACLE (test infrastructure only; included by
 * mdfit_oracle.c).
 *
 * MDFIT-HPDI v2: the 68 % highest-probability window of the MAP predictive
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
 *                 predictive sd is <= 40 points (round 6; 100 before) (or the mode alone holds 68 %),
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
 * v2 (round 5) changes only the path to the window, not its definition: the
 * level Newton in z = sqrt(-2t) on sqrt(2) erfinv(M) (series about 0.68), the
 * one-sided Newton on the complementary log-log of M, root starts moved by the
 * last level step, settled roots at 2 counts, and each iteration's mass from the
 * previous one plus the strips its ends moved over (2/3/6-point Gauss-Legendre
 * by the strip's width) with the Euler-Maclaurin ends' f and s reused as the
 * Newton slopes and the fix-up's end pmfs -- 40.6 -> 25.4 evaluations of ln p
 * per wide window on the bench's windows (tools/hpdi_study.py), and closer to
 * the point-by-point greedy (29 vs 55 of 90k windows differ by a count).
 * The oracle evaluates ln p with long-double lgammal; the kernel with the
 * cancellation-free lnGamma differences of mdfit_special.h.
 */

#define HP_MASS 0.68
#ifndef HP_SIG_GREEDY
#define HP_SIG_GREEDY 40.0 /* sd (counts) up to which the greedy itself runs (round 6: 100 before) */
#endif
#define HP_T0 (-0.49447329849) /* -Z68^2 / 2: the Gaussian 68 % level */
#define HP_K0 16               /* exact sums this close to a support end */
#define HP_LV 4.0              /* max panel length in a log variable */
#define HP_LX 2.5              /* max linear panel length, in units of sd */
#define HP_STOP 16.0           /* Newton stops when the ends would move < this (counts): the
                                * exact fix-up walk (~20 instructions a count) finishes */
#define HP_RTOL 2.0            /* a window end's Newton root is settled (counts; v2: 0.05 in v1) */

/* development counters (-DHP_COUNT, tools/hpdi_study.py): evaluations of ln p
 * per site, the level iterations and the walk steps */
#ifdef HP_COUNT
unsigned long long hp_cnt[24];
#define HPC(k) __atomic_fetch_add(&hp_cnt[k], 1ull, __ATOMIC_RELAXED)
void oracle_hpdi_counts(unsigned long long* o) {
  for (int i = 0; i < 24; i++) {
    o[i] = hp_cnt[i];
    hp_cnt[i] = 0;
  }
}
#else
#define HPC(k) ((void)0)
#endif

static const double HP_GLX[3] = {0.2386191860831969, 0.6612093864662645, 0.9324695142031521};
static const double HP_GLW[3] = {0.4679139345726910, 0.3607615730481386, 0.1713244923791704};
#define HP_GL2X 0.57735026918962576451 /* 1/sqrt(3) */
#define HP_GL3X 0.77459666924148337704 /* sqrt(3/5) */
#define HP_GL3W0 0.88888888888888888889
#define HP_GL3W1 0.55555555555555555556
#define HP_S6 0.5 /* strips up to half the local scale: 6 nodes */

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
  HPC(10);
  for (double y = A; y <= B; y += 1.0) {
    HPC(6);
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
        HPC(2);
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
        HPC(2);
        I += HP_GLW[i < 3 ? 2 - i : i - 3] * h * hp_f(P, x);
      }
    }
  }
  return I;
}

/* What one mass evaluation leaves for the next level iteration: the window, its
 * Euler-Maclaurin range [A1, B1] (the window less its exact heads), the
 * integral over that range, the exact sums, and f, s at A1 and B1 (v2). */
typedef struct {
  double A, B, A1, B1, I, tot, fA, sA, fB, sB;
  int em; /* [A1, B1] summed by Euler-Maclaurin (else the window is all exact sums) */
} hp_mass_t;

/* Gauss-Legendre nodes of a strip between consecutive windows' ends: 0 for an
 * empty strip, 2 within 2 % of the local scale (min(sd, distance to a support
 * end)), 3 within 10 % (a Gaussian pmf: <= 2e-13 of the mass, the full
 * computation's class), -1 wider (recompute) */
static int hp_strip_nodes(const hpd_t* P, double u0, double u1, double sd) {
  const double lo = fmin(u0, u1), hi = fmax(u0, u1), w = hi - lo;
  if (w == 0.0) return 0;
  const double l = fmin(sd, fmin(lo + P->a, P->N - hi + P->b));
  return w <= 0.02 * l ? 2 : (w <= 0.1 * l ? 3 : (w <= HP_S6 * l ? 6 : -1));
}

/* signed int_{u0}^{u1} p(x)/p(m) dx by n-point Gauss-Legendre (n = 0, 2, 3) */
static double hp_strip(const hpd_t* P, double u0, double u1, int n) {
  if (n == 0) return 0.0;
  const double h = 0.5 * (u1 - u0), c = 0.5 * (u0 + u1);
  double acc = 0.0;
  for (int i = 0; i < n; i++) {
    double x, w;
    if (n == 6) {
      x = i < 3 ? -HP_GLX[2 - i] : HP_GLX[i - 3];
      w = HP_GLW[i < 3 ? 2 - i : i - 3];
    } else if (n == 3) {
      x = (i - 1) * HP_GL3X;
      w = i == 1 ? HP_GL3W0 : HP_GL3W1;
    } else {
      x = i == 0 ? -HP_GL2X : HP_GL2X;
      w = 1.0;
    }
    HPC(2);
    acc += w * hp_f(P, c + h * x);
  }
  return h * acc;
}

/* sum_{y=A}^{B} p(y)/p(m): exact within HP_K0 of the support ends and for
 * short windows, Euler-Maclaurin elsewhere (integral + (f(A1)+f(B1))/2 +
 * (f'(B1)-f'(A1))/12).  The integral: split at the mode into Gauss-Legendre
 * panels; or, when `pv` (the previous iteration's window) has the same exact
 * heads and both ends moved by narrow strips, pv's integral plus the strips
 * (v2).  f, s at an unmoved range end are pv's. */
static double hp_mass(const hpd_t* P, double A, double B, double sd, const hp_mass_t* pv, hp_mass_t* o) {
  const double N = P->N;
  double A1 = A, B1 = B;
  /* the exact heads: [A, A1 - 1] within HP_K0 of 0, [B1 + 1, B] within HP_K0 of N */
  if (A1 < HP_K0) A1 = fmin(HP_K0 - 1, B) + 1;
  if (B1 > N - HP_K0 && B1 >= A1) B1 = fmax(N - HP_K0 + 1, A1) - 1;
  /* ... the same as pv's (same ends and extents) */
  const int same = pv && pv->em && (A1 == A) == (pv->A1 == pv->A) && (A1 == A || (A == pv->A && A1 == pv->A1)) &&
                   (B1 == B) == (pv->B1 == pv->B) && (B1 == B || (B == pv->B && B1 == pv->B1));
  double tot = 0.0;
  if (same) {
    tot = pv->tot;
  } else {
    if (A1 > A) tot += hp_exact_sum(P, A, A1 - 1);
    if (B1 < B) tot += hp_exact_sum(P, B1 + 1, B);
  }
  o->A = A;
  o->B = B;
  o->A1 = A1;
  o->B1 = B1;
  o->em = 0;
  if (same) tot = pv->tot;
  if (B1 < A1) {
    o->tot = tot;
    return tot;
  }
  if (B1 - A1 < 32) {
    o->tot = tot + hp_exact_sum(P, A1, B1);
    return o->tot;
  }
  const int nl = same ? hp_strip_nodes(P, A1, pv->A1, sd) : -1;
  const int nr = same ? hp_strip_nodes(P, pv->B1, B1, sd) : -1;
  double I = 0.0;
  if (nl >= 0 && nr >= 0) {
    HPC(15);
    I = pv->I + hp_strip(P, A1, pv->A1, nl) + hp_strip(P, pv->B1, B1, nr);
  } else {
    const double c = fmin(fmax(P->m, A1), B1);
    if (c > A1) I += hp_part(P, A1, c, sd);
    if (B1 > c) I += hp_part(P, c, B1, sd);
  }
  if (same && A1 == pv->A1) {
    o->fA = pv->fA;
    o->sA = pv->sA;
  } else {
    HPC(3);
    o->fA = hp_f(P, A1);
    o->sA = hp_s(P, A1);
  }
  if (same && B1 == pv->B1) {
    o->fB = pv->fB;
    o->sB = pv->sB;
  } else {
    HPC(3);
    o->fB = hp_f(P, B1);
    o->sB = hp_s(P, B1);
  }
  o->I = I;
  o->tot = tot;
  o->em = 1;
  return tot + I + 0.5 * (o->fA + o->fB) + (o->fB * o->sB - o->fA * o->sA) / 12.0;
}

/* x in [lo, hi] with g(x) = t (g monotone there; rising = g - t < 0 at lo):
 * safeguarded Newton */
static double hp_root(const hpd_t* P, double t, double lo, double hi, double x0, int rising) {
  double x = fmin(fmax(x0, lo), hi);
  for (int it = 0; it < 60; it++) {
    HPC(1);
    const double gx = hp_g(P, x) - t;
    if (fabs(gx) < 1e-12) return x;
    if ((gx < 0) == (rising != 0)) lo = x;
    else hi = x;
    const double sx = hp_s(P, x);
    double xn = sx != 0.0 ? x - gx / sx : 0.5 * (lo + hi);
    if (!(lo < xn && xn < hi)) xn = 0.5 * (lo + hi);
    if (fabs(xn - x) < HP_RTOL) return xn;
    x = xn;
  }
  return x;
}

#define HP_Z68 0.99445788320975304 /* sqrt(2) erfinv(0.68) */
#define HP_D68 0.48662348157070173 /* d erf(z / sqrt 2) / dz at HP_Z68 */
#define HP_C2 0.49722894160487652 /* HP_Z68 / 2 */
#define HP_C3 0.49631549382600754 /* (2 HP_Z68^2 + 1) / 6 */
#define HP_CLL68 0.13053189641996385 /* ln(-ln(1 - 0.68)) */

/* window [A, B] holding mass M (absolute) -> the greedy's window */
static void hp_fixup(const hpd_t* P, double A, double B, long double M, long double pA, long double pB, double* lo,
                     double* hi) {
  const double N = P->N;
  long double pl = A > 0 ? pA / hp_R(P, A - 1) : 0.0L;
  long double pr = B < N ? pB * hp_R(P, B) : 0.0L;
  while (M < HP_MASS && (pl > 0 || pr > 0)) {
    HPC(7);
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
    HPC(7);
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

/* MDFIT-HPDI v2 (see the header): window of BetaBinomial(a, b, N), N >= 1 */
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
  HPC(8);
  /* g(0), g(N) only when that support end is within 4 tau of the mode (tau^2 =
   * sd^2 + (mean - mode)^2): beyond, the 68 % window (inside mode +- 2.4 tau,
   * Gauss's inequality) never reaches it */
  const double tau = sqrt(sd * sd + (mu - m) * (mu - m));
  if (m > 0 && m <= 4.0 * tau) HPC(0);
  if (m < N && N - m <= 4.0 * tau) HPC(0);
  const double g0 = m > 0 ? (m <= 4.0 * tau ? hp_g(&P, 0.0) : -INFINITY) : 0.0;
  const double gN = m < N ? (N - m <= 4.0 * tau ? hp_g(&P, N) : -INFINITY) : 0.0;
  double A, B;
  long double M;
  double t = HP_T0;
  hp_mass_t ms, pv;
  int have = 0;
  /* one-sided when exactly one end is clamped at the start level (both
   * clamped: a near-flat pmf -- the level Newton below raises t) */
  const int L0 = m == 0 || g0 >= t, R0 = m == N || gN >= t;
  const int one = (L0 && !R0) ? 0 : ((R0 && !L0) ? 1 : -1);
  HPC(one >= 0 ? 16 : 17);
  if (one >= 0) {
    /* window [0, B] (one = 0) or [A, N] (one = 1): Newton on the free end in
     * w = ln(end + alpha) (resp. ln(N - end + beta)) for logit(M) */
    double x = one == 0 ? fmax(mu, m + 1.0) : fmin(mu, m - 1.0);
    double lb = one == 0 ? m : 0.0, hb = one == 0 ? N : m;
    for (int it = 0;; it++) {
      A = one == 0 ? 0.0 : ceil(x);
      B = one == 0 ? floor(x) : N;
      M = (long double)hp_mass(&P, A, B, sd, have ? &pv : NULL, &ms) * P.pm;
      pv = ms;
      have = 1;
      HPC(9);
      HPC(18);
      /* p at the free end: the Euler-Maclaurin end's when that is the window's
       * end (v2), else evaluated at x */
      double fx;
      if (ms.em && (one == 0 ? ms.B1 == B : ms.A1 == A)) {
        fx = (one == 0 ? ms.fB : ms.fA) * P.pm;
      } else {
        HPC(4);
        fx = hp_f(&P, x) * P.pm;
      }
      /* Newton on the complementary log-log of M against ln(end + alpha)
       * (v2; v1: logit M): linear for a Gamma-like pmf both near the clamped
       * end (M ~ x^alpha) and in its exponential tail */
      const double Mc = fmin((double)M, 1.0 - 1e-16);
      const double jac = one == 0 ? x + a : N - x + b;
      const double Lc = -log1p(-Mc);
      const double F = log(Lc) - HP_CLL68;
      const double dF = fx * jac / ((1.0 - Mc) * Lc);
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
      if (fabs(xn - x) < HP_STOP || it >= 40) {
        HPC(11 + (it < 3 ? it : 3));
        break;
      }
      x = xn;
    }
  } else {
    double tL = -INFINITY, tH = 0.0, sl = 0.0, sr = 0.0, dtp = 0.0;
    double xl = m - sd, xr = m + sd;
    for (int it = 0;; it++) {
      int cl, cr;
      /* the free ends' roots of g = t, from the previous roots moved by the
       * level step over their slopes (v2) */
      if (m == 0 || g0 >= t) {
        xl = 0.0;
        cl = 1;
      } else {
        if (it > 0 && sl > 0) xl += dtp / sl;
        xl = hp_root(&P, t, 0.0, m, xl, 1);
        cl = 0;
      }
      if (m == N || gN >= t) {
        xr = N;
        cr = 1;
      } else {
        if (it > 0 && sr > 0) xr -= dtp / sr;
        xr = hp_root(&P, t, m, N, xr, 0);
        cr = 0;
      }
      A = ceil(xl);
      B = floor(xr);
      M = (long double)hp_mass(&P, A, B, sd, have ? &pv : NULL, &ms) * P.pm;
      pv = ms;
      have = 1;
      HPC(9);
      if (M >= HP_MASS) tL = t;
      else tH = t;
      /* the slopes at the ends: the Euler-Maclaurin ends' when those are the
       * window's ends (v2), else at the roots */
      double Dp = 0.0, mv = 0.0;
      if (!cl) {
        if (ms.em && ms.A1 == A) {
          sl = ms.sA;
        } else {
          HPC(4);
          sl = hp_s(&P, xl);
        }
        Dp += exp(t) / sl;
        mv += 1.0 / sl;
      }
      if (!cr) {
        if (ms.em && ms.B1 == B) {
          sr = -ms.sB;
        } else {
          HPC(4);
          sr = -hp_s(&P, xr);
        }
        Dp += exp(t) / sr;
        mv += 1.0 / sr;
      }
      Dp *= P.pm;
      if (it >= 40) {
        HPC(11 + 3);
        break;
      }
      double tn;
      if (Dp > 0.0) {
        /* Newton in z = sqrt(-2t) on u(M) = sqrt(2) erfinv(M), which is z itself
         * for a Gaussian pmf (v2; v1: Newton on ln M in t) -- u by its cubic
         * Taylor series about 0.68, used within |q| < 0.3 (beyond, the v1
         * step); the stop: the ends would move < HP_STOP counts */
        const double Md = (double)M;
        const double z = sqrt(-2.0 * t);
        const double q = (Md - HP_MASS) / HP_D68;
        const double u = HP_Z68 + q * (1.0 + q * (HP_C2 + q * HP_C3));
        const double du = (1.0 + q * (2.0 * HP_C2 + q * 3.0 * HP_C3)) / HP_D68 * Dp * z;
        const double zn = fabs(q) < 0.3 ? z - (u - HP_Z68) / du : -1.0;
        const double step = zn > 0.0 ? -0.5 * zn * zn - t : (log(Md) - log(HP_MASS)) * Md / Dp;
        if (fabs(step) * mv < HP_STOP) {
          HPC(11 + (it < 3 ? it : 3));
          break;
        }
        tn = t + step;
      } else {
        tn = 0.5 * (tL + tH); /* both ends clamped: all the mass, raise the level */
      }
      if (!(tL < tn && tn < tH)) tn = tL > -INFINITY ? 0.5 * (tL + tH) : t - fmax(1.0, fabs(t));
      dtp = tn - t;
      t = tn;
    }
  }
  /* p at the window's ends for the fix-up: the Euler-Maclaurin ends' (v2) */
  long double pA, pB;
  if (ms.em && ms.A1 == A) {
    pA = (long double)ms.fA * P.pm;
  } else {
    HPC(5);
    pA = (long double)hp_f(&P, A) * P.pm;
  }
  if (B == A) {
    pB = pA;
  } else if (ms.em && ms.B1 == B) {
    pB = (long double)ms.fB * P.pm;
  } else {
    HPC(5);
    pB = (long double)hp_f(&P, B) * P.pm;
  }
  hp_fixup(&P, A, B, M, pA, pB, lo, hi);
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
