/*
 * mdfit_nuts.c — CPU ORACLE of the sampling mode (test infrastructure only;
 * #included by mdfit_oracle.c, shares its special functions and the record
 * helpers n_sigma / asymmetry / noise).
 *
 * MDFIT-NUTS v1: the reference samples every sub-fit with
 * numpyro ^0.4.1 NUTS (fits.py:382-387; mcmc_kwargs fits.py:792-799:
 * num_warmup 500, num_samples 1000, one chain, Key(0)).  numpyro / jax are
 * not importable here, so the sampler is restated from its
 * published algorithm -- same defaults, same trajectory construction, same
 * adaptation -- with a counter-based Philox4x32-10 stream in place of jax's
 * threefry keys (the GPU kernel draws the identical numbers):
 *
 *   potential   -(log density + log|J|) in unconstrained v:
 *               q, A, c = sigmoid(v0..v2) (Beta priors, fits.py:46-48),
 *               delta = exp(v3) (Exponential(1/1000), fits.py:53); null: v0, v3
 *   dynamics    velocity Verlet, diagonal inverse mass matrix
 *   trajectory  iterative NUTS, multinomial sampling: uniform progressive
 *               sampling inside a subtree, biased progressive sampling across
 *               doublings (a turning / diverging subtree is never moved to),
 *               generalised U-turn on momentum sums with the iterative
 *               checkpoints of all sub-subtrees, max tree depth 10,
 *               divergence at delta energy > 1000
 *   adaptation  Stan windows for 500 warmup iterations: 75 / 25 / 50 / 100 /
 *               200 / 50; dual averaging (t0 10, kappa 0.75, gamma 0.05, target
 *               accept 0.8, prox centre log(10 eps)); regularised diagonal
 *               Welford variance in the slow windows ((n/(n+5)) var +
 *               1e-3 * 5/(n+5)); find_reasonable_step_size (doubling /
 *               halving until the log(0.8) criterion flips) at the start and
 *               after every slow window; final step size exp(log eps avg)
 *   init        v ~ U(-2, 2) per coordinate, up to 100 attempts for a finite
 *               potential (init_to_uniform)
 *
 * Post-processing per taxon (the reference's functions on the 1000 draws):
 *   pointwise log-likelihood incl. log C(N,y)   fits.py:126-141
 *   lppd_i, pWAIC_i (var, ddof 0), waic_i      fits.py:147-172
 *   n_sigma / asymmetry                         fits.py:194-227
 *   posterior predictive: p ~ Beta(a, b),
 *     obs ~ Binomial(N, p), frac = obs / N      fits.py:89-106
 *   median, 68 % HPDI of frac                   fits.py:112-120 (np.median,
 *                                               numpyro.diagnostics.hpdi)
 *   record                                      fits.py:230-356 (D_max =
 *     median at z=+1, HPDI there, means of q / phi / D_max; forward / reverse
 *     fits with the data_forward quirk of :343-348), noise fits.py:359-376
 *
 * Random streams: key = (lo32 seed, hi32 seed); counter = (lo32 g,
 * hi32 g + (sub << 24), word2, word3) with g = index_base + taxon.  A
 * uniform takes words 0-1 (53 bits) or 2-3; a pair of normals is Box-Muller
 * on one block, words 0-1 the radius, 2-3 the angle: cos, then sin (draw
 * convention 2, round 6: a block yields two draws where the chain kernel
 * used one -- half the Philox work of its per-iteration draws).
 *   chain iteration it:   word2 = it; word3 = 0, 1 momentum dims 2m, 2m+1,
 *                         4 + j doubling j: transition uniform words 0-1,
 *                         direction bit 0 of word 2,
 *                         32 + m progressive-sampling uniforms of leaves
 *                         2m (words 0-1) and 2m + 1 (words 2-3)
 *   init attempt a:       word2 = 0xFFFF0000 + a, word3 = dim
 *   step-size search f,m: word2 = 0xFFFE0000 + 4096 f + m, word3 = dim
 *   predictive draw s, i: word2 = 0xFFFD0000 + s, word3 = (i << 16) + k, the
 *                         k-th block of the draw: two uniforms or two normals
 *                         (predictive draw convention 2, round 6)
 */

#define NUTS_MAX_DEPTH 10
#define NUTS_MAX_DELTA 1000.0
#define NUTS_TARGET 0.8

/* ---------------------------------------------------------------------------
 * Philox4x32-10
 * ------------------------------------------------------------------------- */
static void philox4x32(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1, n3 = (uint32_t)p0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

void oracle_philox(const uint32_t* ctr4, const uint32_t* key2, uint32_t* out4) {
  philox4x32(ctr4, key2, out4);
}

typedef struct {
  uint32_t key[2];
  uint32_t c0, c1;
} nstream;

static nstream nstream_make(uint64_t seed, int64_t g, int sub) {
  nstream s;
  s.key[0] = (uint32_t)seed;
  s.key[1] = (uint32_t)(seed >> 32);
  s.c0 = (uint32_t)(uint64_t)g;
  s.c1 = (uint32_t)((uint64_t)g >> 32) + ((uint32_t)sub << 24);
  return s;
}

static void nblock(const nstream* s, uint32_t w2, uint32_t w3, uint32_t out[4]) {
  uint32_t c[4] = {s->c0, s->c1, w2, w3};
  philox4x32(c, s->key, out);
}

static double u53(uint32_t a, uint32_t b) { /* [0, 1) */
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

static double nuniform(const nstream* s, uint32_t w2, uint32_t w3) {
  uint32_t o[4];
  nblock(s, w2, w3, o);
  return u53(o[0], o[1]);
}

/* the Box-Muller pair of one block: cos (k = 0) or sin (k = 1) */
static double nnormal_k(const nstream* s, uint32_t w2, uint32_t w3, int k) {
  uint32_t o[4];
  nblock(s, w2, w3, o);
  const double u1 = 1.0 - u53(o[0], o[1]); /* (0, 1] */
  const double u2 = u53(o[2], o[3]);
  const double r = sqrt(-2.0 * log(u1)), a = 6.283185307179586 * u2;
  return r * (k ? sin(a) : cos(a));
}

/* ---------------------------------------------------------------------------
 * potential energy and gradient in unconstrained v (numpyro's potential_fn)
 * ------------------------------------------------------------------------- */
static int nuts_active(int model, int j) { return model == M_PMD || j == 0 || j == 3; }

/* theta = (q, A, c, phi) of v (null: A = c = 0) */
static void nuts_theta(int model, const double v[4], double th[4]) {
  th[0] = sigm(v[0]);
  th[1] = model == M_PMD ? sigm(v[1]) : 0.0;
  th[2] = model == M_PMD ? sigm(v[2]) : 0.0;
  th[3] = exp(v[3]) + 2.0;
}

/* U(v) and dU/dv; a non-finite U (infeasible A + c >= 1, i.e. D clipped to 1,
 * fits.py:50, or an overflow) is reported as +inf with a zero gradient. */
static double nuts_potential(int model, const uint32_t* y, const uint32_t* N, int lo, int hi,
                             const double v[4], double g[4]) {
  const double q = sigm(v[0]), lq = -softplus(-v[0]), l1q = -softplus(v[0]);
  const double delta = exp(v[3]), phi = delta + 2.0;
  double A = 0, c = 0, lA = 0, l1A = 0, lc = 0, l1c = 0;
  if (model == M_PMD) {
    A = sigm(v[1]);
    lA = -softplus(-v[1]);
    l1A = -softplus(v[1]);
    c = sigm(v[2]);
    lc = -softplus(-v[2]);
    l1c = -softplus(v[2]);
  }
  /* log prior + log|J|: q, A ~ Beta(2,3) -> 2 ln p + 3 ln(1-p); c ~ Beta(1,9)
   * -> ln c + 9 ln(1-c); delta ~ Exp(1/1000) -> v3 - delta/1000 */
  /* Exponential(rate 1/1000).log_prob = log(rate) - rate * delta (numpyro's form) */
  double lp = 2.0 * lq + 3.0 * l1q + v[3] - delta * 1e-3;
  double gq = 2.0 - 5.0 * q, gA = 0, gc = 0, gd = 1.0 - delta * 1e-3;
  if (model == M_PMD) {
    lp += 2.0 * lA + 3.0 * l1A + lc + 9.0 * l1c;
    gA = 2.0 - 5.0 * A;
    gc = 1.0 - 10.0 * c;
  }
  double ell = 0, sDq = 0, sDA = 0, sDc = 0, sF = 0;
  int bad = model == M_PMD && A + c >= 1.0;
  const double psi_phi = o_digamma(phi), lg_phi = o_lgamma(phi);
  for (int i = lo; i < hi && !bad; i++) {
    const int k = kpos(i);
    double D, dq, dA = 0.0;
    if (model == M_PMD) {
      const double w = pow(1.0 - q, (double)k);
      D = A * w + c;
      dq = k > 0 ? -A * k * pow(1.0 - q, (double)(k - 1)) : 0.0;
      dA = w;
    } else {
      D = q;
      dq = 1.0;
    }
    if (!(D < 1.0)) {
      bad = 1;
      break;
    }
    const double yy = y[i], nn = N[i], a = D * phi, b = (1.0 - D) * phi;
    ell += o_lgamma(yy + a) - o_lgamma(a) + o_lgamma(nn - yy + b) - o_lgamma(b) - o_lgamma(nn + phi) + lg_phi;
    const double Pa = o_digamma(yy + a) - o_digamma(a), Pb = o_digamma(nn - yy + b) - o_digamma(b);
    const double lD = phi * (Pa - Pb);
    sF += D * Pa + (1.0 - D) * Pb + psi_phi - o_digamma(nn + phi);
    sDq += lD * dq;
    sDA += lD * dA;
    sDc += lD;
  }
  const double U = -(ell + lp);
  if (bad || !isfinite(U)) {
    for (int j = 0; j < 4; j++) g[j] = 0.0;
    return INFINITY;
  }
  g[0] = -(sDq * q * (1.0 - q) + gq);
  g[1] = model == M_PMD ? -(sDA * A * (1.0 - A) + gA) : 0.0;
  g[2] = model == M_PMD ? -(sDc * c * (1.0 - c) + gc) : 0.0;
  g[3] = -(sF * delta + gd);
  return U;
}

void oracle_nuts_potential(int model, int subset, const uint32_t* y, const uint32_t* N, const double* v,
                           double* U, double* g4) {
  int lo = subset == 2 ? NHALF : 0, hi = subset == 1 ? NHALF : NPOS;
  *U = nuts_potential(model, y, N, lo, hi, v, g4);
}

/* ---------------------------------------------------------------------------
 * NUTS
 * ------------------------------------------------------------------------- */
typedef struct {
  int model, lo, hi;
  const uint32_t* y;
  const uint32_t* N;
} nctx;

typedef struct {
  double z[4], r[4], g[4], pe;
} nps; /* phase-space point */

static double kinetic(int model, const double invm[4], const double r[4]) {
  double k = 0;
  for (int j = 0; j < 4; j++)
    if (nuts_active(model, j)) k += invm[j] * r[j] * r[j];
  return 0.5 * k;
}

static void leapfrog(const nctx* cx, double eps, const double invm[4], nps* s) {
  for (int j = 0; j < 4; j++)
    if (nuts_active(cx->model, j)) s->r[j] -= 0.5 * eps * s->g[j];
  for (int j = 0; j < 4; j++)
    if (nuts_active(cx->model, j)) s->z[j] += eps * invm[j] * s->r[j];
  s->pe = nuts_potential(cx->model, cx->y, cx->N, cx->lo, cx->hi, s->z, s->g);
  for (int j = 0; j < 4; j++)
    if (nuts_active(cx->model, j)) s->r[j] -= 0.5 * eps * s->g[j];
}

static double logaddexp(double a, double b) {
  const double m = a > b ? a : b;
  if (m == -INFINITY) return -INFINITY;
  return m + log1p(exp(-fabs(a - b)));
}

static int is_turning(int model, const double invm[4], const double rl[4], const double rr[4],
                      const double rsum[4]) {
  double dl = 0, dr = 0;
  for (int j = 0; j < 4; j++) {
    if (!nuts_active(model, j)) continue;
    const double rs = rsum[j] - 0.5 * (rl[j] + rr[j]);
    dl += invm[j] * rl[j] * rs;
    dr += invm[j] * rr[j] * rs;
  }
  return dl <= 0.0 || dr <= 0.0;
}

typedef struct {
  nps left, right;
  double zp[4], gp[4], pep; /* proposal */
  double weight, rsum[4], sum_acc;
  int nprop, turning, diverging, depth;
} ntree;

static void momentum(const nctx* cx, const nstream* st, uint32_t w2, const double invm[4], double r[4]) {
  for (int j = 0; j < 4; j++)
    r[j] = nuts_active(cx->model, j) ? nnormal_k(st, w2, (uint32_t)(j >> 1), j & 1) * sqrt(1.0 / invm[j]) : 0.0;
}

/* numpyro find_reasonable_step_size (hmc_util) */
static double find_step(const nctx* cx, const nstream* st, int call, double eps, const double invm[4],
                        const nps* cur) {
  int last = 0, dir = 0;
  for (int m = 0; m < 4000; m++) {
    if (m > 0) {
      const int not_small = eps > 2.2250738585072014e-308 || dir >= 0;
      const int not_large = eps < 1.7976931348623157e308 || dir <= 0;
      if (!(not_small && not_large && (last == 0 || dir == last))) break;
    }
    eps = ldexp(eps, dir);
    nps s = *cur;
    momentum(cx, st, 0xFFFE0000u + 4096u * (uint32_t)call + (uint32_t)m, invm, s.r);
    const double e0 = cur->pe + kinetic(cx->model, invm, s.r);
    leapfrog(cx, eps, invm, &s);
    const double e1 = s.pe + kinetic(cx->model, invm, s.r);
    const double de = e1 - e0;
    const int dnew = log(NUTS_TARGET) < -de ? 1 : -1;
    last = dir;
    dir = dnew;
  }
  return eps;
}

/* checkpoint indices of leaf n (numpyro _leaf_idx_to_ckpt_idxs) */
static void ckpt_idxs(int n, int* idx_min, int* idx_max) {
  int x = n >> 1, mx = 0;
  while (x > 0) {
    mx += x & 1;
    x >>= 1;
  }
  int ns = 0;
  x = n;
  while (x & 1) {
    ns++;
    x >>= 1;
  }
  *idx_max = mx;
  *idx_min = mx - ns + 1;
}

/* one NUTS transition from cur (z, pe, g); returns the new state in cur,
 * the mean acceptance statistic, depth and divergence */
static void nuts_step(const nctx* cx, const nstream* st, uint32_t it, double eps, const double invm[4], nps* cur,
                      double* acc_out, int* depth_out, int* div_out, int* nleap_out) {
  ntree t;
  memset(&t, 0, sizeof(t));
  t.left = *cur;
  momentum(cx, st, it, invm, t.left.r);
  t.right = t.left;
  const double e0 = cur->pe + kinetic(cx->model, invm, t.left.r);
  memcpy(t.zp, cur->z, sizeof(t.zp));
  memcpy(t.gp, cur->g, sizeof(t.gp));
  t.pep = cur->pe;
  memcpy(t.rsum, t.left.r, sizeof(t.rsum));
  int leaf_ctr = 0, nleap = 0;
  double rck[NUTS_MAX_DEPTH][4], rsck[NUTS_MAX_DEPTH][4];
  while (t.depth < NUTS_MAX_DEPTH && !t.turning && !t.diverging) {
    const int j = t.depth;
    uint32_t o[4];
    nblock(st, it, 4u + (uint32_t)j, o);
    const int right = (int)(o[2] & 1u);
    const double u_tr = u53(o[0], o[1]);
    /* subtree of 2^depth leaves in the chosen direction */
    ntree s;
    memset(&s, 0, sizeof(s));
    const int nmax = 1 << t.depth;
    for (int n = 0; n < nmax; n++) {
      nps p = n == 0 ? (right ? t.right : t.left) : (right ? s.right : s.left);
      leapfrog(cx, right ? eps : -eps, invm, &p);
      nleap++;
      double en = p.pe + kinetic(cx->model, invm, p.r);
      double de = en - e0;
      if (isnan(de)) de = INFINITY;
      const double w = -de;
      const int dv = de > NUTS_MAX_DELTA;
      const double acc = de > 0 ? exp(-de) : 1.0;
      if (n == 0) {
        s.left = s.right = p;
        memcpy(s.zp, p.z, sizeof(s.zp));
        memcpy(s.gp, p.g, sizeof(s.gp));
        s.pep = p.pe;
        s.weight = w;
        memcpy(s.rsum, p.r, sizeof(s.rsum));
        s.sum_acc = acc;
        s.nprop = 1;
        s.diverging = dv;
      } else {
        const double nw = logaddexp(s.weight, w);
        const double prob = exp(w - nw);
        uint32_t ol[4];
        nblock(st, it, 32u + ((uint32_t)leaf_ctr >> 1), ol);
        const double u = (leaf_ctr & 1) ? u53(ol[2], ol[3]) : u53(ol[0], ol[1]);
        if (u < prob) {
          memcpy(s.zp, p.z, sizeof(s.zp));
          memcpy(s.gp, p.g, sizeof(s.gp));
          s.pep = p.pe;
        }
        if (right) s.right = p;
        else s.left = p;
        s.weight = nw;
        for (int k = 0; k < 4; k++) s.rsum[k] += p.r[k];
        s.sum_acc += acc;
        s.nprop += 1;
        s.diverging = dv;
      }
      leaf_ctr++;
      int imin, imax;
      ckpt_idxs(n, &imin, &imax);
      if ((n & 1) == 0) {
        memcpy(rck[imax], p.r, sizeof(p.r));
        memcpy(rsck[imax], s.rsum, sizeof(s.rsum));
      }
      int turning = 0;
      for (int i = imax; i >= imin && !turning; i--) {
        double sub_rsum[4];
        for (int k = 0; k < 4; k++) sub_rsum[k] = s.rsum[k] - rsck[i][k] + rck[i][k];
        turning = is_turning(cx->model, invm, rck[i], p.r, sub_rsum);
      }
      s.turning = turning;
      if (s.turning || s.diverging) break;
    }
    /* biased progressive sampling across the doubling */
    const double prob = (s.turning || s.diverging) ? 0.0 : fmin(1.0, exp(s.weight - t.weight));
    if (u_tr < prob) {
      memcpy(t.zp, s.zp, sizeof(t.zp));
      memcpy(t.gp, s.gp, sizeof(t.gp));
      t.pep = s.pep;
    }
    if (right) t.right = s.right;
    else t.left = s.left;
    t.weight = logaddexp(t.weight, s.weight);
    for (int k = 0; k < 4; k++) t.rsum[k] += s.rsum[k];
    t.turning = s.turning || is_turning(cx->model, invm, t.left.r, t.right.r, t.rsum);
    t.diverging = s.diverging;
    t.sum_acc += s.sum_acc;
    t.nprop += s.nprop;
    t.depth += 1;
  }
  memcpy(cur->z, t.zp, sizeof(t.zp));
  memcpy(cur->g, t.gp, sizeof(t.gp));
  cur->pe = t.pep;
  *acc_out = t.sum_acc / t.nprop;
  *depth_out = t.depth;
  *div_out = t.diverging;
  *nleap_out = nleap;
}

/* Stan / numpyro adaptation windows for num_warmup (build_adaptation_schedule) */
static int adapt_windows(int nw, int win[][2], int maxw) {
  int n = 0;
  if (nw < 20) {
    win[n][0] = 0;
    win[n][1] = nw - 1;
    return 1;
  }
  int init_buffer = 75, term_buffer = 50, base_window = 25;
  if (nw < init_buffer + term_buffer + base_window) {
    init_buffer = (int)(0.15 * nw);
    term_buffer = (int)(0.1 * nw);
    base_window = nw - init_buffer - term_buffer;
  }
  win[n][0] = 0;
  win[n][1] = init_buffer - 1;
  n++;
  const int end_start = nw - term_buffer;
  int next_size = base_window, next_start = init_buffer;
  while (next_start < end_start && n < maxw - 1) {
    const int cs = next_start;
    int csz = next_size;
    if (3 * csz <= end_start - cs) next_size = 2 * csz;
    else csz = end_start - cs;
    next_start = cs + csz;
    win[n][0] = cs;
    win[n][1] = next_start - 1;
    n++;
  }
  win[n][0] = end_start;
  win[n][1] = nw - 1;
  return n + 1;
}

typedef struct {
  double step, div, leap, acc; /* final step size, divergences, leapfrogs/iter, mean accept (sampling) */
  int status;
} nchain_stats;

/* one chain: samples[s] = theta (q, A, c, phi) */
static void nuts_chain(const nctx* cx, const nstream* st, int nwarm, int nsamp, double* samples,
                       nchain_stats* cs) {
  nps cur;
  memset(&cur, 0, sizeof(cur));
  cs->status = MDFIT_NONFINITE;
  for (int a = 0; a < 100; a++) {
    for (int j = 0; j < 4; j++)
      cur.z[j] = nuts_active(cx->model, j) ? -2.0 + 4.0 * nuniform(st, 0xFFFF0000u + (uint32_t)a, (uint32_t)j) : 0.0;
    cur.pe = nuts_potential(cx->model, cx->y, cx->N, cx->lo, cx->hi, cur.z, cur.g);
    if (isfinite(cur.pe)) {
      cs->status = MDFIT_OK;
      break;
    }
  }
  if (cs->status != MDFIT_OK) {
    for (int s = 0; s < nsamp; s++)
      for (int j = 0; j < 4; j++) samples[4 * s + j] = NAN;
    cs->step = cs->div = cs->leap = cs->acc = NAN;
    return;
  }
  double invm[4] = {1, 1, 1, 1};
  double eps = find_step(cx, st, 0, 1.0, invm, &cur);
  /* dual averaging state */
  double x_avg = 0, g_avg = 0, mu = log(10.0 * eps);
  int t_da = 0;
  /* Welford */
  double wmean[4] = {0, 0, 0, 0}, wm2[4] = {0, 0, 0, 0};
  int wn = 0;
  int win[16][2];
  const int nwin = nwarm > 0 ? adapt_windows(nwarm, win, 16) : 0;
  int widx = 0, n_find = 0;
  double div = 0, leap = 0, accs = 0;
  for (int it = 0; it < nwarm + nsamp; it++) {
    double acc;
    int depth, dv, nl;
    nuts_step(cx, st, (uint32_t)it, eps, invm, &cur, &acc, &depth, &dv, &nl);
    if (it < nwarm) {
      /* dual averaging (numpyro hmc_util.dual_averaging) */
      t_da++;
      const double gg = NUTS_TARGET - acc;
      g_avg = (1.0 - 1.0 / (t_da + 10.0)) * g_avg + gg / (t_da + 10.0);
      const double x_t = mu - sqrt((double)t_da) / 0.05 * g_avg;
      const double wt = pow((double)t_da, -0.75);
      x_avg = (1.0 - wt) * x_avg + wt * x_t;
      eps = exp(it == nwarm - 1 ? x_avg : x_t);
      if (eps < 2.2250738585072014e-308) eps = 2.2250738585072014e-308;
      const int middle = widx > 0 && widx < nwin - 1;
      if (middle) {
        wn++;
        for (int j = 0; j < 4; j++) {
          if (!nuts_active(cx->model, j)) continue;
          const double d0 = cur.z[j] - wmean[j];
          wmean[j] += d0 / wn;
          wm2[j] += d0 * (cur.z[j] - wmean[j]);
        }
      }
      const int at_end = it == win[widx][1];
      if (at_end && middle) {
        for (int j = 0; j < 4; j++) {
          if (!nuts_active(cx->model, j)) continue;
          const double var = wm2[j] / (wn - 1);
          invm[j] = ((double)wn / (wn + 5.0)) * var + 1e-3 * (5.0 / (wn + 5.0));
          wmean[j] = wm2[j] = 0.0;
        }
        wn = 0;
        eps = find_step(cx, st, ++n_find, eps, invm, &cur);
        mu = log(10.0 * eps);
        x_avg = g_avg = 0.0;
        t_da = 0;
      }
      if (at_end) widx++;
    } else {
      double th[4];
      nuts_theta(cx->model, cur.z, th);
      memcpy(samples + 4 * (it - nwarm), th, sizeof(th));
      div += dv;
      leap += nl;
      accs += acc;
    }
  }
  cs->step = eps;
  cs->div = div;
  cs->leap = leap / nsamp;
  cs->acc = accs / nsamp;
}

/* ---------------------------------------------------------------------------
 * predictive draws (numpyro BetaBinomial.sample: p ~ Beta, obs ~ Binomial)
 * ------------------------------------------------------------------------- */
typedef struct {
  const nstream* st;
  uint32_t w2, w3;
  double uc, nc; /* the current block's second uniform / normal */
  int uh, nh;
} ndraw; /* sequential draws of one variate */

/* predictive draw convention 2 (round 6): a block gives two uniforms (words
 * 0-1, then 2-3) or a Box-Muller pair of normals (cos, then sin); the two
 * kinds take blocks from one counter in the order they run dry */
static double dr_uniform(ndraw* d) {
  if (d->uh) {
    d->uh = 0;
    return d->uc;
  }
  uint32_t o[4];
  nblock(d->st, d->w2, d->w3++, o);
  d->uc = u53(o[2], o[3]);
  d->uh = 1;
  return u53(o[0], o[1]);
}
static double dr_normal(ndraw* d) {
  if (d->nh) {
    d->nh = 0;
    return d->nc;
  }
  uint32_t o[4];
  nblock(d->st, d->w2, d->w3++, o);
  const double u1 = 1.0 - u53(o[0], o[1]), u2 = u53(o[2], o[3]);
  const double r = sqrt(-2.0 * log(u1)), a = 6.283185307179586 * u2;
  d->nc = r * sin(a);
  d->nh = 1;
  return r * cos(a);
}

/* log of a Gamma(alpha, 1) draw (Marsaglia & Tsang; alpha < 1 boosted by u^(1/alpha)) */
static double log_gamma_draw(ndraw* d, double alpha) {
  double boost = 0.0;
  if (alpha < 1.0) {
    const double u = 1.0 - dr_uniform(d);
    boost = log(u) / alpha;
    alpha += 1.0;
  }
  const double dd = alpha - 1.0 / 3.0, cc = 1.0 / sqrt(9.0 * dd);
  for (int k = 0; k < 256; k++) {
    const double x = dr_normal(d);
    double v = 1.0 + cc * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = dr_uniform(d);
    if (u < 1.0 - 0.0331 * x * x * x * x) return log(dd * v) + boost;
    if (log(u) < 0.5 * x * x + dd * (1.0 - v + log(v))) return log(dd * v) + boost;
  }
  return log(dd) + boost;
}

static double beta_draw(ndraw* d, double a, double b) {
  const double lx = log_gamma_draw(d, a), ly = log_gamma_draw(d, b);
  return 1.0 / (1.0 + exp(ly - lx));
}

/* Binomial(n, p): inversion for n*min(p,1-p) < 10, else BTRS (Hormann 1993) */
static double binomial_draw(ndraw* d, double n, double p) {
  if (n <= 0.0 || p <= 0.0) return 0.0;
  if (p >= 1.0) return n;
  const int flip = p > 0.5;
  const double pp = flip ? 1.0 - p : p, qq = 1.0 - pp;
  double k;
  if (n * pp < 10.0) {
    const double u = dr_uniform(d);
    double pmf = exp(n * log1p(-pp)), cdf = pmf;
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
    const double vr = 0.92 - 4.2 / bb, alpha = (2.83 + 5.1 / bb) * spq;
    const double lpq = log(pp / qq), m = floor((n + 1.0) * pp);
    const double h = o_lgamma(m + 1.0) + o_lgamma(n - m + 1.0);
    k = floor(cc);
    for (int it = 0; it < 256; it++) {
      const double u = dr_uniform(d) - 0.5, v = dr_uniform(d);
      const double us = 0.5 - fabs(u);
      const double kk = floor((2.0 * aa / us + bb) * u + cc);
      if (kk < 0.0 || kk > n) continue;
      if (us >= 0.07 && v <= vr) {
        k = kk;
        break;
      }
      const double lv = log(v * alpha / (aa / (us * us) + bb));
      if (lv <= h - o_lgamma(kk + 1.0) - o_lgamma(n - kk + 1.0) + (kk - m) * lpq) {
        k = kk;
        break;
      }
    }
  }
  return flip ? n - k : k;
}

/* frac = obs / N of predictive draw s at all-position column i (|z|-1 = k) */
static double predictive_frac(const nstream* st, int s, int i, int k, double Nn, const double th[4], int pmd) {
  double D = pmd ? th[1] * pow(1.0 - th[0], (double)k) + th[2] : th[0];
  D = D < 0.0 ? 0.0 : (D > 1.0 ? 1.0 : D);
  ndraw d = {st, 0xFFFD0000u + (uint32_t)s, (uint32_t)i << 16, 0.0, 0.0, 0, 0};
  const double p = beta_draw(&d, D * th[3], (1.0 - D) * th[3]);
  const double obs = binomial_draw(&d, Nn, p);
  return obs / Nn; /* 0/0 -> NaN like numpy */
}

static int cmp_double(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  if (isnan(x)) return isnan(y) ? 0 : 1;
  if (isnan(y)) return -1;
  return (x > y) - (x < y);
}

/* np.median and numpyro.diagnostics.hpdi(prob=0.68) of n values (sorted in place) */
static void median_hpdi(double* v, int n, double out3[3]) {
  qsort(v, (size_t)n, sizeof(double), cmp_double);
  int anynan = 0;
  for (int i = 0; i < n; i++) anynan |= isnan(v[i]);
  if (anynan) {
    out3[0] = out3[1] = out3[2] = NAN;
    return;
  }
  out3[0] = (n & 1) ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2]);
  const int len = (int)(0.68 * n);
  int best = 0;
  double bw = INFINITY;
  for (int i = 0; i < n - len; i++) {
    const double w = v[i + len] - v[i];
    if (w < bw) {
      bw = w;
      best = i;
    }
  }
  out3[1] = v[best];
  out3[2] = v[best + len];
}

/* pointwise log-likelihood incl. log C(N,y) (numpyro log_likelihood, fits.py:126-141) */
static double point_loglik(double yy, double nn, double D, double phi) {
  const double a = D * phi, b = (1.0 - D) * phi;
  return o_lgamma(nn + 1.0) - o_lgamma(yy + 1.0) - o_lgamma(nn - yy + 1.0) + o_lgamma(yy + a) - o_lgamma(a) +
         o_lgamma(nn - yy + b) - o_lgamma(b) - o_lgamma(nn + phi) + o_lgamma(a + b);
}

/* waic_i over the points [lo, hi) of one chain's samples (fits.py:147-172) */
static void waic_points(const uint32_t* y, const uint32_t* N, int lo, int hi, int pmd, const double* smp, int S,
                        double* waic_out /* [hi-lo] */) {
  double* lp = (double*)malloc(sizeof(double) * (size_t)S);
  for (int i = lo; i < hi; i++) {
    const int k = kpos(i);
    double mx = -INFINITY;
    for (int s = 0; s < S; s++) {
      const double* th = smp + 4 * s;
      double D = pmd ? th[1] * pow(1.0 - th[0], (double)k) + th[2] : th[0];
      D = D < 0.0 ? 0.0 : (D > 1.0 ? 1.0 : D);
      lp[s] = point_loglik((double)y[i], (double)N[i], D, th[3]);
      if (lp[s] > mx) mx = lp[s];
    }
    double se = 0, mean = 0;
    for (int s = 0; s < S; s++) {
      se += exp(lp[s] - mx);
      mean += lp[s];
    }
    mean /= S;
    double var = 0;
    for (int s = 0; s < S; s++) var += (lp[s] - mean) * (lp[s] - mean);
    var /= S;
    const double lppd = mx + log(se) - log((double)S);
    waic_out[i - lo] = -2.0 * (lppd - var);
  }
  free(lp);
}

/* n_sigma / asymmetry of mdfit_oracle.c take pointwise log-likelihoods
 * (waic_i = -2 ell_i); with samples waic_i is given, so pass -waic_i / 2 */
static void nuts_taxon(const uint32_t* y, const uint32_t* N, const uint32_t* mm, const mdfit_opts* o, int64_t g,
                       double* out, float* pred, int32_t* status, double* samples_out /* [6][S][4] or NULL */) {
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
  const int S = o->num_samples;
  double* smp = samples_out ? samples_out : (double*)malloc(sizeof(double) * 6 * 4 * (size_t)S);
  int st = MDFIT_OK;
  for (int j = 0; j < MDFIT_NOUT; j++) out[j] = 0.0;
  for (int s = 0; s < 6; s++) {
    nctx cx = {models[s], los[s], his[s], y, N};
    nstream ns = nstream_make(o->seed, g, s);
    nchain_stats cs;
    nuts_chain(&cx, &ns, o->num_warmup, S, smp + (size_t)s * 4 * S, &cs);
    if (cs.status > st) st = cs.status;
    double m[4] = {0, 0, 0, 0};
    for (int k = 0; k < S; k++)
      for (int j = 0; j < 4; j++) m[j] += smp[(size_t)s * 4 * S + 4 * k + j];
    double* dg = out + MDFIT_F_DIAG + MDFIT_DIAG_STRIDE * s;
    for (int j = 0; j < 4; j++) dg[j] = m[j] / S; /* posterior means of q, A, c, phi */
    dg[4] = cs.step;
    dg[5] = cs.leap;
    dg[6] = cs.status;
    dg[7] = cs.div;
  }
  if (st != MDFIT_OK) {
    for (int j = 0; j < MDFIT_NRESULT; j++) out[j] = NAN;
    if (pred)
      for (int j = 0; j < 3 * NPOS; j++) pred[j] = NAN;
    *status = st;
    if (!samples_out) free(smp);
    return;
  }
  const double* sP = smp;
  const double* sN = smp + 4 * (size_t)S;
  const double* sPf = smp + 8 * (size_t)S;
  const double* sPr = smp + 12 * (size_t)S;
  const double* sNf = smp + 16 * (size_t)S;
  const double* sNr = smp + 20 * (size_t)S;
  double wP[NPOS], wN[NPOS], wPf[NHALF], wPr[NHALF], wNf[NHALF], wNr[NHALF];
  waic_points(y, N, 0, NPOS, 1, sP, S, wP);
  waic_points(y, N, 0, NPOS, 0, sN, S, wN);
  waic_points(y, N, 0, NHALF, 1, sPf, S, wPf);
  waic_points(y, N, NHALF, NPOS, 1, sPr, S, wPr);
  waic_points(y, N, 0, NHALF, 0, sNf, S, wNf);
  waic_points(y, N, NHALF, NPOS, 0, sNr, S, wNr);
  double lP[NPOS], lN[NPOS], lC[NPOS];
  for (int i = 0; i < NPOS; i++) {
    lP[i] = -0.5 * wP[i];
    lN[i] = -0.5 * wN[i];
    lC[i] = -0.5 * (i < NHALF ? wPf[i] : wPr[i - NHALF]);
  }
  double lnf[NHALF], lpf[NHALF], lnr[NHALF], lpr[NHALF];
  for (int i = 0; i < NHALF; i++) {
    lpf[i] = -0.5 * wPf[i];
    lnf[i] = -0.5 * wNf[i];
    lpr[i] = -0.5 * wPr[i];
    lnr[i] = -0.5 * wNr[i];
  }
  out[MDFIT_F_N_SIGMA] = n_sigma(lP, lN, NPOS);
  out[MDFIT_F_N_SIGMA_FORWARD] = n_sigma(lpf, lnf, NHALF);
  out[MDFIT_F_N_SIGMA_REVERSE] = n_sigma(lpr, lnr, NHALF);
  out[MDFIT_F_ASYMMETRY] = asymmetry(lP, lC, lC);
  /* means (fits.py:266-270, 329, 350) */
  double mq = 0, mphi = 0, mdm = 0, mqf = 0, mqr = 0;
  for (int k = 0; k < S; k++) {
    mq += sP[4 * k];
    mphi += sP[4 * k + 3];
    mdm += sP[4 * k + 1] + sP[4 * k + 2];
    mqf += sPf[4 * k];
    mqr += sPr[4 * k];
  }
  out[MDFIT_F_Q_MEAN] = mq / S;
  out[MDFIT_F_CONCENTRATION_MEAN] = mphi / S;
  out[MDFIT_F_D_MAX_MARGINALIZED_MEAN] = mdm / S;
  out[MDFIT_F_Q_MEAN_FORWARD] = mqf / S;
  out[MDFIT_F_Q_MEAN_REVERSE] = mqr / S;
  /* posterior predictive (fits.py:89-120) */
  double* v = (double*)malloc(sizeof(double) * (size_t)S);
  double p3[3];
  for (int i = 0; i < NPOS; i++) {
    nstream ns = nstream_make(o->seed, g, 0);
    for (int k = 0; k < S; k++) v[k] = predictive_frac(&ns, k, i, kpos(i), (double)N[i], sP + 4 * k, 1);
    median_hpdi(v, S, p3);
    if (pred)
      for (int r = 0; r < 3; r++) pred[r * NPOS + i] = (float)p3[r];
    if (i == 0) {
      out[MDFIT_F_D_MAX] = p3[0];
      out[MDFIT_F_D_MAX_LOWER_HPDI] = p3[1];
      out[MDFIT_F_D_MAX_UPPER_HPDI] = p3[2];
    }
  }
  {
    nstream ns = nstream_make(o->seed, g, 2);
    for (int k = 0; k < S; k++) v[k] = predictive_frac(&ns, k, 0, 0, (double)N[0], sPf + 4 * k, 1);
    median_hpdi(v, S, p3);
    out[MDFIT_F_D_MAX_FORWARD] = p3[0];
  }
  {
    /* the reverse fit's predictive on data_forward (fits.py:343-348) */
    nstream ns = nstream_make(o->seed, g, 3);
    for (int k = 0; k < S; k++) v[k] = predictive_frac(&ns, k, 0, 0, (double)N[0], sPr + 4 * k, 1);
    median_hpdi(v, S, p3);
    out[MDFIT_F_D_MAX_REVERSE] = p3[0];
  }
  free(v);
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
  if (!samples_out) free(smp);
}

/* Host batch of the sampling mode; samples (optional) = double[T][6][S][4] */
int oracle_nuts_batch(const uint32_t* y, const uint32_t* N, const uint32_t* mm, int64_t n_taxa,
                      const mdfit_opts* opts, double* out, float* pred, int32_t* status, double* samples,
                      int n_threads) {
  mdfit_opts o = *opts;
#ifdef _OPENMP
  int nt = n_threads > 0 ? n_threads : omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#endif
  for (int64_t t = 0; t < n_taxa; t++) {
    nuts_taxon(y + t * MDFIT_LD, N + t * MDFIT_LD, mm ? mm + t * NPOS * MDFIT_NMM : NULL, &o, o.index_base + t,
               out + t * MDFIT_NOUT, pred ? pred + t * MDFIT_NPRED * NPOS : NULL, status + t,
               samples ? samples + (size_t)t * 6 * 4 * o.num_samples : NULL);
  }
  return 0;
}

/* one chain (tests): samples[S][4], stats[4] = (step, divergences, leapfrogs/iter, accept) */
int oracle_nuts_chain(int model, int subset, const uint32_t* y, const uint32_t* N, uint64_t seed, int64_t g,
                      int sub, int nwarm, int nsamp, double* samples, double* stats4) {
  nctx cx = {model, subset == 2 ? NHALF : 0, subset == 1 ? NHALF : NPOS, y, N};
  nstream ns = nstream_make(seed, g, sub);
  nchain_stats cs;
  nuts_chain(&cx, &ns, nwarm, nsamp, samples, &cs);
  stats4[0] = cs.step;
  stats4[1] = cs.div;
  stats4[2] = cs.leap;
  stats4[3] = cs.acc;
  return cs.status;
}

/* predictive fractions of the draws th[S][4] at all-position column col
 * (|z|-1 = k, N = Nn) on stream (seed, g, sub) -- for tests of the median /
 * HPDI step */
void oracle_nuts_predictive(uint64_t seed, int64_t g, int sub, int col, int k, double Nn, const double* th, int S,
                            double* frac, double* med_lo_hi) {
  nstream ns = nstream_make(seed, g, sub);
  for (int s = 0; s < S; s++) frac[s] = predictive_frac(&ns, s, col, k, Nn, th + 4 * s, 1);
  double* v = (double*)malloc(sizeof(double) * (size_t)S);
  memcpy(v, frac, sizeof(double) * (size_t)S);
  median_hpdi(v, S, med_lo_hi);
  free(v);
}
