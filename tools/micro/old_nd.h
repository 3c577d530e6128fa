__device__ __forceinline__ bool newton_dir_old(bool pmd, const double u[4], const double g[4],
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
  if (!ok) {  // indefinite: shift the diagonal by 1e-10 * scale, x10 per retry
    double sc = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (fr[j]) sc = fmax(sc, fabs(H[hidx(j, j)]));
    if (sc == 0.0) sc = 1.0;
    double mu = 1e-10 * sc;
    for (int attempt = 1; attempt < 40 && !ok; ++attempt, mu *= 10.0) ok = chol4(fr, H, mu, L, iL) < 0;
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
      for (int p = 0; p < j; ++p) s -= L[hidx(p, j)] * z[p];
      z[j] = s * iL[j];
    }
#pragma unroll
    for (int j = 3; j >= 0; --j) {  // L^T d = z
      double s = z[j];
#pragma unroll
      for (int p = j + 1; p < 4; ++p) s -= L[hidx(j, p)] * d[p];
      d[j] = s * iL[j];
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
  return indef;
}
