"""Generate the scipy-pinned golden vectors (run here, output committed).

    python tests/golden/make_golden_scipy.py

Writes tests/golden/scipy_golden.npz with
  (1) special-function known answers: scipy.special.gammaln / digamma /
      polygamma(1, .) on a log-spaced grid (the kernel's lgamma/digamma/trigamma);
  (2) beta-binomial log-pmf + d/dalpha, d/dbeta known answers from
      scipy.stats.betabinom.logpmf (numpyro's BetaBinomial.log_prob, used by
      /root/reference/metadamage/fits.py:59,67, is the same formula);
      extremes N in {0, 1, 1e9}, y in {0, N}, alpha, beta in [1e-3, 1e6];
  (3) MAP goldens: the MDFIT-MAP v1 objective restated here in
      numpy/scipy (independent of oracle/ and the kernel) and minimised by
      scipy.optimize (L-BFGS-B from 7 starts incl. the spec's initial point,
      then a finite-difference-Hessian Newton polish; best objective kept) for the 6
      taxa of the reference's fixture files + 120 seeded synthetic taxa.

Nothing here imports the reference.
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
from scipy import optimize, special, stats

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from metadamage_amd.synthetic import NHALF, NPOS, abs_z, generate  # noqa: E402

# u = (logit q, logit A, c, log delta): the box of MDFIT-MAP v1
U_LO = np.array([-25.0, -25.0, 0.0, -25.0])
U_HI = np.array([25.0, 25.0, 0.999, 20.0])


def objective(u, model, y, N, lo, hi):
    """F(u) = -(sum_i ell_i + log prior) of MDFIT-MAP v1, with gradient.

    model_PMD / model_null of fits.py:43-67 with theta = (q, A, c, delta):
    q, A = sigmoid(u), c = u_c, delta = exp(u_delta), phi = delta + 2; the log
    prior is Beta(2,3)(q) [Beta(2,3)(A), Beta(1,9)(c)], Exponential(1/1000)(delta)
    without the Jacobian (a mode of the constrained density).
    """
    y = y[lo:hi].astype(float)
    N = N[lo:hi].astype(float)
    k = (abs_z() - 1)[lo:hi].astype(float)
    q = special.expit(u[0])
    delta = np.exp(u[3])
    phi = delta + 2.0
    if model == 0:
        A = special.expit(u[1])
        c = u[2]
        if A + c >= 1.0:
            return np.inf, np.zeros(4)
        w = (1.0 - q) ** k
        D = A * w + c
        dD = np.stack([-A * k * (1.0 - q) ** np.maximum(k - 1, 0) * (k > 0), w, np.ones_like(w)])
    else:
        A = c = 0.0
        D = np.full_like(y, q)
        dD = np.stack([np.ones_like(y), np.zeros_like(y), np.zeros_like(y)])
    a = D * phi
    b = (1.0 - D) * phi
    ell = (
        special.gammaln(y + a) + special.gammaln(N - y + b) - special.gammaln(N + phi)
        - special.gammaln(a) - special.gammaln(b) + special.gammaln(phi)
    )
    Pa = special.digamma(y + a) - special.digamma(a)
    Pb = special.digamma(N - y + b) - special.digamma(b)
    lD = phi * (Pa - Pb)
    lF = D * Pa + (1 - D) * Pb + special.digamma(phi) - special.digamma(N + phi)
    g_theta = np.array([np.sum(lD * dD[0]), np.sum(lD * dD[1]), np.sum(lD * dD[2]), np.sum(lF)])
    lp = np.log(q) + 2 * np.log1p(-q) - delta / 1000.0
    gp = np.array([1 - 3 * q, 0.0, 0.0, -delta / 1000.0])
    J = np.array([q * (1 - q), A * (1 - A), 1.0, delta])
    if model == 0:
        lp += np.log(A) + 2 * np.log1p(-A) + 8 * np.log1p(-c)
        gp[1] = 1 - 3 * A
        gp[2] = -8 / (1 - c)
    F = -(ell.sum() + lp)
    g = -(J * g_theta + gp)
    if model == 1:
        g[1] = g[2] = 0.0
    return F, g


def spec_init(model, y, N, lo, hi):
    """Initial point of MDFIT-MAP v1, restated: pooled ratios
    r(S) = (sum y + 0.5)/(sum N + 1) over |z| = 1, |z| = 2 and |z| >= 10."""
    k = (abs_z() - 1)[lo:hi]
    yy = y[lo:hi].astype(float)
    NN = N[lo:hi].astype(float)

    def r(mask):
        return (yy[mask].sum() + 0.5) / (NN[mask].sum() + 1.0)

    if model == 1:
        q0 = np.clip(r(np.ones_like(k, bool)), 1e-4, 0.9)
        return np.array([special.logit(q0), 0.0, 0.0, np.log(100.0)])
    c0 = np.clip(r(k >= 9), 1e-4, 0.3)
    r1, r2 = r(k == 0), r(k == 1)
    A0 = np.clip(r1 - c0, 1e-3, 0.9 * (1 - c0))
    q0 = np.clip(1 - (r2 - c0) / (r1 - c0), 0.05, 0.95) if r1 - c0 > 1e-3 else 1.0 / 3.0
    return np.array([special.logit(q0), special.logit(A0), c0, np.log(100.0)])


def _newton_polish(fun, x, lo, hi, iters=60):
    """Bounded Newton with a finite-difference Hessian of the analytic
    gradient (independent of the oracle's analytic Hessian)."""
    F, g = fun(x)
    for _ in range(iters):
        n = len(x)
        H = np.zeros((n, n))
        for j in range(n):
            h = 1e-5 * max(1.0, abs(x[j]))
            e = np.zeros(n)
            e[j] = h
            H[:, j] = (fun(np.clip(x + e, lo, hi))[1] - fun(np.clip(x - e, lo, hi))[1]) / (2 * h)
        H = 0.5 * (H + H.T)
        act = ((x <= lo) & (g > -1e-8)) | ((x >= hi) & (g < 1e-8))
        fr = ~act
        d = np.zeros(n)
        if fr.any():
            Hf = H[np.ix_(fr, fr)]
            mu = 0.0
            for _t in range(40):
                try:
                    np.linalg.cholesky(Hf + mu * np.eye(fr.sum()))
                    break
                except np.linalg.LinAlgError:
                    mu = 1e-10 * np.abs(np.diag(Hf)).max() if mu == 0 else mu * 10
            d[fr] = np.linalg.solve(Hf + mu * np.eye(fr.sum()), -g[fr])
        if np.abs(d).max() > 4:
            d *= 4 / np.abs(d).max()
        t = 1.0
        while t > 1e-12:
            xn = np.clip(x + t * d, lo, hi)
            Fn, gn = fun(xn)
            if Fn < F or (Fn <= F + 1e-12 * abs(F) and np.abs(gn).max() < np.abs(g).max()):
                break
            t *= 0.5
        if t <= 1e-12:
            break
        x, F, g = xn, Fn, gn
        if np.abs(t * d).max() < 1e-11:
            break
    return F, x


def map_fit(model, y, N, lo, hi, starts):
    """Multi-start bounded L-BFGS-B + Newton polish; returns best (F, u).
    The spec's own initial point is always one of the starts."""
    best = (np.inf, None)
    free = [0, 1, 2, 3] if model == 0 else [0, 3]
    for u0 in [spec_init(model, y, N, lo, hi)] + list(starts):
        u0 = np.asarray(u0, float)

        def fun(v):
            u = u0.copy()
            u[free] = v
            F, g = objective(u, model, y, N, lo, hi)
            if not np.isfinite(F):
                return 1e300, np.zeros(len(free))
            return F, g[free]

        bounds = list(zip(U_LO[free], U_HI[free]))
        res = optimize.minimize(fun, u0[free], jac=True, method="L-BFGS-B", bounds=bounds,
                                options=dict(maxiter=20000, maxfun=40000, ftol=1e-16, gtol=1e-12))
        F, x = _newton_polish(fun, res.x, U_LO[free], U_HI[free])
        if F < best[0]:
            u = u0.copy()
            u[free] = x
            best = (float(F), u)
    return best


def starts_for(model):
    """Fixed extra starts (besides the spec's initial point)."""
    rng = np.random.default_rng(7)
    base = [[-0.7, -2.0, 0.02, np.log(100.0)], [0.0, -4.0, 0.002, np.log(1000.0)],
            [1.0, -1.0, 0.05, np.log(20.0)], [-4.0, -3.0, 0.0, np.log(5000.0)]]
    for _ in range(2):
        base.append([rng.uniform(-6, 2), rng.uniform(-5, -0.5), rng.uniform(0.0, 0.1), rng.uniform(1, 9)])
    if model == 1:
        base = [[b[0], 0.0, 0.0, b[3]] for b in base]
    return base


def fixture_taxa():
    """The 6 taxa of data/input/data_{ancient,control}.txt packed as in
    fits.py:398-419 (rows fwd z=1..15 then rev z=-1..-15), from the committed
    reference-generated golden (tests/golden/reference_golden.npz)."""
    g = np.load(ROOT / "tests/golden/reference_golden.npz")
    out = []
    for name in ("data_ancient", "data_control"):
        out.append((g[f"{name}__y"], g[f"{name}__N"]))
    y = np.concatenate([o[0] for o in out])
    N = np.concatenate([o[1] for o in out])
    return y, N


def main():
    rng = np.random.default_rng(12345)
    res = {}
    # (1) special functions
    x = np.concatenate([np.logspace(-6, 10, 400), rng.uniform(0.01, 30, 200), [0.5, 1.0, 2.0, 10.0, 12.0]])
    res["special_x"] = x
    res["special_lgamma"] = special.gammaln(x)
    res["special_digamma"] = special.digamma(x)
    res["special_trigamma"] = special.polygamma(1, x)
    # (2) beta-binomial
    Ns = np.concatenate([[0, 0, 1, 1, 1e9, 1e9, 1e9], rng.integers(1, 10**7, 193).astype(float)])
    ys = np.concatenate([[0, 0, 0, 1, 0, 1e9, 5e8], np.floor(rng.uniform(0, 1, 193) * Ns[7:])])
    al = np.concatenate([[1e-3, 1e6, 1.0, 1e-3, 1e6, 1e-3, 2.5], np.exp(rng.uniform(np.log(1e-3), np.log(1e6), 193))])
    be = np.concatenate([[1e6, 1e-3, 1.0, 1e6, 1e-3, 1e6, 7.5], np.exp(rng.uniform(np.log(1e-3), np.log(1e6), 193))])
    res["bb_y"], res["bb_N"], res["bb_a"], res["bb_b"] = ys, Ns, al, be
    res["bb_logpmf"] = stats.betabinom.logpmf(ys, Ns, al, be)
    ps = special.digamma(al + be) - special.digamma(Ns + al + be)
    res["bb_dalpha"] = special.digamma(ys + al) - special.digamma(al) + ps
    res["bb_dbeta"] = special.digamma(Ns - ys + be) - special.digamma(be) + ps

    # (3) MAP goldens
    yf, Nf = fixture_taxa()
    b = generate(120, seed=11)
    y = np.concatenate([yf, b.y[:, :NPOS]]).astype(np.uint32)
    N = np.concatenate([Nf, b.N[:, :NPOS]]).astype(np.uint32)
    T = y.shape[0]
    subsets = [(0, 0, NPOS), (1, 0, NPOS), (0, 0, NHALF), (0, NHALF, NPOS), (1, 0, NHALF), (1, NHALF, NPOS)]
    U = np.zeros((T, 6, 4))
    F = np.zeros((T, 6))
    for t in range(T):
        for s, (model, lo, hi) in enumerate(subsets):
            F[t, s], U[t, s] = map_fit(model, y[t], N[t], lo, hi, starts_for(model))
        if t % 10 == 0:
            print(f"MAP golden {t}/{T}", flush=True)
    res["map_y"], res["map_N"], res["map_u"], res["map_F"] = y, N, U, F
    np.savez_compressed(ROOT / "tests/golden/scipy_golden.npz", **res)
    print("wrote tests/golden/scipy_golden.npz")


if __name__ == "__main__":
    main()
