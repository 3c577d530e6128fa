"""CPU baseline in the reference's own dispatch shape (CPU
baseline item 2): a Python restatement of the per-taxon fit -- scipy L-BFGS-B
on the MDFIT-MAP v1 objective with its analytic gradient, 6
sub-fits per taxon plus the pointwise log-likelihoods and n_sigma / asymmetry
-- dispatched like fits.py:569-626 / 692-706: a multiprocessing Pool per
1,000-taxon chunk, one task per taxon.  numpyro itself is not installed, so
this is the closest runnable stand-in for the reference's CPU path; its rate on
a 1,000-taxon sample is extrapolated and labelled as such.

    python tools/cpu_reference_dispatch.py [--taxa 1000] [--cores 16]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from multiprocessing import Pool
from pathlib import Path

import numpy as np
from scipy.optimize import minimize
from scipy.special import digamma, gammaln

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

LO = np.array([-25.0, -25.0, 0.0, -25.0])
HI = np.array([25.0, 25.0, 0.999, 20.0])
K = np.r_[np.arange(15), np.arange(15)]  # |z| - 1 of the 30 positions


def _theta(u, pmd):
    q = 1.0 / (1.0 + np.exp(-u[0]))
    A = 1.0 / (1.0 + np.exp(-u[1])) if pmd else 0.0
    c = u[2] if pmd else 0.0
    delta = np.exp(u[3])
    return q, A, c, delta


def objective(u, y, N, k, pmd):
    """F(u) = -(sum_i ell_i + ln p(theta)) and dF/du."""
    q, A, c, delta = _theta(u, pmd)
    if pmd and A + c >= 1.0:
        return np.inf, np.zeros(4)
    phi = delta + 2.0
    w = (1.0 - q) ** k
    D = A * w + c if pmd else np.full_like(y, q)
    a, b = D * phi, (1.0 - D) * phi
    ell = gammaln(y + a) - gammaln(a) + gammaln(N - y + b) - gammaln(b) - gammaln(N + phi) + gammaln(phi)
    lp = np.log(q) + 2.0 * np.log1p(-q) - delta / 1000.0
    if pmd:
        lp += np.log(A) + 2.0 * np.log1p(-A) + 8.0 * np.log1p(-c)
    F = -(ell.sum() + lp)
    Pa = digamma(y + a) - digamma(a)
    Pb = digamma(N - y + b) - digamma(b)
    dl_dD = phi * (Pa - Pb)
    dl_dphi = D * Pa + (1.0 - D) * Pb + digamma(phi) - digamma(N + phi)
    g = np.zeros(4)
    if pmd:
        dD_dq = np.where(k > 0, -A * k * w / (1.0 - q), 0.0)
        g[0] = (dl_dD * dD_dq).sum() + (1.0 / q - 2.0 / (1.0 - q))
        g[1] = (dl_dD * w).sum() + (1.0 / A - 2.0 / (1.0 - A))
        g[2] = dl_dD.sum() - 8.0 / (1.0 - c)
    else:
        g[0] = dl_dD.sum() + (1.0 / q - 2.0 / (1.0 - q))
    g[3] = dl_dphi.sum() - 1.0 / 1000.0
    g[0] *= q * (1.0 - q)
    if pmd:
        g[1] *= A * (1.0 - A)
    g[3] *= delta
    return F, -g


def _u0(y, N, k, pmd):
    """Initial point."""
    def r(m):
        return (y[m].sum() + 0.5) / (N[m].sum() + 1.0)

    allm = np.ones_like(y, dtype=bool)
    if not pmd:
        q0 = np.clip(r(allm), 1e-4, 0.9)
        return np.array([np.log(q0 / (1 - q0)), 0.0, 0.0, np.log(100.0)])
    c0 = np.clip(r(k >= 9), 1e-4, 0.3)
    r1, r2 = r(k == 0), r(k == 1)
    A0 = np.clip(r1 - c0, 1e-3, 0.9 * (1 - c0))
    q0 = 1.0 / 3.0 if r1 - c0 <= 1e-3 else np.clip(1 - (r2 - c0) / (r1 - c0), 0.05, 0.95)
    return np.array([np.log(q0 / (1 - q0)), np.log(A0 / (1 - A0)), c0, np.log(100.0)])


def fit_taxon(args):
    y30, N30 = args
    y30, N30 = y30.astype(float), N30.astype(float)
    ells = {}
    for pmd in (True, False):
        for name, sl in (("all", slice(0, 30)), ("fwd", slice(0, 15)), ("rev", slice(15, 30))):
            y, N, k = y30[sl], N30[sl], K[sl]
            bounds = list(zip(LO, HI)) if pmd else [(LO[0], HI[0]), (0, 0), (0, 0), (LO[3], HI[3])]
            res = minimize(objective, _u0(y, N, k, pmd), args=(y, N, k, pmd), jac=True, method="L-BFGS-B",
                           bounds=bounds, options={"maxiter": 200})
            q, A, c, delta = _theta(res.x, pmd)
            phi = delta + 2.0
            D = A * (1 - q) ** k + c if pmd else np.full_like(y, q)
            a, b = D * phi, (1 - D) * phi
            ells[(pmd, name)] = (gammaln(y + a) - gammaln(a) + gammaln(N - y + b) - gammaln(b)
                                 - gammaln(N + phi) + gammaln(phi))
    # n_sigma and asymmetry (fits.py:194-227) on the modes' waic_i = -2 ell_i
    d = -2 * ells[(True, "all")] + 2 * ells[(False, "all")]
    n_sigma = -d.sum() / np.sqrt(len(d) * d.var())
    fr = np.r_[ells[(True, "fwd")], ells[(True, "rev")]]
    dc = -2 * ells[(True, "all")] + 2 * fr
    asym = -dc.sum() / np.sqrt(len(dc) * dc.var())
    return n_sigma, asym


def measure(taxa: int = 1000, cores: int = 16) -> dict:
    """The reference-dispatch-shape rate on the first `taxa` taxa of C2."""
    from metadamage_amd.synthetic import generate

    b = generate(max(taxa, 1), seed=1)  # C2's workload (seed 1); its first taxa
    tasks = [(b.y[i, :30], b.N[i, :30]) for i in range(taxa)]
    t0 = time.perf_counter()
    out = []
    for lo in range(0, taxa, 1000):  # a new Pool per 1,000-taxon chunk, as fits.py:692-706
        with Pool(cores) as pool:
            out += pool.map(fit_taxon, tasks[lo:lo + 1000])
    dt = time.perf_counter() - t0
    return {
        "kind": "python-restatement in the reference's dispatch shape (Pool per 1,000-taxon chunk, scipy "
                "L-BFGS-B MAP per sub-fit); numpyro itself is not installed",
        "value": round(taxa / dt, 2), "unit": "fits/s", "cores": cores,
        "sample": f"the first {taxa} taxa of C2 (seed 1), {dt:.2f} s including Pool start-up; extrapolated rate",
        "finite_n_sigma": float(np.isfinite([o[0] for o in out]).mean()),
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", type=int, default=1000)
    ap.add_argument("--cores", type=int, default=min(16, os.cpu_count() or 1))
    a = ap.parse_args()
    print(json.dumps(measure(a.taxa, a.cores)), flush=True)


if __name__ == "__main__":
    main()
