"""Golden vectors for the MAP predictive HPDI (MDFIT-HPDI v2), from scipy.

    python tests/golden/make_golden_hpdi.py      # writes tests/golden/hpdi_golden.npz

The reference reports numpyro.diagnostics.hpdi(obs / N, prob=0.68) over its
predictive draws (/root/reference/metadamage/fits.py:112-120, 260-261); the MAP
counterpart is the population version: the shortest window
of BetaBinomial(alpha, beta, N) holding >= 68 % of the mass.  Computed here
independently of the oracle and the kernel: scipy.stats.betabinom.pmf over the
support (the whole of it up to N = 3e6, else +-60 sd around the mean), sorted
by probability (a stable sort: ties keep the lower count first), cumulated
until >= 0.68; the window is [min, max] of the counts taken.  Only data
(inputs and expected windows) is written.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
from scipy import stats

ROOT = Path(__file__).resolve().parents[2]
MASS = 0.68


def hpdi_window(N: float, a: float, b: float) -> tuple[float, float]:
    """[lo, hi] (counts) of the shortest 68 % window of BetaBinomial(a, b, N)."""
    N = int(N)
    if N == 0:
        return np.nan, np.nan
    if N <= 3_000_000:
        y = np.arange(N + 1)
    else:
        phi = a + b
        mu = N * a / phi
        sd = np.sqrt(N * a * b * (phi + N) / (phi * phi * (phi + 1)))
        y = np.arange(max(0, int(mu - 60 * sd)), min(N, int(mu + 60 * sd)) + 1)
    p = stats.betabinom.pmf(y, N, a, b)
    order = np.argsort(-p, kind="stable")
    cs = np.cumsum(p[order])
    k = int(np.searchsorted(cs, MASS, side="left"))
    take = y[order[: k + 1]]
    return float(take.min()), float(take.max())


def cases(seed: int = 2026):
    rng = np.random.default_rng(seed)
    N, a, b = [], [], []

    def add(n, aa, bb):
        N.append(float(n))
        a.append(float(aa))
        b.append(float(bb))

    # hand-picked edges: tiny N, point-mass-like, near-flat (phi -> 2+),
    # mode at 0 / at N, symmetric, large N
    for n in (1, 2, 3, 5, 10, 30):
        for D, phi in ((0.01, 100.0), (0.5003, 2.5), (0.2, 10.0), (0.9, 50.0), (1e-5, 3.0)):
            add(n, D * phi, (1 - D) * phi)
    for n in (1000, 100_000, 2_500_000):
        for D, phi in ((1e-6, 20.0), (0.02, 2.01), (0.5003, 2.001), (0.3, 1e4), (0.97, 5.0), (0.001, 1e5),
                       (0.05, 40.0), (0.5003, 1e6)):
            add(n, D * phi, (1 - D) * phi)
    # random: the synthetic generator's ranges and wider
    for _ in range(260):
        n = np.floor(np.exp(rng.uniform(np.log(1), np.log(2.5e6))))
        D = np.exp(rng.uniform(np.log(1e-4), np.log(0.95)))
        phi = np.exp(rng.uniform(np.log(2.05), np.log(1e5)))
        add(n, D * phi, (1 - D) * phi)
    # two N beyond the full-support limit (the +-60 sd window)
    for D, phi in ((0.01, 300.0), (0.2, 50.0)):
        add(2.0e8, D * phi, (1 - D) * phi)
    return np.array(N), np.array(a), np.array(b)


def main():
    N, a, b = cases()
    lo = np.zeros_like(N)
    hi = np.zeros_like(N)
    for i in range(N.size):
        lo[i], hi[i] = hpdi_window(N[i], a[i], b[i])
    np.savez_compressed(ROOT / "tests/golden/hpdi_golden.npz", N=N, a=a, b=b, lo=lo, hi=hi)
    print(f"wrote tests/golden/hpdi_golden.npz ({N.size} cases)")


if __name__ == "__main__":
    main()
