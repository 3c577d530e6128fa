"""CPU tests of the sampling-mode oracle (MDFIT-NUTS v1, oracle/mdfit_nuts.c).

numpyro / jax cannot run here, so the sampler is pinned by:
  * Philox4x32-10 against the Random123 known-answer vectors;
  * the potential's analytic gradient against finite differences;
  * posterior means against an independent importance sampler (Student-t
    proposal at the Laplace approximation) on well-identified taxa;
  * the post-processing (WAIC, n_sigma, asymmetry, means, median / HPDI)
    recomputed from the oracle's own draws with the numpy restatements that
    tests/test_oracle_golden.py pins against the reference's functions.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest
from scipy.special import gammaln

from oracle import oracle as orc


def test_philox_known_answers(oracle_lib):
    # Random123 kat_vectors, philox4x32 R=10
    kat = [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
         [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
    ]
    for ctr, key, expect in kat:
        assert oracle_lib.philox(ctr, key).tolist() == expect


def _batch(n, seed):
    from metadamage_amd.synthetic import generate

    return generate(n, seed=seed)


def test_potential_gradient_matches_finite_differences(oracle_lib):
    b = _batch(12, 5)
    rng = np.random.default_rng(1)
    for t in range(12):
        for model, subset in ((0, 0), (1, 0), (0, 1), (0, 2), (1, 2)):
            v = rng.uniform(-2, 2, 4)
            if model == 1:
                v[1:3] = 0
            U, g = oracle_lib.nuts_potential(model, subset, b.y[t, :30], b.N[t, :30], v)
            if not np.isfinite(U):
                continue
            for j in ((0, 1, 2, 3) if model == 0 else (0, 3)):
                h = 1e-3

                def f(d):
                    return oracle_lib.nuts_potential(model, subset, b.y[t, :30], b.N[t, :30], v + d * np.eye(4)[j])[0]

                fd = (-f(2 * h) + 8 * f(h) - 8 * f(-h) + f(-2 * h)) / (12 * h)
                # U is a sum of lnGamma terms of up to |U| ~ 1e8: FD noise ~ ulp(U) / h
                tol = 1e-4 * max(1.0, abs(g[j])) + 200 * np.spacing(abs(U)) / h
                assert abs(fd - g[j]) <= tol, (t, model, subset, j, fd, g[j])


def test_infeasible_region_has_infinite_potential(oracle_lib):
    b = _batch(2, 5)
    v = np.array([0.0, 3.0, 3.0, 5.0])  # A = c = 0.95: A + c >= 1 -> D clipped to 1 (fits.py:50)
    U, g = oracle_lib.nuts_potential(0, 0, b.y[0, :30], b.N[0, :30], v)
    assert U == np.inf and (g == 0).all()


def _importance_posterior(oracle_lib, model, subset, y, N, draws, n=40000, seed=0):
    """Self-normalised importance sampling of the exact posterior with a
    Student-t proposal in v-space.  The proposal is only TUNED by the chain's
    draws (location, 1.5x scale); the weights use the exact density, so the
    estimate does not inherit the chain's errors."""
    act = [0, 1, 2, 3] if model == 0 else [0, 3]
    vd = np.stack([np.log(draws[:, 0] / (1 - draws[:, 0])),
                   np.log(draws[:, 1] / (1 - draws[:, 1])) if model == 0 else 0 * draws[:, 0],
                   np.log(draws[:, 2] / (1 - draws[:, 2])) if model == 0 else 0 * draws[:, 0],
                   np.log(draws[:, 3] - 2)], 1)[:, act]
    x, d = vd.mean(0), len(act)
    C = np.cov(vd.T).reshape(d, d) * 1.5**2
    L = np.linalg.cholesky(C)
    rng = np.random.default_rng(seed)
    df = 4
    X = x + (rng.standard_normal((n, d)) @ L.T) / np.sqrt(rng.chisquare(df, n) / df)[:, None]
    q = np.einsum("ni,ij,nj->n", X - x, np.linalg.inv(C), X - x)

    def U(xx):
        v = np.zeros(4)
        v[act] = xx
        return oracle_lib.nuts_potential(model, subset, y, N, v)[0]

    lw = -np.array([U(xx) for xx in X]) + (df + d) / 2 * np.log1p(q / df)
    w = np.exp(lw - lw.max())
    w /= w.sum()
    v = np.zeros((n, 4))
    v[:, act] = X
    sig = 1 / (1 + np.exp(-v))
    th = np.stack([sig[:, 0], sig[:, 1] if model == 0 else 0 * sig[:, 0], sig[:, 2] if model == 0 else 0 * sig[:, 0],
                   np.exp(v[:, 3]) + 2], 1)
    mean = w @ th
    return mean, np.sqrt(w @ (th - mean) ** 2), 1 / np.sum(w**2)


def _mcse(x, nb=20):
    m = len(x) // nb
    return x[: m * nb].reshape(nb, m).mean(1).std(ddof=1) / np.sqrt(nb)


def test_posterior_means_match_importance_sampling(oracle_lib):
    """NUTS (500 warmup + 1000 draws, the reference's settings) agrees with an
    independent importance sampler on taxa whose posteriors are well
    identified (ancient: A >> 0), within 5 combined standard errors."""
    b = _batch(60, 2)
    ancient = np.where(b.truth["ancient"] & (b.N[:, :30].sum(1) > 1e4))[0][:3]
    assert len(ancient) == 3
    zs = []
    for t in ancient:
        for model, subset, sub in ((0, 0, 0), (1, 0, 1), (0, 1, 2)):
            y, N = b.y[t, :30], b.N[t, :30]
            smp, stats, rc = oracle_lib.nuts_chain(model, subset, y, N, seed=0, g=int(t), sub=sub)
            assert rc == 0 and 0.6 < stats[3] <= 1.0  # mean acceptance near the 0.8 target
            m_is, sd_is, ess = _importance_posterior(oracle_lib, model, subset, y, N, smp)
            assert ess > 1000
            for j in ((0, 1, 2, 3) if model == 0 else (0, 3)):
                se = np.hypot(_mcse(smp[:, j]), sd_is[j] / np.sqrt(ess))
                zs.append(abs(smp[:, j].mean() - m_is[j]) / se)
    zs = np.array(zs)
    assert zs.max() < 5.0, zs
    assert np.median(zs) < 1.5, zs


def _loglik(y, N, th, k, pmd):
    D = th[:, 1] * (1 - th[:, 0]) ** k + th[:, 2] if pmd else th[:, 0]
    D = np.clip(D, 0, 1)
    a, b = D * th[:, 3], (1 - D) * th[:, 3]
    return (gammaln(N + 1) - gammaln(y + 1) - gammaln(N - y + 1) + gammaln(y + a) + gammaln(N - y + b)
            - gammaln(N + a + b) - gammaln(a) - gammaln(b) + gammaln(a + b))


def test_record_recomputed_from_the_draws(oracle_lib):
    """The oracle's WAIC-based fields and means equal the reference formulas
    (numpy restatements, pinned in test_oracle_golden.py) applied to its draws."""
    b = _batch(4, 7)
    out, pred, st, smp = oracle_lib.nuts_batch(b.y, b.N, b.mm, num_warmup=150, num_samples=400, keep_samples=True)
    assert (st == 0).all()
    cols = {0: range(30), 1: range(30), 2: range(15), 3: range(15, 30), 4: range(15), 5: range(15, 30)}
    for t in range(4):
        # (WAIC terms are lnGamma sums of ~1e6-1e8 that cancel: compare at 1e-7)
        d = {}
        for s, cc in cols.items():
            pmd = s in (0, 2, 3)
            lp = np.stack([_loglik(float(b.y[t, c]), float(b.N[t, c]), smp[t, s], c % 15, pmd) for c in cc], 1)
            d[s] = orc.lppd_and_waic(lp)
        r = out[t]
        np.testing.assert_allclose(r[1], orc.n_sigma(d[0], d[1]), rtol=1e-7, atol=1e-7)  # n_sigma
        np.testing.assert_allclose(r[15], orc.n_sigma(d[2], d[4]), rtol=1e-7, atol=1e-7)  # n_sigma_forward
        np.testing.assert_allclose(r[18], orc.n_sigma(d[3], d[5]), rtol=1e-7, atol=1e-7)  # n_sigma_reverse
        np.testing.assert_allclose(r[21], orc.asymmetry(d[0], d[2], d[3]), rtol=1e-7, atol=1e-7)
        np.testing.assert_allclose(r[4], smp[t, 0, :, 0].mean(), rtol=1e-12)  # q_mean
        np.testing.assert_allclose(r[5], smp[t, 0, :, 3].mean(), rtol=1e-12)  # concentration_mean
        np.testing.assert_allclose(r[6], (smp[t, 0, :, 1] + smp[t, 0, :, 2]).mean(), rtol=1e-12)
        np.testing.assert_allclose(r[17], smp[t, 2, :, 0].mean(), rtol=1e-12)  # q_mean_forward
        np.testing.assert_allclose(r[20], smp[t, 3, :, 0].mean(), rtol=1e-12)  # q_mean_reverse
        # predictive median / HPDI at z = +1 (fits.py:249-261) = numpy median / numpyro hpdi of the draws
        frac, m3 = oracle_lib.nuts_predictive(smp[t, 0], 0, 0, b.N[t, 0], seed=0, g=t, sub=0)
        lo, hi = orc.hpdi(frac, 0.68)
        assert (r[0], r[2], r[3]) == (np.median(frac), lo, hi) == tuple(m3)
        assert pred[t, 0, 0] == np.float32(r[0])
        # the reverse fit's D_max uses data_forward (fits.py:343-348)
        frac_r, m3r = oracle_lib.nuts_predictive(smp[t, 3], 0, 0, b.N[t, 0], seed=0, g=t, sub=3)
        assert r[19] == np.median(frac_r) == m3r[0]


def test_predictive_draws_follow_the_beta_binomial(oracle_lib):
    """obs / N of the predictive draws has the BetaBinomial(a, b, N) / N mean and variance."""
    S = 20000
    for A, q, c, phi, N in ((0.3, 0.4, 0.02, 50.0, 200), (0.01, 0.3, 0.01, 3000.0, 10**6), (0.0, 0.5, 0.002, 5.0, 30)):
        th = np.tile([q, A, c, phi], (S, 1))
        frac, _ = oracle_lib.nuts_predictive(th, 0, 0, N, seed=3, g=1, sub=0)
        D = A + c
        var = D * (1 - D) * (phi + N) / (N * (phi + 1))
        assert abs(frac.mean() - D) < 5 * np.sqrt(var / S)
        # the sample variance's relative standard error from the sample's own
        # kurtosis (the a = 0.01 case is heavy-tailed: ~0.14 at S = 20k)
        dev = frac - frac.mean()
        se = np.sqrt((np.mean(dev**4) / frac.var() ** 2 - 1.0) / S)
        assert abs(frac.var() / var - 1) < max(0.1, 4 * se)


def test_sharded_calls_draw_the_same_numbers(oracle_lib):
    """Streams are keyed by index_base + taxon: fitting taxa [3, 6) as their own
    call with index_base 3 reproduces those rows of the whole batch."""
    b = _batch(6, 9)
    kw = dict(num_warmup=40, num_samples=60)
    full = oracle_lib.nuts_batch(b.y, b.N, b.mm, **kw)[0]
    part = oracle_lib.nuts_batch(b.y[3:], b.N[3:], b.mm[3:], index_base=3, **kw)[0]
    np.testing.assert_array_equal(full[3:], part)
    other = oracle_lib.nuts_batch(b.y[3:], b.N[3:], b.mm[3:], index_base=0, **kw)[0]
    assert not np.array_equal(full[3:], other)


def test_invalid_input_status(oracle_lib):
    b = _batch(2, 9)
    y = b.y.copy()
    y[1, 4] = b.N[1, 4] + 1
    out, pred, st = oracle_lib.nuts_batch(y, b.N, b.mm, num_warmup=20, num_samples=20)
    assert st[1] == 3 and np.isnan(out[1]).all() and np.isnan(pred[1]).all()
    assert st[0] == 0


@pytest.mark.parametrize("nw,expect", [
    (500, [(0, 74), (75, 99), (100, 149), (150, 249), (250, 449), (450, 499)]),
    (100, [(0, 14), (15, 89), (90, 99)]),
    (10, [(0, 9)]),
])
def test_adaptation_windows(nw, expect):
    """Stan / numpyro build_adaptation_schedule, restated in numpy: the oracle
    and the kernel follow the same construction (mdfit_nuts.c adapt_windows)."""
    def schedule(n):
        if n < 20:
            return [(0, n - 1)]
        ib, tb, bw = 75, 50, 25
        if n < ib + tb + bw:
            ib, tb = int(0.15 * n), int(0.1 * n)
            bw = n - ib - tb
        out = [(0, ib - 1)]
        end, nsz, nst = n - tb, bw, ib
        while nst < end:
            cs, csz = nst, nsz
            if 3 * csz <= end - cs:
                nsz = 2 * csz
            else:
                csz = end - cs
            nst = cs + csz
            out.append((cs, nst - 1))
        out.append((end, n - 1))
        return out

    assert schedule(nw) == expect


def test_nuts_columns_fixture_reproduces(oracle_lib):
    """tests/golden/nuts_columns_oracle.npz (the GPU test's reference) is the
    committed oracle's output: two of its taxa re-run under one of its seeds."""
    g = np.load(Path(__file__).resolve().parent / "golden" / "nuts_columns_oracle.npz")
    si = 3
    out, _, st = oracle_lib.nuts_batch(g["y"][:2], g["N"][:2], g["mm"][:2], seed=int(g["seeds"][si]), threads=2)
    assert (st == g["status"][si][:2]).all()
    assert np.array_equal(out[:, :25], g["out"][si][:2], equal_nan=True)
