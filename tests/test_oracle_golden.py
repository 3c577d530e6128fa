"""CPU tests: pin the oracle against the golden vectors (no GPU needed).

  * special functions and beta-binomial log-pmf vs scipy known answers;
  * the MAP mode of every sub-fit vs an independent scipy optimiser;
  * the per-taxon record vs the reference's own record assembly
    (compute_fit_results, fits.py:230-356) with MAP quantities injected;
  * WAIC / n_sigma / asymmetry restatements vs the reference's functions;
  * noise vs the reference's add_noise_estimates.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as orc
from tests.helpers import RTOL, mixed_rel, mm_from_counts_parquet, pack_golden


def test_oracle_special_functions(oracle_lib, scipy_golden):
    o = oracle_lib.special(scipy_golden["special_x"])
    for j, key in enumerate(("special_lgamma", "special_digamma", "special_trigamma")):
        ref = scipy_golden[key]
        err = np.abs(o[:, j] - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() < 1e-13, (key, err.max())


def test_oracle_betabinom_logpmf(oracle_lib, scipy_golden):
    from scipy.special import gammaln

    g = scipy_golden
    y, N, a, b = g["bb_y"], g["bb_N"], g["bb_a"], g["bb_b"]
    lp, grad = oracle_lib.betabinom_logpmf(y, N, a, b)
    mag = sum(np.abs(gammaln(v)) for v in (N + 1, y + 1, N - y + 1, y + a, N - y + b, N + a + b, a, b, a + b))
    assert (np.abs(lp - g["bb_logpmf"]) <= 1e-15 * mag + 1e-12).all()
    for j, key in enumerate(("bb_dalpha", "bb_dbeta")):
        assert (np.abs(grad[:, j] - g[key]) / np.maximum(1e-6, np.abs(g[key]))).max() < 1e-8


def _bb_cases(n=300, seed=0):
    """Beta-binomial points over the whole input range (N up to 4e9, phi up
    to 1e6): y spread over [0, N], near N D, and the ends 0 and N."""
    rng = np.random.default_rng(seed)
    N = np.floor(np.exp(rng.uniform(0, np.log(4e9), n)))
    phi = np.exp(rng.uniform(np.log(2.0), np.log(1e6), n))
    D = rng.uniform(1e-3, 0.9, n)
    y = np.concatenate([np.floor(N * rng.uniform(0, 1, n) ** 3), np.floor(N * D), 0 * N, N])
    rep = lambda v: np.tile(v, 4)  # noqa: E731
    return y, rep(N), rep(D * phi), rep((1 - D) * phi)


def test_oracle_full_logpmf_vs_mpmath(oracle_lib):
    """The record's pointwise log-likelihood (full log-pmf, cancellation-free
    long-double form) against 40-digit mpmath lnGamma sums of the same
    double inputs: within 1e-10 of max(1, |logpmf|) everywhere, where a plain
    double lnGamma sum carries up to ~1e-5 at N ~ 4e9."""
    mpmath = pytest.importorskip("mpmath")
    mpmath.mp.dps = 40
    y, N, a, b = _bb_cases()
    lg = mpmath.loggamma
    ref = np.array([float(lg(n_ + 1) - lg(y_ + 1) - lg(n_ - y_ + 1) + lg(y_ + a_) + lg(n_ - y_ + b_) - lg(n_ + a_ + b_)
                          - lg(a_) - lg(b_) + lg(a_ + b_))
                    for y_, n_, a_, b_ in ((mpmath.mpf(float(v)) for v in t) for t in zip(y, N, a, b))])
    got = oracle_lib.bb_logpmf_full(y, N, a, b)
    assert (np.abs(got - ref) / np.maximum(1.0, np.abs(ref))).max() < 1e-10


SUBSETS = [(0, 0), (1, 0), (0, 1), (0, 2), (1, 1), (1, 2)]  # (model, subset) of the 6 sub-fits


def test_oracle_map_vs_scipy_optimiser(oracle_lib, scipy_golden):
    """The oracle's Newton finds the same optimum as multi-start L-BFGS-B +
    finite-difference Newton polish (scipy) for 6 fixture + 120 synthetic taxa."""
    Y, NN, U, F = (scipy_golden[k] for k in ("map_y", "map_N", "map_u", "map_F"))
    worst_dF = 0.0
    for t in range(len(Y)):
        for s, (m, sub) in enumerate(SUBSETS):
            u, Fo, ev, st = oracle_lib.fit_subfit(m, sub, Y[t], NN[t])
            assert st == 0, (t, s, ev)
            # never worse than scipy beyond the objective's rounding scale
            tolF = 1e-12 * abs(F[t, s]) + 1e-9
            assert Fo <= F[t, s] + tolF, (t, s, Fo, F[t, s])
            worst_dF = max(worst_dF, abs(Fo - F[t, s]) / max(1.0, abs(F[t, s])))
            # parameters: q, A on logit scale, c absolute, phi on log scale
            assert np.abs(u[[0, 1, 3]] - U[t, s][[0, 1, 3]]).max() < 1e-4, (t, s, u, U[t, s])
            assert abs(u[2] - U[t, s][2]) < 1e-6
    assert worst_dF < 1e-12


def test_oracle_record_vs_reference_assembly(oracle_lib, ref_golden, ref_meta):
    from metadamage_amd._lib import RESULT_FIELDS

    keys = ref_meta["record_keys"][3:]
    for name in ("data_ancient", "data_control", "synthetic"):
        y, N = pack_golden(ref_golden, [name])
        mm = mm_from_counts_parquet(name)
        out, pred, st = oracle_lib.fit_batch(y, N, mm)
        rec = ref_golden[f"record_{name}__values"]
        n = rec.shape[0]
        assert (st[:n] == 0).all()
        for k in keys:
            if k == "N_alignments":
                continue
            rel = mixed_rel(out[:n, RESULT_FIELDS.index(k)], rec[:, keys.index(k)])
            assert rel.max() < RTOL, (name, k, rel.max())
        assert np.nanmax(mixed_rel(pred[:n, 0], ref_golden[f"record_{name}__median"])) < 1e-5
        hp = ref_golden[f"record_{name}__hpdi"]
        assert np.nanmax(mixed_rel(pred[:n, 1], hp[:, 0])) < 1e-5
        assert np.nanmax(mixed_rel(pred[:n, 2], hp[:, 1])) < 1e-5


def test_record_keys_are_the_engine_field_order(ref_meta):
    """Column order of fit_results (fits.py:244-293 + 317-356 + 374-376): the
    engine's record fields are the reference's numeric columns in order."""
    from metadamage_amd._lib import RESULT_FIELDS

    keys = ref_meta["record_keys"]
    assert keys[:3] == ["tax_id", "tax_name", "tax_rank"]
    numeric = [k for k in keys[3:] if k != "N_alignments"]
    assert numeric == RESULT_FIELDS
    assert ref_meta["fit_results_columns"] == keys + ["shortname"]
    assert ref_meta["fit_predictions_columns"] == ["tax_id", "position", "median", "hdpi_lower",
                                                   "hdpi_upper", "shortname"]
    assert ref_meta["fit_predictions_position"] == list(range(1, 16)) + list(range(-1, -16, -1))


@pytest.mark.parametrize("case", [0, 1, 2])
def test_waic_restatement_vs_reference(ref_golden, case):
    g = {k.split("__", 1)[1]: ref_golden[k] for k in ref_golden.files if k.startswith(f"waic{case}__")}
    dP, dN = orc.lppd_and_waic(g["lP"]), orc.lppd_and_waic(g["lN"])
    dF, dR, dNF = orc.lppd_and_waic(g["lF"]), orc.lppd_and_waic(g["lR"]), orc.lppd_and_waic(g["lNF"])
    np.testing.assert_allclose(dP["waic_i"], g["waic_i_P"], rtol=1e-13)
    np.testing.assert_allclose(dP["waic"], g["waic_P"], rtol=1e-13)
    np.testing.assert_allclose(dP["lppd"], g["lppd_P"], rtol=1e-13)
    np.testing.assert_allclose(dP["pWAIC"], g["pWAIC_P"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(orc.n_sigma(dP, dN), g["n_sigma"], rtol=1e-12)
    np.testing.assert_allclose(orc.n_sigma(dF, dNF), g["n_sigma_fwd"], rtol=1e-12)
    np.testing.assert_allclose(orc.asymmetry(dP, dF, dR), g["asymmetry"], rtol=1e-12)


def test_map_n_sigma_is_the_reference_formula_with_one_sample(oracle_lib, ref_golden):
    """MDFIT-MAP's n_sigma = the reference's WAIC n_sigma with one posterior
    sample at the mode (pWAIC = 0): recompute it from the oracle's pointwise
    log-likelihoods with the numpy restatement of fits.py:147-201."""
    y, N = pack_golden(ref_golden, ["data_ancient", "data_control"])
    out, _, st = oracle_lib.fit_batch(y, N)
    for t in range(y.shape[0]):
        uP = [np.log(out[t, 32 + j] / (1 - out[t, 32 + j])) if j < 2 else out[t, 32 + j] for j in range(3)]
        uP.append(np.log(out[t, 35] - 2))
        uN = [np.log(out[t, 40] / (1 - out[t, 40])), 0.0, 0.0, np.log(out[t, 43] - 2)]
        _, _, _, lP = oracle_lib.objective(0, 0, y[t, :30], N[t, :30], np.array(uP))
        _, _, _, lN = oracle_lib.objective(1, 0, y[t, :30], N[t, :30], np.array(uN))
        ns = orc.n_sigma(orc.lppd_and_waic(lP[None]), orc.lppd_and_waic(lN[None]))
        assert abs(ns - out[t, 1]) <= 1e-6 * max(1.0, abs(ns))


def test_noise_vs_reference(oracle_lib, ref_golden):
    for name in ("data_ancient", "data_control", "synthetic", "synthetic_CA_GT"):
        mm = mm_from_counts_parquet(name)
        ref = ref_golden[f"{name}__noise"]
        for t in range(mm.shape[0]):
            np.testing.assert_allclose(orc.noise(mm[t]), ref[t], rtol=1e-12)
        y = np.zeros((mm.shape[0], 32), np.uint32)
        N = np.ones((mm.shape[0], 32), np.uint32)
        out, _, _ = oracle_lib.fit_batch(y, N, mm)
        np.testing.assert_allclose(out[:, 22:25], ref, rtol=1e-12)


def test_packing_vs_group_to_numpyro_data(ref_golden):
    """The dense layout (include/mdfit.h) is group_to_numpyro_data's z/y/N
    (fits.py:398-419) for every golden case."""
    for name in ("data_ancient", "data_control", "synthetic", "synthetic_strict", "synthetic_CA_GT"):
        z = ref_golden[f"{name}__z"]
        assert (z == np.r_[np.arange(1, 16), -np.arange(1, 16)]).all()


# --------------------------------------------------------------------------
# MAP predictive HPDI (MDFIT-HPDI v2, oracle/mdfit_hpdi.c)
# --------------------------------------------------------------------------
def _window_rel(lo, hi, rlo, rhi):
    """relative error of the reported bounds lo/N, hi/N (counts >= 1 as scale)"""
    return np.maximum(np.abs(lo - rlo) / np.maximum(rlo, 1.0), np.abs(hi - rhi) / np.maximum(rhi, 1.0))


def test_hpdi_vs_scipy_golden(oracle_lib):
    """Both the spec (greedy / Newton + Euler-Maclaurin + fix-up) and the
    point-by-point definition against scipy's sort-based shortest 68 % window
    (tests/golden/make_golden_hpdi.py): identical integers up to N = 1e5, and
    within 1e-5 relative beyond (the wide, near-flat windows where a rounding
    of the pmf decides between neighbouring counts)."""
    g = np.load(Path(__file__).resolve().parent / "golden" / "hpdi_golden.npz")
    for greedy in (False, True):
        lo, hi = oracle_lib.hpdi68(g["N"], g["a"], g["b"], greedy=greedy)
        small = g["N"] <= 1e5
        assert np.array_equal(lo[small], g["lo"][small]) and np.array_equal(hi[small], g["hi"][small]), greedy
        rel = _window_rel(lo, hi, g["lo"], g["hi"])
        assert rel.max() < 1e-5, (greedy, rel.max())
        assert ((lo == g["lo"]) & (hi == g["hi"])).mean() > 0.98


def test_hpdi_spec_matches_the_definition():
    """The spec against the greedy definition on 20k random (N, D, phi) over
    the whole input range (N up to 3e6, phi down to 2+): within 1e-4 of the
    bounds everywhere (the bar of the fit outputs), identical integers for
    >= 99.9 %."""
    from oracle.oracle import OracleLib

    o = OracleLib()
    rng = np.random.default_rng(7)
    n = 20000
    N = np.floor(np.exp(rng.uniform(np.log(1), np.log(3e6), n)))
    D = np.exp(rng.uniform(np.log(1e-4), np.log(0.99), n))
    phi = np.exp(rng.uniform(np.log(2.0001), np.log(1e5), n))
    lo, hi = o.hpdi68(N, D * phi, (1 - D) * phi)
    glo, ghi = o.hpdi68(N, D * phi, (1 - D) * phi, greedy=True)
    assert _window_rel(lo, hi, glo, ghi).max() < 1e-4
    assert ((lo == glo) & (hi == ghi)).mean() > 0.999


def test_hpdi_edges(oracle_lib):
    """N = 0 -> NaN; alpha -> 0 (D = 0): the point mass at 0; one count;
    the mode alone holding 68 %."""
    lo, hi = oracle_lib.hpdi68([0.0, 5.0, 1.0, 1e6], [1.0, 0.0, 0.5, 1e-9], [1.0, 3.0, 0.5 + 2.0, 50.0])
    assert np.isnan(lo[0]) and np.isnan(hi[0])
    assert (lo[1], hi[1]) == (0.0, 0.0)
    assert lo[2] == 0.0 and hi[2] in (0.0, 1.0)
    assert (lo[3], hi[3]) == (0.0, 0.0)
