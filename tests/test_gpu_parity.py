"""GPU parity tests: the HIP path (through the C-ABI) vs the CPU oracle and the
committed golden vectors.  Run on an MI355X: pytest -m gpu."""

from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import RTOL, mixed_rel, mm_from_counts_parquet, pack_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    from metadamage_amd import engine as eng

    return eng


def _result_parity(out, ref_out, fields=slice(0, 25)):
    rel = mixed_rel(out[:, fields], ref_out[:, fields])
    return float(rel.max()) if rel.size else 0.0


# --------------------------------------------------------------------------
# special functions and the beta-binomial log-pmf vs scipy known answers
# --------------------------------------------------------------------------
def test_special_functions_vs_scipy(engine, scipy_golden):
    x = scipy_golden["special_x"]
    o = engine.special(x)
    for j, key in enumerate(("special_lgamma", "special_digamma", "special_trigamma")):
        ref = scipy_golden[key]
        err = np.abs(o[:, j] - ref) / np.maximum(1.0, np.abs(ref))
        assert err.max() < 1e-13, (key, err.max(), x[err.argmax()])


def test_betabinom_logpmf_vs_scipy(engine, scipy_golden):
    g = scipy_golden
    lp, grad = engine.betabinom_logpmf(g["bb_y"], g["bb_N"], g["bb_a"], g["bb_b"])
    ref = g["bb_logpmf"]
    # the log-pmf is a sum of 9 lnGamma terms of up to ~2e10 that cancel to
    # O(10): the bar is a few ulp of the terms' magnitude, not of the result
    from scipy.special import gammaln

    y, N, a, b = g["bb_y"], g["bb_N"], g["bb_a"], g["bb_b"]
    mag = sum(np.abs(gammaln(v)) for v in (N + 1, y + 1, N - y + 1, y + a, N - y + b, N + a + b, a, b, a + b))
    err = np.abs(lp - ref)
    assert (err <= 1e-15 * mag + 1e-12).all(), (err / (mag + 1)).max()
    for j, key in enumerate(("bb_dalpha", "bb_dbeta")):
        e = np.abs(grad[:, j] - g[key]) / np.maximum(1e-6, np.abs(g[key]))
        assert e.max() < 1e-8, (key, e.max())


def test_full_logpmf_vs_long_double_oracle(engine, oracle_lib):
    """The value of mdfit_betabinom_logpmf is the record's cancellation-free
    log-pmf (bb_logpmf): against the oracle's long-double restatement over
    N up to 4e9, within 1e-9 of max(1, |logpmf|) (phi <= 1e5)."""
    from tests.test_oracle_golden import _bb_cases

    y, N, a, b = _bb_cases(seed=5)
    phi = a + b
    keep = phi <= 1e5
    y, N, a, b = y[keep], N[keep], a[keep], b[keep]
    lp, _ = engine.betabinom_logpmf(y, N, a, b)
    ref = oracle_lib.bb_logpmf_full(y, N, a, b)
    err = np.abs(lp - ref) / np.maximum(1.0, np.abs(ref))
    assert err.max() < 1e-9, (err.max(), err.argmax())


def test_objective_vs_oracle(engine, oracle_lib):
    """mdfit_objective (the fit kernel's own lane layout and point code) vs the
    oracle's objective: F, gradient, Hessian and pointwise ell of all 6
    sub-fit kinds at seeded points around the data-driven start."""
    from metadamage_amd.synthetic import generate

    b = generate(40, seed=21)
    rng = np.random.default_rng(3)
    kinds = [(0, 0), (1, 0), (0, 1), (0, 2), (1, 1), (1, 2)]
    model, subset, us, rows = [], [], [], []
    for t in range(b.n_taxa):
        for m, s in kinds:
            u = oracle_lib_init(oracle_lib, m, s, b.y[t, :30], b.N[t, :30]) + 0.05 * rng.standard_normal(4)
            u[2] = np.clip(u[2], 0.0, 0.5)
            model.append(m)
            subset.append(s)
            us.append(u)
            rows.append(t)
    rows = np.array(rows)
    F, g, H, ell = engine.objective(np.array(model), np.array(subset), b.y[rows], b.N[rows], np.array(us))
    for i in range(len(rows)):
        Fo, go, Ho, lo = oracle_lib.objective(model[i], subset[i], b.y[rows[i], :30], b.N[rows[i], :30], us[i])
        scale = max(1.0, abs(Fo))
        assert abs(F[i] - Fo) <= 1e-12 * scale + 1e-9, (i, F[i], Fo)
        gs = max(1.0, np.abs(go).max())
        assert np.abs(g[i] - go).max() <= 1e-8 * gs, (i, g[i], go)
        hs = max(1.0, np.abs(Ho).max())
        assert np.abs(H[i] - Ho).max() <= 1e-8 * hs, (i, H[i], Ho)
        assert np.abs(ell[i] - lo).max() <= 1e-12 * max(1.0, np.abs(lo).max()) + 1e-9


def oracle_lib_init(oracle_lib, model, subset, y30, N30):
    u = np.zeros(4)
    oracle_lib.lib.oracle_init_u(model, subset, np.ascontiguousarray(y30, np.uint32).ctypes.data,
                                 np.ascontiguousarray(N30, np.uint32).ctypes.data, u.ctypes.data)
    return u


# --------------------------------------------------------------------------
# MAP predictive HPDI (MDFIT-HPDI v2): the kernel's window vs scipy and the oracle
# --------------------------------------------------------------------------
def test_hpdi_kernel_vs_scipy_and_oracle(engine, oracle_lib):
    from pathlib import Path

    g = np.load(Path(__file__).resolve().parent / "golden" / "hpdi_golden.npz")
    lo, hi = engine.hpdi68(g["N"], g["a"], g["b"])
    small = g["N"] <= 1e5
    bad = np.where(small & ((lo != g["lo"]) | (hi != g["hi"])))[0]
    assert bad.size == 0, [(g["N"][i], g["a"][i], g["b"][i], lo[i], hi[i], g["lo"][i], g["hi"][i]) for i in bad[:5]]
    rel = np.maximum(np.abs(lo - g["lo"]) / np.maximum(g["lo"], 1), np.abs(hi - g["hi"]) / np.maximum(g["hi"], 1))
    assert rel.max() < 1e-5, rel.max()
    # 20k random windows (N up to 1e9 per position, phi down to 2+) vs the
    # oracle's spec.  (Beyond 1e9 with phi < 3 -- a nearly flat pmf whose window
    # spans ~1e9 counts -- a 1e-7 relative rounding of ln p moves the ends by
    # ~1e4 counts: kernel and oracle then agree to ~1.3e-4; the
    # N = 4e9 fit edge case below stays in the suite.)
    rng = np.random.default_rng(17)
    n = 20000
    N = np.floor(np.exp(rng.uniform(0.0, np.log(1e9), n)))
    D = np.exp(rng.uniform(np.log(1e-4), np.log(0.99), n))
    phi = np.exp(rng.uniform(np.log(2.0001), np.log(1e5), n))
    lo, hi = engine.hpdi68(N, D * phi, (1 - D) * phi)
    olo, ohi = oracle_lib.hpdi68(N, D * phi, (1 - D) * phi)
    # the reported bounds lo/N, hi/N under the result columns' bar (mixed_rel:
    # 1e-4 relative, 1e-6 absolute below 1e-2): a one-count difference at the
    # small end of a window ~1e8 counts wide is a rounding of its ~1e-10 mass
    rel = np.maximum(mixed_rel(lo / N, olo / N), mixed_rel(hi / N, ohi / N))
    assert rel.max() < RTOL, (rel.max(), N[rel.argmax()], D[rel.argmax()], phi[rel.argmax()])
    # identical counts for every window up to N = 1e6 (round 6 on the box: 0 of
    # the 13,425 differ); beyond, the two FP64 evaluations of ln p (lnGamma
    # differences vs long-double lgamma) may round the window mass across one
    # count (~1e-8 relative): 98.7 % of all 20k windows identical
    small = N <= 1e6
    same = (lo == olo) & (hi == ohi)
    print(f"HPDI windows identical: N <= 1e6 {same[small].mean():.6f} ({int((~same[small]).sum())} of "
          f"{int(small.sum())} differ), all {same.mean():.6f}")
    assert same[small].all(), np.nonzero(small & ~same)[0][:5]
    assert same.mean() > 0.98


# --------------------------------------------------------------------------
# the fit vs the oracle
# --------------------------------------------------------------------------
def test_fixture_taxa_vs_oracle(engine, oracle_lib, ref_golden):
    names = ["data_ancient", "data_control"]
    y, N = pack_golden(ref_golden, names)
    mm = np.concatenate([mm_from_counts_parquet(n) for n in names])
    out, pred, st = engine.fit_batch(y, N, mm)
    ref_out, ref_pred, ref_st = oracle_lib.fit_batch(y, N, mm)
    assert (st == 0).all() and (ref_st == 0).all()
    assert _result_parity(out, ref_out) < RTOL
    # everything but the WAIC-difference statistics (n_sigma*, asymmetry:
    # differences of ~1e5-sized sums) agrees to ~1e-10
    plain = [j for j in range(25) if j not in (1, 15, 18, 21)]
    assert _result_parity(out, ref_out, plain) < 1e-9
    assert np.nanmax(mixed_rel(pred, ref_pred)) < 1e-6


def test_synthetic_vs_oracle(engine, oracle_lib):
    from metadamage_amd.synthetic import generate

    b = generate(2000, seed=1)
    out, pred, st = engine.fit_batch(b.y, b.N, b.mm)
    ref_out, ref_pred, ref_st = oracle_lib.fit_batch(b.y, b.N, b.mm)
    assert (st == ref_st).all()
    rel = mixed_rel(out[:, :25], ref_out[:, :25])
    assert rel.max() < RTOL, (rel.max(), np.unravel_index(rel.argmax(), rel.shape))
    # p99.9 is far tighter than the bar: same algorithm, FP64 on both sides
    assert np.quantile(rel, 0.999) < 1e-6
    # fitted parameters of all 6 sub-fits (q, A, c on their scale; phi on log scale)
    for s in range(6):
        base = 32 + 8 * s
        for j in range(3):
            assert mixed_rel(out[:, base + j], ref_out[:, base + j]).max() < RTOL
        dlphi = np.abs(np.log(out[:, base + 3]) - np.log(ref_out[:, base + 3]))
        assert dlphi.max() < RTOL
    assert np.nanmax(mixed_rel(pred, ref_pred)) < 1e-5


def test_record_vs_reference_assembly(engine, ref_golden, ref_meta):
    """The record assembled by the reference's own compute_fit_results
    (fits.py:230-356) with MAP quantities injected at the numpyro boundary."""
    keys = ref_meta["record_keys"][3:]
    from metadamage_amd._lib import RESULT_FIELDS

    for name in ("data_ancient", "data_control", "synthetic"):
        y, N = pack_golden(ref_golden, [name])
        mm = mm_from_counts_parquet(name)
        out, pred, st = engine.fit_batch(y, N, mm)
        rec = ref_golden[f"record_{name}__values"]
        n = rec.shape[0]
        for k in keys:
            if k == "N_alignments":
                continue
            j = RESULT_FIELDS.index(k)
            rel = mixed_rel(out[:n, j], rec[:, keys.index(k)])
            assert rel.max() < RTOL, (name, k, rel.max())
        med = ref_golden[f"record_{name}__median"]
        hp = ref_golden[f"record_{name}__hpdi"]
        assert np.nanmax(mixed_rel(pred[:n, 0], med)) < 1e-5
        assert np.nanmax(mixed_rel(pred[:n, 1], hp[:, 0])) < 1e-5
        assert np.nanmax(mixed_rel(pred[:n, 2], hp[:, 1])) < 1e-5
        noise = ref_golden[f"{name}__noise"][:n]
        assert np.nanmax(mixed_rel(out[:n, 22:25], noise)) < 1e-10


# --------------------------------------------------------------------------
# edge cases (empty / ragged / extreme inputs)
# --------------------------------------------------------------------------
def _edge_batch():
    from metadamage_amd.synthetic import generate

    b = generate(16, seed=9)
    y, N, mm = b.y.copy(), b.N.copy(), b.mm.copy()
    N[0, :30] = 0  # no coverage at all
    y[0, :30] = 0
    N[1, 5:12] = 0  # ragged coverage
    y[1, 5:12] = 0
    N[2, 0] = 0  # N_z1 = 0 -> D_max NaN like the reference's 0/0
    y[2, 0] = 0
    y[3, :30] = N[3, :30]  # y == N everywhere
    y[4, :30] = 0  # no damage signal at all
    N[5, :30] = 4_000_000_000  # near the uint32 ceiling
    y[5, :30] = (N[5, :30] // 100).astype(np.uint32)
    y[6, 3] = N[6, 3] + 1  # invalid -> status 3
    N[7, :30] = 1  # minimal coverage
    y[7, :30] = np.arange(30) % 2
    mm[8] = 0  # all mismatch columns zero -> noise NaN
    return y, N, mm


def test_edge_cases_vs_oracle(engine, oracle_lib):
    y, N, mm = _edge_batch()
    out, pred, st = engine.fit_batch(y, N, mm)
    ref_out, ref_pred, ref_st = oracle_lib.fit_batch(y, N, mm)
    assert (st == ref_st).all(), (st, ref_st)
    assert st[6] == 3 and np.isnan(out[6, :25]).all()
    ok = st != 3
    rel = mixed_rel(out[ok, :25], ref_out[ok, :25])
    # every field of every taxon meets the 1e-4 bar -- taxon 5 too (N = 4e9 at
    # every position: its WAIC statistics come from the cancellation-free
    # log-pmf, not from differences of lnGamma values ~8e10)
    assert rel.max() < RTOL, (rel.max(), np.unravel_index(rel.argmax(), rel.shape))
    assert np.isnan(out[2, 0]) and np.isnan(ref_out[2, 0])
    assert np.isnan(out[8, 22:25]).all()


def test_empty_batch(engine):
    from metadamage_amd import _lib

    lib = _lib.load()
    assert lib.mdfit_fit_batch(None, None, None, 0, None, None, None, None, None, None) == 0


def test_no_mismatch_counts_gives_nan_noise(engine):
    from metadamage_amd.synthetic import generate

    b = generate(8, seed=4)
    out, _, st = engine.fit_batch(b.y, b.N, None)
    assert (st == 0).all()
    assert np.isnan(out[:, 22:25]).all()


# --------------------------------------------------------------------------
# size-independent properties at the benchmark size (10k taxa, config C2)
# --------------------------------------------------------------------------
def test_bench_size_properties(engine, oracle_lib):
    from metadamage_amd.synthetic import generate

    b = generate(10_000, seed=1)
    out1, pred1, st1 = engine.fit_batch(b.y, b.N, b.mm)
    out2, pred2, st2 = engine.fit_batch(b.y, b.N, b.mm)
    # deterministic: bit-identical reruns
    assert np.array_equal(out1, out2, equal_nan=True) and np.array_equal(st1, st2)
    # order-independent: a permuted batch gives the same per-taxon bits
    perm = np.random.default_rng(0).permutation(b.n_taxa)
    out3, _, st3 = engine.fit_batch(b.y[perm], b.N[perm], b.mm[perm])
    assert np.array_equal(out3, out1[perm], equal_nan=True)
    assert (st1 == 0).mean() > 0.999
    # a seeded 400-taxon sample against the oracle
    idx = np.sort(np.random.default_rng(1).choice(b.n_taxa, 400, replace=False))
    ref_out, _, ref_st = oracle_lib.fit_batch(b.y[idx], b.N[idx], b.mm[idx])
    assert (ref_st == st1[idx]).all()
    assert mixed_rel(out1[idx, :25], ref_out[:, :25]).max() < RTOL


def test_lane_layouts_are_bitwise_identical(engine, monkeypatch):
    """The fit kernel's two lane layouts (1 point per lane below 13k taxa, 2
    above) sum in the same tree order, so a taxon's record does
    not depend on the batch size that picked the layout -- nor on where the
    predictive HPDI ran (streamed beside the fit kernel below 60k taxa, K4a /
    K4b after it above)."""
    from metadamage_amd.synthetic import generate

    b = generate(3_000, seed=11)
    res = {}
    for ppl in ("1", "2"):
        monkeypatch.setenv("MDFIT_FIT_PPL", ppl)
        res[ppl] = engine.fit_batch(b.y, b.N, b.mm)
    for a, c in zip(res["1"], res["2"]):
        assert np.array_equal(a, c, equal_nan=True)
    # and a taxon fitted inside larger batches matches it too: 16k (2 points
    # per lane, HPDI streamed) and 66k (HPDI after the fit)
    monkeypatch.delenv("MDFIT_FIT_PPL")
    more = generate(63_000, seed=12)
    for extra in (13_000, 63_000):
        cat = [np.concatenate([getattr(b, f), getattr(more, f)[:extra]]) for f in ("y", "N", "mm")]
        out_big, pred_big, st_big = engine.fit_batch(*cat)
        assert np.array_equal(out_big[:3_000], res["1"][0], equal_nan=True)
        assert np.array_equal(pred_big[:3_000], res["1"][1], equal_nan=True)
        assert np.array_equal(st_big[:3_000], res["1"][2])
