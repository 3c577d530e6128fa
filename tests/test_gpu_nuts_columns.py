"""The default (sampling) mode's written fit_results columns at the
reference's settings (500 warmup + 1000 draws, fits.py:792-799), kernel vs
CPU oracle, in distribution.

Inputs: a seeded 128-taxon subsample of config C3 with the oracle's records
under 8 sampler seeds (tests/golden/nuts_columns_oracle.npz, made by
tests/golden/make_golden_nuts_columns.py).  The kernel runs the same taxa under
the same 8 seeds.  Full-length chains of the two implementations are not equal
draw for draw (the adapted step size amplifies last-ulp differences of the
lnGamma sums), so each written column is compared per taxon as
z = |mean_gpu - mean_oracle| / sqrt(var_gpu / 8 + var_oracle / 8) over the
seeds (each side's Monte-Carlo spread).  Calibration (the oracle's own seeds
0-3 against 4-7, 4 vs 4): median z 0.70, 0.45 % above 4, per-column medians
0.58-0.88.  The data-only columns (N / y sums, noise) must agree exactly.

Columns (fits.py:230-295, 298-356): D_max (predictive median at z = +1),
D_max_{lower,upper}_hpdi, n_sigma, q_mean, concentration_mean,
D_max_marginalized_mean, n_sigma / D_max / q_mean forward and reverse,
asymmetry.
"""

from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from tests.helpers import RTOL, mixed_rel

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).resolve().parent / "golden" / "nuts_columns_oracle.npz"
MC_COLS = (0, 1, 2, 3, 4, 5, 6, 15, 16, 17, 18, 19, 20, 21)
DATA_COLS = (7, 8, 9, 10, 11, 12, 13, 14, 22, 23, 24)


def test_nuts_written_columns_vs_oracle_in_distribution():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    from metadamage_amd import _lib, engine

    g = np.load(GOLDEN)
    seeds = [int(s) for s in g["seeds"]]
    ref = g["out"]  # [S, T, 25]
    assert (g["status"] == 0).all()
    ty, tN, tm = engine.to_device_counts(g["y"], g["N"], g["mm"])
    outs = []
    for s in seeds:
        opts = _lib.default_opts(mode=_lib.MODE_NUTS, seed=s)
        res = engine.fit_batch_device(ty, tN, tm, opts)
        torch.cuda.synchronize()
        st = res.status.cpu().numpy()
        assert (st == 0).all(), (s, np.bincount(st))  # every taxon OK, as the oracle's
        outs.append(res.out.cpu().numpy()[:, :25])
    got = np.stack(outs)
    k = len(seeds)
    # data-only columns: exactly the oracle's (any seed)
    for j in DATA_COLS:
        assert mixed_rel(got[:, :, j], ref[:, :, j]).max() < RTOL, _lib.RESULT_FIELDS[j]
    se = np.sqrt(got.var(0, ddof=1) / k + ref.var(0, ddof=1) / k)
    z = np.abs(got.mean(0) - ref.mean(0)) / np.maximum(se, 1e-12)
    z = z[:, MC_COLS]
    per_col = np.median(z, 0)
    report = {_lib.RESULT_FIELDS[j]: round(float(m), 2) for j, m in zip(MC_COLS, per_col)}
    assert np.median(z) < 0.9, (np.median(z), report)
    assert (z > 4).mean() < 0.02, ((z > 4).mean(), np.sort(z.ravel())[-10:])
    assert per_col.max() < 1.1, report
    # no systematic offset in any column: the mean signed difference in units of
    # its standard error stays small
    signed = (got.mean(0) - ref.mean(0))[:, MC_COLS] / np.maximum(se[:, MC_COLS], 1e-12)
    assert np.abs(np.median(signed, 0)).max() < 0.5, np.round(np.median(signed, 0), 2)
