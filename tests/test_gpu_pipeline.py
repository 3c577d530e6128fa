"""GPU end-to-end: `metadamage fit` (CLI -> counts -> batched HIP fit ->
parquet) on the reference's fixture files and a synthetic 22-column file,
checked against the oracle and the reference's column contract."""

from __future__ import annotations

import numpy as np
import pandas as pd
import pytest
from typer.testing import CliRunner

from tests.helpers import GOLDEN, RTOL, mixed_rel

pytestmark = pytest.mark.gpu


def _run(args):
    from metadamage_amd.cli import cli_app

    r = CliRunner().invoke(cli_app, args)
    assert r.exit_code == 0, (r.output, r.exception)
    return r


def test_cli_fit_fixture_files(tmp_path, oracle_lib, ref_meta):
    import torch

    assert torch.cuda.is_available()
    out_dir = tmp_path / "out"
    _run(["fit", "--max-fits", "10", "--max-cores", "1", "--out-dir", str(out_dir), "--inference", "map",
          str(GOLDEN / "data_ancient.txt"), str(GOLDEN / "data_control.txt")])
    from metadamage_amd import _lib, fits, io, utils

    for name in ("data_ancient", "data_control"):
        res = io.Parquet(out_dir / "fit_results" / f"{name}.parquet")
        pred = io.Parquet(out_dir / "fit_predictions" / f"{name}.parquet")
        cnt = io.Parquet(out_dir / "counts" / f"{name}.parquet")
        dfr, dfp, dfc = res.load(), pred.load(), cnt.load()
        assert list(dfr.columns) == ref_meta["fit_results_columns"]
        assert list(dfp.columns) == ref_meta["fit_predictions_columns"]
        assert res.load_metadata()["N_fits"] == 3 and res.load_metadata()["shortname"] == name
        cfg = utils.Config(out_dir=out_dir, max_fits=10, max_cores=1, min_alignments=10, min_y_sum=10,
                           substitution_bases_forward="CT", substitution_bases_reverse="GA", forced=False,
                           version="0.0.0", inference="map")
        cfg.add_filename(GOLDEN / f"{name}.txt")
        p = fits.pack_counts(dfc, cfg)
        o, pr, st = oracle_lib.fit_batch(p.y, p.N, p.mm)
        for j, f in enumerate(_lib.RESULT_FIELDS):
            rel = mixed_rel(dfr[f].to_numpy().astype(float), o[:, j].astype(np.float32).astype(float))
            assert rel.max() < RTOL, (name, f, rel.max())
        assert len(dfp) == 90


def test_cli_default_is_the_reference_sampler(tmp_path, oracle_lib):
    """Without --inference the fit samples like the reference (NUTS 500 / 1000):
    same frames; results agree with the oracle's sampler within Monte-Carlo error."""
    out_dir = tmp_path / "out"
    _run(["fit", "--out-dir", str(out_dir), str(GOLDEN / "data_ancient.txt")])
    from metadamage_amd import fits, io, utils

    res = io.Parquet(out_dir / "fit_results" / "data_ancient.parquet")
    assert res.load_metadata()["inference"] == "nuts"
    dfr = res.load()
    dfc = io.Parquet(out_dir / "counts" / "data_ancient.parquet").load()
    cfg = utils.Config(out_dir=out_dir, max_fits=None, max_cores=1, min_alignments=10, min_y_sum=10,
                       substitution_bases_forward="CT", substitution_bases_reverse="GA", forced=False,
                       version="0.0.0")
    cfg.add_filename(GOLDEN / "data_ancient.txt")
    p = fits.pack_counts(dfc, cfg)
    o, pr, st = oracle_lib.nuts_batch(p.y, p.N, p.mm)
    assert (st == 0).all() and len(dfr) == len(st)
    # posterior summaries: within a few posterior standard deviations (D_max's HPDI width)
    width = o[:, 3] - o[:, 2]
    assert (np.abs(dfr["D_max"].to_numpy() - o[:, 0]) < 0.5 * width + 1e-3).all()
    np.testing.assert_allclose(dfr["q_mean"].to_numpy(), o[:, 4], rtol=0.2, atol=0.02)


def test_cli_cache_and_forced(tmp_path):
    out_dir = tmp_path / "out"
    args = ["fit", "--out-dir", str(out_dir), "--inference", "map", str(GOLDEN / "data_ancient.txt")]
    _run(args)
    f = out_dir / "fit_results" / "data_ancient.parquet"
    m1 = f.stat().st_mtime_ns
    _run(args)  # cache hit: file untouched
    assert f.stat().st_mtime_ns == m1
    _run(args + ["--forced"])
    assert f.stat().st_mtime_ns != m1


def test_cli_synthetic_22col_with_cuts(tmp_path, oracle_lib):
    out_dir = tmp_path / "out"
    _run(["fit", "--out-dir", str(out_dir), "--min-alignments", "20000", "--min-y-sum", "2000",
          str(GOLDEN / "synthetic_counts_22col.tsv")])
    from metadamage_amd import io

    dfr = io.Parquet(out_dir / "fit_results" / "synthetic_counts_22col.parquet").load()
    ref = pd.read_parquet(GOLDEN / "counts_synthetic_strict.parquet")
    assert list(dfr["tax_id"].astype(int)) == [int(t) for t in pd.unique(ref["tax_id"])]
