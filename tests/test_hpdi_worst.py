"""The 64 taxa of C4's whole million (generate(1_000_000, seed=3)) whose HPDI
columns -- D_max_{lower,upper}_hpdi and the per-position prediction bounds --
ended furthest from the CPU oracle in the round-6 full-size parity run
(tools/parity_at_scale.py --sizes 1000000:3 --dump, worst 1.5e-5 relative
in round 5), committed as a fixture: inputs, the oracle's record and
predictions (tests/golden/hpdi_worst_1m.npz).  The fit of a taxon does not
depend on its batch, so these taxa alone reproduce the worst cases of the 1M
run at every -m gpu run (the reference's columns:
/root/reference/metadamage/fits.py:112-120, 260-261).

  * CPU: the oracle re-run on the fixture's inputs reproduces its records bit
    for bit (the fixture is the oracle's, not a stale copy);
  * GPU: every result column and prediction bound within 2e-5 (mixed
    relative, the columns' 1e-4 bar's floor) of the oracle, statuses equal."""

from __future__ import annotations

import numpy as np
import pytest

from tests.helpers import GOLDEN, mixed_rel

FIX = GOLDEN / "hpdi_worst_1m.npz"
TOL = 2e-5


@pytest.fixture(scope="module")
def fx():
    if not FIX.exists():
        pytest.fail(f"{FIX} missing: tools/parity_at_scale.py --sizes 1000000:3 --dump")
    return np.load(FIX)


def test_fixture_is_the_oracles_record(fx, oracle_lib):
    out, pred, st = oracle_lib.fit_batch(fx["y"], fx["N"], fx["mm"], threads=4)
    assert np.array_equal(st, fx["cpu_status"])
    assert np.array_equal(out[:, :25], fx["cpu"][:, :25], equal_nan=True)
    assert np.array_equal(pred, fx["cpu_pred"], equal_nan=True)
    assert int(fx["n_taxa"]) == 1_000_000 and int(fx["seed"]) == 3 and len(fx["idx"]) == 64


@pytest.mark.gpu
def test_worst_hpdi_taxa_of_the_million_on_the_gpu(fx):
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    from metadamage_amd import engine

    out, pred, st = engine.fit_batch(fx["y"], fx["N"], fx["mm"])
    assert np.array_equal(st, fx["cpu_status"])
    ok = st == 0
    rel = mixed_rel(out[ok, :25], fx["cpu"][ok, :25])
    prel = mixed_rel(pred[ok], fx["cpu_pred"][ok])
    worst = max(float(rel.max()), float(prel.max()))
    print(f"worst-HPDI taxa of the 1M run: result columns {rel.max():.3e}, prediction bounds {prel.max():.3e}")
    assert worst <= TOL, worst
