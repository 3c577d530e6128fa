"""Generate the NUTS written-column fixture (run here, output committed).

    python tests/golden/make_golden_nuts_columns.py

The default (sampling) mode's fit_results columns at the reference's settings
(500 warmup + 1000 draws, fits.py:792-799) on a seeded 128-taxon subsample of
config C3 (the SURVEY.md §8(d) generator, seed 2), computed by the CPU oracle
(oracle/mdfit_nuts.c, MDFIT-NUTS v1) under 8 sampler seeds: each taxon's
Monte-Carlo spread of every written column (D_max and its HPDI bounds from the
predictive draws, n_sigma / asymmetry from WAIC, the posterior means, the
forward / reverse columns; fits.py:230-295, 298-356, 89-172).  The GPU test
(tests/test_gpu_nuts_columns.py) runs the kernel on the same inputs under 8
seeds and compares the two per-taxon means in units of their combined standard
error.  Inputs are stored with the outputs, so the test does not depend on the
generator.  Writes tests/golden/nuts_columns_oracle.npz.
"""

from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from metadamage_amd.synthetic import generate  # noqa: E402
from oracle.oracle import OracleLib  # noqa: E402

N_TAXA = 128
SEEDS = tuple(range(8))


def main() -> None:
    b = generate(100_000, seed=2)  # config C3
    idx = np.sort(np.random.default_rng(5).choice(b.n_taxa, N_TAXA, replace=False))
    y, N, mm = b.y[idx], b.N[idx], b.mm[idx]
    lib = OracleLib()
    outs, preds, sts = [], [], []
    for s in SEEDS:
        t0 = time.time()
        o, p, st = lib.nuts_batch(y, N, mm, seed=s)
        print(f"seed {s}: {time.time() - t0:.1f} s, status counts {np.bincount(st)}", flush=True)
        outs.append(o[:, :25])
        preds.append(p)
        sts.append(st)
    np.savez_compressed(ROOT / "tests" / "golden" / "nuts_columns_oracle.npz", idx=idx, y=y, N=N, mm=mm,
                        seeds=np.array(SEEDS), out=np.stack(outs), pred=np.stack(preds), status=np.stack(sts))


if __name__ == "__main__":
    main()
