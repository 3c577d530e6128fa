"""Find the taxa where the GPU fit and the oracle disagree on a synthetic C5
file (development tool): prints the worst fields and saves their counts.

    python tools/c5_mismatch.py --seed 101 --taxa 20000 --out gpurun_out/c5_bad.npz
"""

from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=101)
    ap.add_argument("--taxa", type=int, default=20_000)
    ap.add_argument("--fail", type=float, default=0.05)
    ap.add_argument("--out", default="gpurun_out/c5_bad.npz")
    a = ap.parse_args()

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate
    from oracle.oracle import OracleLib
    from tests.helpers import mixed_rel

    b = generate(a.taxa, seed=a.seed, fail_fraction=a.fail)
    out, _, st = engine.fit_batch(b.y, b.N, b.mm)
    ref, _, rst = OracleLib().fit_batch(b.y, b.N, b.mm, hpdi=False)
    both = (st == 0) & (rst == 0)
    print("status mismatches", np.where(st != rst)[0][:20])
    cols = [j for j in range(25) if j not in (2, 3)]
    rel = mixed_rel(out[:, cols], ref[:, cols])
    rel[~both] = 0
    worst = np.argsort(rel.max(1))[::-1][:10]
    for t in worst:
        j = cols[int(rel[t].argmax())]
        print(f"taxon {t} field {_lib.RESULT_FIELDS[j]} rel {rel[t].max():.3e} gpu {out[t, j]!r} oracle {ref[t, j]!r}")
        for k in range(6):
            d = 32 + 8 * k
            print(f"   sub {k} gpu {out[t, d:d + 8]}\n          orc {ref[t, d:d + 8]}")
    bad = worst[rel[worst].max(1) > 1e-4]
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    np.savez(a.out, idx=bad, y=b.y[bad], N=b.N[bad], mm=b.mm[bad], gpu=out[bad], orc=ref[bad])


if __name__ == "__main__":
    main()
