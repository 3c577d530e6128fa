"""GPU sampling mode vs the CPU oracle on a small batch (development check).

    python tools/nuts_check.py [--taxa 64] [--warmup 500] [--samples 1000]

Prints, per sub-fit, how many chains reproduce the oracle's draws (max
|delta| over all draws), and the record fields' worst relative difference.
"""

from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--samples", type=int, default=1000)
    a = ap.parse_args()
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd._lib import RESULT_FIELDS
    from metadamage_amd.synthetic import generate
    from oracle.oracle import OracleLib

    b = generate(a.taxa, seed=2)
    opts = _lib.default_opts(mode=_lib.MODE_NUTS, num_warmup=a.warmup, num_samples=a.samples)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    res = engine.alloc_outputs(a.taxa, opts=opts)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    engine.fit_batch_device(ty, tN, tm, opts, res)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = res.out.cpu().numpy()
    st = res.status.cpu().numpy()
    smp = engine.samples_view(res, a.taxa, opts).cpu().numpy()
    print(f"GPU: {a.taxa} taxa in {dt * 1e3:.1f} ms  status {np.bincount(st)}")
    o = OracleLib()
    t0 = time.perf_counter()
    ro, rp, rs, rsmp = o.nuts_batch(b.y, b.N, b.mm, num_warmup=a.warmup, num_samples=a.samples, threads=8,
                                   keep_samples=True)
    print(f"oracle: {time.perf_counter() - t0:.2f} s  status {np.bincount(rs)}")
    for s in range(6):
        d = np.abs(smp[:, s] - rsmp[:, s]).max(axis=(1, 2))
        same = (d < 1e-6).sum()
        print(f"sub {s}: {same}/{a.taxa} chains match the oracle (max |d| < 1e-6); median max|d| {np.median(d):.2e}; "
              f"step gpu/oracle {np.median(out[:, 36 + 8 * s]):.4f}/{np.median(ro[:, 36 + 8 * s]):.4f} "
              f"leapfrogs {np.mean(out[:, 37 + 8 * s]):.2f}/{np.mean(ro[:, 37 + 8 * s]):.2f} "
              f"div {np.sum(out[:, 39 + 8 * s]):.0f}/{np.sum(ro[:, 39 + 8 * s]):.0f}")
    ok = (st == 0) & (rs == 0)
    rel = np.abs(out[ok, :25] - ro[ok, :25]) / np.maximum(np.abs(ro[ok, :25]), 1e-2)
    for j in np.argsort(-np.nanmax(rel, 0))[:8]:
        print(f"  {RESULT_FIELDS[j]:26s} max rel {np.nanmax(rel[:, j]):.2e}  median {np.nanmedian(rel[:, j]):.2e}")
    np.savez("gpurun_out/nuts_check.npz", out=out, ro=ro, smp=smp, rsmp=rsmp, st=st, rs=rs)


if __name__ == "__main__":
    main()
