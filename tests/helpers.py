"""Shared test helpers (packing golden fixtures into the engine layout, tolerances)."""

from __future__ import annotations

from pathlib import Path

import numpy as np
import pandas as pd

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
MM_COLUMNS = ["AC", "AG", "AT", "CA", "CG", "CT", "GA", "GC", "GT", "TA", "TC", "TG"]

# per-taxon parity bar of the north star: 1e-4 relative, with an absolute floor
# for quantities that sit near zero (n_sigma, asymmetry): |d| <= 1e-4 * max(|ref|, 1e-2)
RTOL = 1e-4
FLOOR = 1e-2


def mixed_rel(a, r, floor=FLOOR):
    a = np.asarray(a, float)
    r = np.asarray(r, float)
    both_nan = np.isnan(a) & np.isnan(r)
    rel = np.abs(a - r) / np.maximum(np.abs(r), floor)
    return np.where(both_nan, 0.0, rel)


def pack_golden(g, names):
    """Stack y/N of golden cases into uint32[T][32]."""
    ys = np.concatenate([g[f"{n}__y"] for n in names])
    Ns = np.concatenate([g[f"{n}__N"] for n in names])
    T = ys.shape[0]
    y = np.zeros((T, 32), np.uint32)
    N = np.zeros((T, 32), np.uint32)
    y[:, :30] = ys
    N[:, :30] = Ns
    return y, N


def mm_from_counts_parquet(name):
    """uint32[T][30][12] mismatch counts, taxa in df order (N_alignments desc)."""
    df = pd.read_parquet(GOLDEN / f"counts_{name}.parquet")
    vals = df[MM_COLUMNS].to_numpy().astype(np.uint32)
    return vals.reshape(-1, 30, 12)
