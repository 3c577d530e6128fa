"""Synthetic per-taxon count tensors for benchmarks and tests.

Generator spec: SURVEY.md §8(d).  Each taxon gets damage parameters
(A, q, c, phi), a sequencing depth and 30 positions (z = 1..15 forward,
-1..-15 reverse) of beta-binomial C->T / G->A counts drawn from the same
model the reference fits (model_PMD, /root/reference/metadamage/fits.py:43-59),
plus the 12 mismatch columns that add_noise_estimates reads
(fits.py:359-376).  Layout is the engine's dense layout (include/mdfit.h):
y, N uint32[T][32] (2 pad columns), mm uint32[T][30][12].

Seeds (§8(d)): C2 = 1, C3 = 2, C4 = 3, C5 file i = 100 + i.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

NPOS = 30
NHALF = 15
LD = 32
NMM = 12
# reference column order of the 12 off-diagonal base columns
MM_COLUMNS = ["AC", "AG", "AT", "CA", "CG", "CT", "GA", "GC", "GT", "TA", "TC", "TG"]
CT_COL = MM_COLUMNS.index("CT")
GA_COL = MM_COLUMNS.index("GA")


@dataclass
class SyntheticBatch:
    tax_id: np.ndarray  # int64[T]
    y: np.ndarray  # uint32[T][32]
    N: np.ndarray  # uint32[T][32]
    mm: np.ndarray  # uint32[T][30][12]
    N_alignments: np.ndarray  # int64[T]
    truth: dict  # generating parameters (A, q, c, phi, ancient)

    @property
    def n_taxa(self) -> int:
        return int(self.y.shape[0])


def abs_z() -> np.ndarray:
    """|z| of the 30 dense columns: 1..15, 1..15."""
    k = np.arange(NPOS)
    return np.where(k < NHALF, k + 1, k - NHALF + 1)


def generate(n_taxa: int, seed: int, fail_fraction: float = 0.0) -> SyntheticBatch:
    """Draw `n_taxa` synthetic taxa.

    fail_fraction > 0 (config C5) builds that fraction of taxa to fail the
    counts cuts (N_alignments < 10 or y_sum < 10).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    T = int(n_taxa)
    ancient = rng.random(T) < 0.3
    A = np.where(ancient, rng.uniform(0.05, 0.5, T), rng.uniform(0.0, 0.01, T))
    q = rng.beta(2.0, 3.0, T)
    c = rng.uniform(0.001, 0.03, T)
    bad = A + c >= 0.95
    while bad.any():  # rejection step of the spec
        nb = int(bad.sum())
        A[bad] = np.where(ancient[bad], rng.uniform(0.05, 0.5, nb), rng.uniform(0.0, 0.01, nb))
        c[bad] = rng.uniform(0.001, 0.03, nb)
        bad = A + c >= 0.95
    phi = np.exp(rng.uniform(np.log(10.0), np.log(1e4), T))
    depth = np.exp(rng.uniform(np.log(1e2), np.log(1e7), T))

    z = abs_z()
    D = A[:, None] * (1.0 - q[:, None]) ** (z[None, :] - 1) + c[:, None]
    D = np.clip(D, 1e-12, 1.0 - 1e-12)
    Nz = np.rint(depth[:, None] * rng.uniform(0.85, 1.15, (T, NPOS))).astype(np.int64)
    p = rng.beta(D * phi[:, None], (1.0 - D) * phi[:, None])
    yz = rng.binomial(Nz, p)
    N_alignments = np.rint(depth * rng.uniform(2.0, 6.0, T)).astype(np.int64)

    if fail_fraction > 0:
        fail = rng.random(T) < fail_fraction
        low_aln = fail & (rng.random(T) < 0.5)
        N_alignments[low_aln] = rng.integers(1, 10, int(low_aln.sum()))
        low_y = fail & ~low_aln
        yz[low_y] = 0
        Nz[low_y] = np.minimum(Nz[low_y], 50)

    mm = rng.binomial(np.repeat(Nz[:, :, None], NMM, axis=2), 1e-3).astype(np.uint32)
    mm[:, :NHALF, CT_COL] = yz[:, :NHALF]
    mm[:, NHALF:, GA_COL] = yz[:, NHALF:]
    # keep the reference-base sums consistent with N (C = CA+CC+CG+CT forward,
    # G = GA+GC+GG+GT reverse) by clipping the background draws to the room left
    for half, ref_cols in ((slice(0, NHALF), ("CA", "CG")), (slice(NHALF, NPOS), ("GC", "GT"))):
        room = (Nz[:, half] - yz[:, half]).astype(np.int64)
        for name in ref_cols:
            j = MM_COLUMNS.index(name)
            v = np.minimum(mm[:, half, j].astype(np.int64), room)
            mm[:, half, j] = v
            room = room - v

    y = np.zeros((T, LD), dtype=np.uint32)
    N = np.zeros((T, LD), dtype=np.uint32)
    y[:, :NPOS] = yz
    N[:, :NPOS] = Nz
    tax_id = np.arange(T, dtype=np.int64) + 1_000_000 * (seed % 1000)
    truth = {"A": A, "q": q, "c": c, "phi": phi, "ancient": ancient}
    return SyntheticBatch(tax_id, y, N, mm, N_alignments, truth)


def to_counts_table(batch: SyntheticBatch) -> "object":
    """Render a batch as the reference's 22-column input table
    (counts.py:37-45: tax_id, tax_name, tax_rank, N_alignments, strand,
    position, AA..TT), positions 0-indexed as in the raw files.

    The 4 diagonal columns (AA, CC, GG, TT) are chosen so that the reference
    sums C = CA+CC+CG+CT and G = GA+GC+GG+GT (counts.py:86-89) reproduce N.
    """
    import pandas as pd

    T = batch.n_taxa
    bases = [r + o for r in "ACGT" for o in "ACGT"]
    cols = {b: np.zeros((T, NPOS), dtype=np.int64) for b in bases}
    for j, name in enumerate(MM_COLUMNS):
        cols[name] = batch.mm[:, :, j].astype(np.int64)
    N = batch.N[:, :NPOS].astype(np.int64)
    # forward rows: N is the C-reference sum; reverse rows: the G-reference sum
    c_other = cols["CA"] + cols["CG"] + cols["CT"]
    g_other = cols["GA"] + cols["GC"] + cols["GT"]
    fwd = np.arange(NPOS) < NHALF
    cols["CC"] = np.where(fwd[None, :], np.maximum(N - c_other, 0), N)
    cols["GG"] = np.where(~fwd[None, :], np.maximum(N - g_other, 0), N)
    cols["AA"] = N
    cols["TT"] = N

    rows = T * NPOS
    pos = np.tile(np.where(fwd, np.arange(NPOS), np.arange(NPOS) - NHALF), T)
    strand = np.tile(np.where(fwd, "5'", "3'"), T)
    df = pd.DataFrame(
        {
            "tax_id": np.repeat(batch.tax_id, NPOS),
            "tax_name": np.repeat([f"taxon_{t}" for t in batch.tax_id], NPOS),
            "tax_rank": "species",
            "N_alignments": np.repeat(batch.N_alignments, NPOS),
            "strand": strand,
            "position": pos,
        }
    )
    for b in bases:
        df[b] = cols[b].reshape(rows)
    return df
