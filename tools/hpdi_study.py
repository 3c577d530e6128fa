"""Evaluations of ln p per wide HPDI window, by site, in the CPU oracle's spec
(development tool; the oracle built with -DHP_COUNT).  The windows: the 30
z = +1 positions of PMD-all fits of a synthetic batch (the bench's workload).

    python tools/hpdi_study.py [--taxa 3000] [--lib /tmp/hpstudy.so] [-D FLAG ...]
"""

from __future__ import annotations

import argparse
import ctypes
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SITES = ["g(0)/g(N)", "root step", "GL node", "E-M end", "after mass", "fix-up end", "exact walk step",
         "fix-up step", "wide window", "level iteration", "walk start", "1 iteration", "2 iterations",
         "3 iterations", ">3 iterations", "strip masses", "one-sided", "two-sided", "one-sided iters"]


def windows(taxa: int, seed: int):
    cache = Path(f"/tmp/hp_in_{taxa}_{seed}.npz")
    if cache.exists():
        z = np.load(cache)
        return z["N"], z["a"], z["b"]
    from metadamage_amd.synthetic import generate
    from oracle.oracle import OracleLib

    b = generate(taxa, seed=seed)
    o, _, _ = OracleLib().fit_batch(b.y, b.N, b.mm, threads=8, hpdi=False)
    q, A, c, phi = (o[:, 32 + j] for j in range(4))
    k = np.r_[np.arange(15), np.arange(15)]
    D = np.minimum(A[:, None] * (1 - q[:, None]) ** k[None, :] + c[:, None], 1.0)
    N = b.N[:, :30].astype(float)
    ok = (N > 0) & ~np.isnan(q)[:, None]
    N, a, bb = N[ok], (D * phi[:, None])[ok], ((1 - D) * phi[:, None])[ok]
    np.savez(cache, N=N, a=a, b=bb)
    return N, a, bb


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", type=int, default=3000)
    ap.add_argument("--seed", type=int, default=3)
    ap.add_argument("--lib", default="/tmp/hpstudy.so")
    ap.add_argument("-D", action="append", default=[])
    a = ap.parse_args()
    subprocess.run(["gcc", "-O2", "-fPIC", "-fopenmp", "-std=c11", "-shared", "-DHP_COUNT",
                    *[f"-D{d}" for d in a.D], "-o", a.lib, str(ROOT / "oracle" / "mdfit_oracle.c"), "-lm"],
                   check=True)
    lib = ctypes.CDLL(a.lib)
    N, al, be = windows(a.taxa, a.seed)
    n = N.size
    lo, hi = np.zeros(n), np.zeros(n)
    vp = ctypes.c_void_p
    lib.oracle_hpdi68.argtypes = [vp, vp, vp, ctypes.c_int64, ctypes.c_int, vp, vp]
    c = (ctypes.c_ulonglong * 24)()
    lib.oracle_hpdi_counts(c)
    lib.oracle_hpdi68(N.ctypes.data, al.ctypes.data, be.ctypes.data, n, 0, lo.ctypes.data, hi.ctypes.data)
    lib.oracle_hpdi_counts(c)
    glo, ghi = np.zeros(n), np.zeros(n)
    lib.oracle_hpdi68(N.ctypes.data, al.ctypes.data, be.ctypes.data, n, 1, glo.ctypes.data, ghi.ctypes.data)
    nw = max(int(c[8]), 1)
    evals = sum(int(c[k]) for k in (0, 1, 2, 3, 4, 5, 10))
    for k, name in enumerate(SITES):
        print(f"{name:16s} {int(c[k]):10d}  per window {int(c[k]) / nw:8.3f}")
    print(f"windows {n}  wide {nw}  evals/wide window {evals / nw:.3f}  "
          f"== greedy {np.mean((lo == glo) & (hi == ghi)):.6f}  ({np.sum((lo != glo) | (hi != ghi))} differ)")
    np.savez("/tmp/hp_out.npz", lo=lo, hi=hi)


if __name__ == "__main__":
    main()
