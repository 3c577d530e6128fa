"""Development experiment: how much of the MAP call at C2 is the fit kernel's
tail (long PMD tasks claimed late in their queue)?  Times mdfit_fit_batch on
the bench batch with its taxa permuted inside each of the 8 task-queue ranges:
identity, longest task first (task lengths from the oracle's evaluation counts:
an oracle-informed bound, not a product ordering), and shortest first.

    python tools/order_exp.py [--taxa 10000]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", type=int, default=10_000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate
    from oracle.oracle import OracleLib

    T = a.taxa
    b = generate(T, seed=a.seed)
    out, _, _ = OracleLib().fit_batch(b.y, b.N, b.mm, threads=16, hpdi=False)
    ev = out[:, [_lib.F_DIAG + _lib.DIAG_STRIDE * k + 5 for k in range(6)]].astype(int)
    L = ev[:, 0] + np.maximum(ev[:, 2], ev[:, 3])  # PMD-all + the longer of its pair
    orders = {"identity": np.arange(T)}
    lpt, spt = [], []
    for qi in range(8):
        tl, th = T * qi // 8, T * (qi + 1) // 8
        idx = np.arange(tl, th)
        lpt.append(idx[np.argsort(-L[tl:th], kind="stable")])
        spt.append(idx[np.argsort(L[tl:th], kind="stable")])
    orders["longest_first"] = np.concatenate(lpt)
    orders["shortest_first"] = np.concatenate(spt)
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    stream = torch.cuda.current_stream()
    for rep in range(2):
        for name, p in orders.items():
            ty, tN, tm = engine.to_device_counts(b.y[p], b.N[p], b.mm[p])
            fb = engine.alloc_outputs(T, opts=opts)
            for _ in range(3):
                engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
            torch.cuda.synchronize()
            engine.profile_enable(True, fit_only=True)
            t0 = time.perf_counter()
            for _ in range(a.steps):
                engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            _, fit_ms, n = engine.profile_read()
            engine.profile_enable(False)
            print(json.dumps({"order": name, "rep": rep, "taxa": T, "call_ms": round(dt * 1e3, 4),
                              "fit_kernel_ms": round(fit_ms / n, 4), "fits_per_s": round(T / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
