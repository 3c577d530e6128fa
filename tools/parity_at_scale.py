"""MAP parity at full BASELINE sizes (evidence for DESIGN.md §5): the HIP fit of
C2 (10k taxa, seed 1), C3's size (100k, seed 2) and C4's per-GPU share (125k,
seed 3) against the CPU oracle on all 25 result columns, with bench.py's
metric (|gpu - cpu| / max(|cpu|, 1e-2) over taxa both fitted) and the status
agreement, as one JSON line per size.

    python tools/parity_at_scale.py > profiles/rNN_parity_at_scale.jsonl
    python tools/parity_at_scale.py --sizes 1000000:4   # C4's whole 1M taxa on one GPU
"""

from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    import argparse

    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", nargs="*", default=None, help="TAXA:SEED pairs (default: C2, C3 size, C4 share)")
    ap.add_argument("--dump", default=None, help="npz path: the --dump-n taxa furthest from the oracle, inputs + both records")
    ap.add_argument("--dump-n", type=int, default=64)
    ap.add_argument("--dump-by", choices=["all", "hpdi"], default="hpdi",
                    help="rank by every result column, or by the HPDI ones (D_max_{lower,upper}_hpdi and the "
                    "per-position prediction bounds)")
    a = ap.parse_args()
    sizes = ((10_000, 1, "C2"), (100_000, 2, "C3 size, MAP"), (125_000, 3, "C4 per-GPU share"))
    if a.sizes:
        sizes = tuple((int(t), int(sd), "C4 whole (1M taxa)" if int(t) == 1_000_000 else f"{t} taxa")
                      for t, sd in (x.split(":") for x in a.sizes))

    from bench import parity
    from metadamage_amd import engine
    from metadamage_amd.synthetic import generate
    from oracle.oracle import OracleLib

    oracle = OracleLib()
    threads = min(16, os.cpu_count() or 1)
    for T, seed, label in sizes:
        b = generate(T, seed=seed)
        print(f"generated {T} taxa", file=sys.stderr, flush=True)
        out, pred, st = engine.fit_batch(b.y, b.N, b.mm)
        torch.cuda.synchronize()
        print(f"GPU fit of {T} taxa done", file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        # in 100k-taxon pieces with a progress line each (taxa are independent,
        # so the pieces give the same records; a silent multi-minute call reads
        # as a hang to the GPU runner)
        parts = []
        for lo in range(0, T, 100_000):
            hi = min(T, lo + 100_000)
            parts.append(oracle.fit_batch(b.y[lo:hi], b.N[lo:hi], b.mm[lo:hi], threads=threads))
            print(f"oracle {hi}/{T} taxa, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
        ref, rpred, rst = (np.concatenate([q[i] for q in parts]) for i in range(3))
        cpu_s = time.perf_counter() - t0
        line = parity(out, st, ref, rst, kind="MAP, same MDFIT-MAP v1.1 + MDFIT-HPDI v2 as the oracle")
        line.update(config=label, n_taxa=T, seed=seed, gpu_status_ok=float((st == 0).mean()),
                    cpu_status_ok=float((rst == 0).mean()),
                    status_mismatch_tax_index=[int(i) for i in np.nonzero(st != rst)[0][:10]],
                    not_ok=[[int(i), int(st[i]), int(rst[i])] for i in np.nonzero((st != 0) | (rst != 0))[0][:20]],
                    polished_subfits=int(out[:, 32 + 7::8][:, :6].sum()),
                    polished_subfits_oracle=int(ref[:, 32 + 7::8][:, :6].sum()),
                    polish_mismatch=int((out[:, 32 + 7::8][:, :6] != ref[:, 32 + 7::8][:, :6]).sum()),
                    pred_max_abs=float(np.nanmax(np.abs(pred - rpred))), oracle_s=round(cpu_s, 2),
                    oracle_threads=threads)
        print(json.dumps(line), flush=True)
        if a.dump:
            cols = [2, 3] if a.dump_by == "hpdi" else list(range(25))
            rel = np.abs(out[:, cols] - ref[:, cols]) / np.maximum(np.abs(ref[:, cols]), 1e-2)
            rel = np.where(np.isnan(out[:, cols]) & np.isnan(ref[:, cols]), 0.0, rel).max(axis=1)
            if a.dump_by == "hpdi":  # the per-position windows too (float32 records)
                pr = np.abs(pred[:, 1:3].astype(np.float64) - rpred[:, 1:3]) / np.maximum(np.abs(rpred[:, 1:3]), 1e-2)
                pr = np.where(np.isnan(pred[:, 1:3]) & np.isnan(rpred[:, 1:3]), 0.0, pr).reshape(T, -1).max(axis=1)
                rel = np.maximum(rel, pr)
            idx = np.sort(np.argsort(-np.nan_to_num(rel, nan=np.inf))[:a.dump_n])
            np.savez_compressed(a.dump, idx=idx, rel=rel[idx], seed=seed, n_taxa=T, y=b.y[idx], N=b.N[idx],
                                mm=b.mm[idx], gpu=out[idx], cpu=ref[idx], cpu_pred=rpred[idx], gpu_pred=pred[idx],
                                gpu_status=st[idx], cpu_status=rst[idx])
        del b, out, pred, st, ref, rpred, rst


if __name__ == "__main__":
    main()
