"""Host-to-host fit rate with the chunked two-stream dispatch (engine.ChunkedFitter)
against the device-resident call, and the PCIe copy rates behind it.

    python tools/h2h_study.py [--taxa 10000,125000] [--chunks 1,2,3,4,6]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def pcie(torch, mb=256, reps=5):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}
    for name in ("h2d", "d2h", "both"):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if name in ("h2d", "both"):
                with torch.cuda.stream(s1):
                    d.copy_(h, non_blocking=True)
            if name in ("d2h", "both"):
                with torch.cuda.stream(s2):
                    h2.copy_(d2, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name + "_GBs"] = round(n / min(ts) / 1e9 * (2 if name == "both" else 1), 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", default="10000,125000")
    ap.add_argument("--chunks", default="1,2,3,4,6")
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    print(json.dumps({"pcie": pcie(torch)}), flush=True)
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    for T in map(int, a.taxa.split(",")):
        b = generate(T, seed=1 if T == 10_000 else 3)
        ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
        fb = engine.alloc_outputs(T, opts=opts)
        for _ in range(3):
            engine.fit_batch_device(ty, tN, tm, opts, fb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            engine.fit_batch_device(ty, tN, tm, opts, fb)
        torch.cuda.synchronize()
        dev_ms = (time.perf_counter() - t0) / a.reps * 1e3
        ref = (fb.out[:, :25].cpu().numpy(), fb.status.cpu().numpy())
        del ty, tN, tm, fb
        pp = engine.PinnedPack(T)
        y, N, mm = pp.views(T)
        y[:], N[:], mm[:] = b.y, b.N, b.mm
        line = {"taxa": T, "device_resident_ms": round(dev_ms, 3), "device_resident_fits_s": round(T / dev_ms * 1e3)}
        for nch in map(int, a.chunks.split(",")):
            cap = -(-T // nch)
            f = engine.ChunkedFitter(cap, opts=opts)
            ch = engine.plan_chunks(T, opts, chunk_taxa=cap)
            for _ in range(2):
                f.run(y, N, mm, opts, pinned=pp, chunks=ch)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                o, p, s = f.run(y, N, mm, opts, pinned=pp, chunks=ch)
                ts.append(time.perf_counter() - t0)
            ok = bool(np.array_equal(o, ref[0], equal_nan=True) and np.array_equal(s, ref[1]))
            ms = float(np.median(ts)) * 1e3
            line[f"chunks{nch}"] = {"ms": round(ms, 3), "fits_s": round(T / ms * 1e3), "frac_of_device": round(dev_ms / ms, 3),
                                    "identical": ok}
            del f
            torch.cuda.empty_cache()
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
