"""Time mdfit_fit_batch of several builds of the engine on the same batch
(development tool: kernel-design A/B at the bench workload).  Each library has
its own side streams; at batches where the HPDI streams beside the fit (C2) a
library loaded second runs ~3.5 % slower whatever its code (the streams share
hardware queues): A/B those one library per process (tools/overlap_exp.py --lib).

    python tools/variant_bench.py metadamage_amd/libmdfit_A.so metadamage_amd/libmdfit_B.so
"""

from __future__ import annotations

import argparse
import ctypes
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--taxa", type=int, default=10_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--mode", choices=["map", "nuts"], default="map")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--split", action="store_true",
                    help="also the library's own event split (mdfit_profile_*): fit / chain kernel and the rest")
    a = ap.parse_args()

    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(a.taxa, seed=a.seed)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    o = _lib.default_opts(mode=_lib.MODE_NUTS if a.mode == "nuts" else _lib.MODE_MAP)
    libs = [(p, _lib.load(p)) for p in a.libs]
    ref = None
    for rep in range(a.reps):
        for path, lib in libs:
            res = engine.alloc_outputs(a.taxa, opts=o)
            # the workspace size of THIS build (it may differ from the default library's)
            res.workspace = torch.empty(int(lib.mdfit_workspace_bytes(a.taxa, ctypes.byref(o))), dtype=torch.uint8,
                                        device="cuda")

            def call():
                _lib.check(lib.mdfit_fit_batch(
                    ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()),
                    ctypes.c_void_p(tm.data_ptr()), a.taxa, ctypes.byref(o),
                    ctypes.c_void_p(res.out.data_ptr()), ctypes.c_void_p(res.pred.data_ptr()),
                    ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(res.workspace.data_ptr()),
                    ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))

            for _ in range(3 if a.mode == "map" else 1):
                call()
            torch.cuda.synchronize()
            if a.split:
                lib.mdfit_profile_enable(1)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                call()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.steps
            split = ""
            if a.split:
                ca, fk, nn = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
                lib.mdfit_profile_read(ctypes.byref(ca), ctypes.byref(fk), ctypes.byref(nn))
                lib.mdfit_profile_enable(0)
                if nn.value:
                    split = f"  [kernel {fk.value / nn.value:.3f} ms, rest {(ca.value - fk.value) / nn.value:.3f} ms]"
            full = res.out.cpu().numpy()
            out = full[:, :25]
            st = res.status.cpu().numpy()
            pred = res.pred.cpu().numpy()
            if ref is None:
                ref, ref_pred = out, pred
            same_pred = np.array_equal(pred, ref_pred, equal_nan=True)
            rel = np.abs(out - ref) / (np.abs(ref) + 1e-300)
            dev = np.nanmax(rel)
            ndiff = int((np.nan_to_num(rel, nan=0.0).max(1) > 1e-9).sum())
            evals = full[:, _lib.F_DIAG + 5::8][:, :6].sum() if a.mode == "map" else float("nan")
            print(f"rep {rep} {Path(path).name:24s} {ms:8.3f} ms  {a.taxa / ms * 1e3 / 1e6:6.2f} M fits/s  "
                  f"ok {np.mean(st == 0):.4f}  max rel dev vs first {dev:.1e} ({ndiff} taxa)  pred identical {same_pred}  "
                  f"evals {evals:.0f}{split}",
                  flush=True)


if __name__ == "__main__":
    main()
