"""Cycle split of the fit kernels from a -DMDFIT_STAMP build (diagnostic only).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DMDFIT_STAMP \
        metadamage_amd/csrc/mdfit.hip -o metadamage_amd/libmdfit_stamp.so
    python tools/stamp_profile.py [--taxa 10000]

Prints, per fit kernel (K1 all-position, K2 forward/reverse), the mean cycles
per wave spent fetching tasks, evaluating points, reducing and in the Newton
logic, and the number of loop trips.  The stamp build's run time is never
quoted; only its shares are read.
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
    ap.add_argument("--taxa", type=int, default=10_000)
    ap.add_argument("--lib", default=str(ROOT / "metadamage_amd" / "libmdfit_stamp.so"))
    a = ap.parse_args()

    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    lib = _lib.load(a.lib)
    lib.mdfit_set_stamp.argtypes = [ctypes.c_void_p]
    b = generate(a.taxa, seed=1)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    res = engine.alloc_outputs(a.taxa)
    # the workspace size of THIS build (it may differ from the default library's)
    res.workspace = torch.empty(int(lib.mdfit_workspace_bytes(a.taxa, None)), dtype=torch.uint8, device="cuda")
    stamps = torch.zeros((65536, 8), dtype=torch.int64, device="cuda")
    lib.mdfit_set_stamp(ctypes.c_void_p(stamps.data_ptr()))
    o = _lib.default_opts()
    for _ in range(2):  # second call is the measured one
        stamps.zero_()
        _lib.check(lib.mdfit_fit_batch(
            ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()),
            a.taxa, ctypes.byref(o), ctypes.c_void_p(res.out.data_ptr()),
            ctypes.c_void_p(res.pred.data_ptr()), ctypes.c_void_p(res.status.data_ptr()),
            ctypes.c_void_p(res.workspace.data_ptr()), None))
        torch.cuda.synchronize()
    s = stamps.cpu().numpy()
    out = res.out.cpu().numpy()
    for name in ("fit_kernel",):
        w = s[s[:, 4] > 0]
        tot = w[:, 5].astype(float)
        print(f"{name}: waves {len(w)}  trips/wave {w[:, 4].mean():.1f}  total cyc/wave {tot.mean():.0f} "
              f"(max {tot.max():.0f})")
        for j, lab in ((3, "fetch"), (0, "eval"), (1, "reduce"), (2, "logic")):
            print(f"   {lab:7s} {w[:, j].mean() / w[:, 4].mean():9.0f} cyc/trip  "
                  f"{100 * w[:, j].sum() / tot.sum():5.1f}%")
        print(f"   claims or (STAMP2) finish_eval+pgnorm {w[:, 6].sum() / tot.sum() * 100:5.1f}%  newton_dir {w[:, 7].sum() / tot.sum() * 100:5.1f}%  "
              f"(of the wave time; includes idle-trip polling)")
    evals = out[:, 32 + 5::8][:, :6]
    print("evals per sub-fit mean:", np.round(evals.mean(0), 2), " max:", evals.max(0))


if __name__ == "__main__":
    main()
