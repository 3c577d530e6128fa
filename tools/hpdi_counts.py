"""SIMD efficiency of the wide-window HPDI loops (development tool).

Runs one fit of the C2 batch through a diagnostic build
(tools/build_variant.sh cnt -DMDFIT_HPDI_COUNT) and prints, per counted site,
lane executions, wave issues and lanes per issue (64 = no divergence).

    python tools/hpdi_counts.py metadamage_amd/libmdfit_cnt.so [--taxa 10000]
"""

from __future__ import annotations

import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

SITES = ["eval g(0)/g(N)", "eval root step", "eval GL node", "eval E-M end", "eval after mass",
         "eval fix-up end", "exact walk step", "fix-up step", "wide window", "level iteration", "eval walk start"]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--taxa", type=int, default=10_000)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()

    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(a.taxa, seed=a.seed)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    o = _lib.default_opts()
    lib = _lib.load(a.lib)
    lib.mdfit_hpdi_counts.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    c = (ctypes.c_ulonglong * 32)()
    res = engine.alloc_outputs(a.taxa, opts=o)
    res.workspace = torch.empty(int(lib.mdfit_workspace_bytes(a.taxa, ctypes.byref(o))), dtype=torch.uint8,
                                device=ty.device)
    torch.cuda.synchronize()
    lib.mdfit_hpdi_counts(c)  # zero
    rc = lib.mdfit_fit_batch(ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()),
                             ctypes.c_void_p(tm.data_ptr()), a.taxa, ctypes.byref(o),
                             ctypes.c_void_p(res.out.data_ptr()), ctypes.c_void_p(res.pred.data_ptr()),
                             ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(res.workspace.data_ptr()),
                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert rc == 0, rc
    lib.mdfit_hpdi_counts(c)
    n_wide = max(int(c[16]), 1)
    for k, name in enumerate(SITES):
        lanes, waves = int(c[2 * k]), int(c[2 * k + 1])
        print(f"{name:16s} lanes {lanes:12d}  issues {waves:10d}  lanes/issue {lanes / max(waves, 1):6.2f}  "
              f"per window {lanes / n_wide:8.2f}")


if __name__ == "__main__":
    main()
