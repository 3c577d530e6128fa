"""Slot utilisation of the NUTS chain kernel (development build -DMDFIT_DEV_UTIL):
running chain slots per trip over the wave's 4 slots.

    tools/build_variant.sh util -DMDFIT_DEV_UTIL
    python tools/nuts_util.py metadamage_amd/libmdfit_util.so [--taxa 100000]
"""

from __future__ import annotations

import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--taxa", type=int, default=100_000)
    ap.add_argument("--seed", type=int, default=2)
    a = ap.parse_args()
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(a.taxa, seed=a.seed)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    o = _lib.default_opts(mode=_lib.MODE_NUTS)
    lib = _lib.load(a.lib)
    res = engine.alloc_outputs(a.taxa, opts=o)
    res.workspace = torch.empty(int(lib.mdfit_workspace_bytes(a.taxa, ctypes.byref(o))), dtype=torch.uint8, device="cuda")
    _lib.check(lib.mdfit_fit_batch(
        ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()), a.taxa,
        ctypes.byref(o), ctypes.c_void_p(res.out.data_ptr()), ctypes.c_void_p(res.pred.data_ptr()),
        ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(res.workspace.data_ptr()),
        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    torch.cuda.synchronize()
    c = res.workspace[128:144].view(torch.int64).cpu().tolist()
    trips, busy = c
    print(f"wave-trips {trips}  running slot-trips {busy}  utilisation {busy / (4 * trips):.4f}")


if __name__ == "__main__":
    main()
