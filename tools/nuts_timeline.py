"""Per-chain timeline of the C3 chain kernel (diagnostic build only: never quote
its run time): each chain's start and end clock (100 MHz) and its wave-trips,
written over diag slots 4, 5, 7 by a -DMDFIT_DEV_TRIPS build, into
gpurun_out/nuts_timeline.npz.

    tools/build_variant.sh ntrips -DMDFIT_DEV_TRIPS
    python tools/nuts_timeline.py [taxa]
"""
import os, sys, ctypes, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
from metadamage_amd import _lib, engine
from metadamage_amd.synthetic import generate
T = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
b = generate(T, seed=2)
ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
o = _lib.default_opts(mode=_lib.MODE_NUTS)
lib = _lib.load(str(ROOT / "metadamage_amd" / "libmdfit_ntrips.so"))
res = engine.alloc_outputs(T, opts=o)
res.workspace = torch.empty(int(lib.mdfit_workspace_bytes(T, ctypes.byref(o))), dtype=torch.uint8, device="cuda")
dump = {}
for order in (0,):
    _lib.check(lib.mdfit_fit_batch(ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()), T, ctypes.byref(o), ctypes.c_void_p(res.out.data_ptr()), ctypes.c_void_p(res.pred.data_ptr()), ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(res.workspace.data_ptr()), None))
    torch.cuda.synchronize()
    out = res.out.cpu().numpy()
    dg = out[:, _lib.F_DIAG:_lib.F_DIAG + 6 * _lib.DIAG_STRIDE].reshape(T, 6, _lib.DIAG_STRIDE)
    dump[f"t0_{order}"] = dg[:, :, 4].copy(); dump[f"t1_{order}"] = dg[:, :, 5].copy(); dump[f"trips_{order}"] = dg[:, :, 7].copy()
    t0, t1 = dg[:, :, 4], dg[:, :, 5]
    print(order, "span s", (np.nanmax(t1) - np.nanmin(t0)) / 1e8, "mean end", (np.nanmean(t1) - np.nanmin(t0)) / 1e8, flush=True)
np.savez_compressed("gpurun_out/nuts_timeline.npz", **dump)
