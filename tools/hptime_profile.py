"""The MAP call's HPDI hand-off timeline at C2 (diagnostic build only: never
quote its run time).  Clock stamps (100 MHz) per taxon -- PMD-all mode
published, pair done -- and per (taxon, position) item -- taken by the HPDI
stream, written -- for three calls, into gpurun_out/hptime.npz; summarised by
tools/hptime_summary.py.

    tools/build_variant.sh hpt -DMDFIT_DEV_HPTIME
    python tools/hptime_profile.py [taxa]
"""
import sys, ctypes, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
from metadamage_amd import _lib, engine
from metadamage_amd.synthetic import generate
T = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
b = generate(T, seed=1)
ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
o = _lib.default_opts()
lib = _lib.load(str(ROOT / "metadamage_amd" / "libmdfit_hpt.so"))
lib.mdfit_dev_set_hptime.argtypes = [ctypes.c_void_p]
res = engine.alloc_outputs(T, opts=o)
res.workspace = torch.empty(int(lib.mdfit_workspace_bytes(T, ctypes.byref(o))), dtype=torch.uint8, device="cuda")
P = 30
buf = torch.zeros(2 * T + 2 * T * P, dtype=torch.int64, device="cuda")
def call():
    _lib.check(lib.mdfit_fit_batch(ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()), T, ctypes.byref(o), ctypes.c_void_p(res.out.data_ptr()), ctypes.c_void_p(res.pred.data_ptr()), ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(res.workspace.data_ptr()), None))
for _ in range(5): call()
torch.cuda.synchronize()
lib.mdfit_profile_enable(1)
outs = []
for rep in range(3):
    buf.zero_()
    lib.mdfit_dev_set_hptime(ctypes.c_void_p(buf.data_ptr()))
    call()
    torch.cuda.synchronize()
    lib.mdfit_dev_set_hptime(None)
    outs.append(buf.cpu().numpy().copy())
cm, fm, nc = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
lib.mdfit_profile_read(ctypes.byref(cm), ctypes.byref(fm), ctypes.byref(nc))
print("call ms avg", cm.value / nc.value, "fit ms avg", fm.value / nc.value, flush=True)
np.savez_compressed("gpurun_out/hptime.npz", *outs, T=T)
