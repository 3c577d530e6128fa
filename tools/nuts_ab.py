"""NUTS A/B at C3 (development tool): calls alternated over (library, ENV=VALUE)
pairs in one process, the chain kernel timed by the library's profile events
(mdfit_profile_enable), every record compared bit for bit with the first.

    python tools/nuts_ab.py 100000 A:X=0,default:X=0,A:X=0,default:X=0
    (A = metadamage_amd/libmdfit_A.so from tools/build_variant.sh; default =
    libmdfit.so; ENV=VALUE is exported before the call, X=0 for none)
"""
import os, sys, ctypes, time, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
from metadamage_amd import _lib, engine
from metadamage_amd.synthetic import generate
T = int(sys.argv[1])
runs = [x.split(":") for x in sys.argv[2].split(",")]
b = generate(T, seed=2)
ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
o = _lib.default_opts(mode=_lib.MODE_NUTS)
libs = {}
res = engine.alloc_outputs(T, opts=o)
ref = None
agg = {}
for name, order in runs:
    if name not in libs:
        libs[name] = _lib.load(str(ROOT / "metadamage_amd" / (f"libmdfit_{name}.so" if name != "default" else "libmdfit.so")))
        libs[name].mdfit_profile_enable(1)
    lib = libs[name]
    ws = torch.empty(int(lib.mdfit_workspace_bytes(T, ctypes.byref(o))), dtype=torch.uint8, device="cuda")
    if "=" in order:
        k, v = order.split("=")
        os.environ[k] = v
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _lib.check(lib.mdfit_fit_batch(ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()), T, ctypes.byref(o), ctypes.c_void_p(res.out.data_ptr()), ctypes.c_void_p(res.pred.data_ptr()), ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(ws.data_ptr()), None))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    cm, fm, nc = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
    lib.mdfit_profile_read(ctypes.byref(cm), ctypes.byref(fm), ctypes.byref(nc))
    r = (res.out.cpu().numpy()[:, :32].copy(), res.pred.cpu().numpy().copy(), res.status.cpu().numpy().copy())
    same = "ref" if ref is None else ("identical" if all(np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(r, ref)) else "DIFFER")
    if ref is None: ref = r
    agg.setdefault((name, order), []).append(fm.value / 1e3)
    print(f"{name:10s} order {order} call {dt:.4f} s chain {fm.value / 1e3:.4f} s  {same}", flush=True)
    del ws
for k, v in agg.items():
    print(k, "chain mean %.4f" % np.mean(v), np.round(v, 3))
