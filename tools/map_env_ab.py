"""MAP A/B at C2 (development tool): the library's environment knobs (read per
call) alternated in one process, 20 timed calls each after 3 warm ones, every
record compared bit for bit with the first.

    python tools/map_env_ab.py 10000 "MDFIT_STREAM_WAVES_PER_CU=3,MDFIT_STREAM_WAVES_PER_CU=4" 4
"""
import os, sys, ctypes, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch
from metadamage_amd import _lib, engine
from metadamage_amd.synthetic import generate
T = int(sys.argv[1]); settings = sys.argv[2].split(","); reps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
b = generate(T, seed=1)
ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
o = _lib.default_opts()
lib = _lib.load()
res = engine.alloc_outputs(T, opts=o)
ref = None
agg = {}
for rep in range(reps):
    for st in settings:
        for kv in st.split(";"):
            k, v = kv.split("=")
            os.environ[k] = v
        def call():
            _lib.check(lib.mdfit_fit_batch(ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()), T, ctypes.byref(o), ctypes.c_void_p(res.out.data_ptr()), ctypes.c_void_p(res.pred.data_ptr()), ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(res.workspace.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
        for _ in range(3): call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): call()
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        r = (res.out.cpu().numpy()[:, :32].copy(), res.pred.cpu().numpy().copy(), res.status.cpu().numpy().copy())
        same = "ref" if ref is None else ("identical" if all(np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(r, ref)) else "DIFFER")
        if ref is None: ref = r
        agg.setdefault(st, []).append(ms)
        print(f"rep {rep} {st:40s} {ms:.4f} ms {same}", flush=True)
for k, v in agg.items():
    print(f"{k:40s} mean {np.mean(v):.4f} ms  min {np.min(v):.4f}  {np.round(v, 4)}")
