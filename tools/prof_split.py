"""Per-call and fit-kernel times of the MAP call for several builds of the
engine (development A/B; the library's own HIP-event profiler,
mdfit_profile_enable: mode 1 events around the call and the fit kernel, mode 2
only around the fit kernel).

    python tools/prof_split.py TAXA metadamage_amd/libmdfit_A.so [...]
"""
import ctypes, sys
sys.path.insert(0, '/root/repo')
import torch
from metadamage_amd import _lib, engine
from metadamage_amd.synthetic import generate
T = int(sys.argv[1]); libs = sys.argv[2:]
b = generate(T, seed=1)
ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
o = _lib.default_opts()
for p in libs:
    lib = _lib.load(p)
    r = engine.alloc_outputs(T, opts=o)
    def call():
        rc = lib.mdfit_fit_batch(ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()),
            ctypes.c_int64(T), ctypes.byref(o), ctypes.c_void_p(r.out.data_ptr()), ctypes.c_void_p(r.pred.data_ptr()),
            ctypes.c_void_p(r.status.data_ptr()), ctypes.c_void_p(r.workspace.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0
    for _ in range(5): call()
    torch.cuda.synchronize()
    for mode in (1, 2):
        lib.mdfit_profile_enable(mode)
        for _ in range(20): call()
        torch.cuda.synchronize()
        a = ctypes.c_double(); f = ctypes.c_double(); n = ctypes.c_int32()
        lib.mdfit_profile_read(ctypes.byref(a), ctypes.byref(f), ctypes.byref(n))
        print(f"{p.split('/')[-1]:24s} mode {mode}: call {a.value/n.value:.3f} ms  fit_kernel {f.value/n.value:.3f} ms", flush=True)
    lib.mdfit_profile_enable(0)
