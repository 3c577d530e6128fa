"""Does the library's event profiling (mdfit_profile_enable) cost the C2 call
time?  20 timed calls with and without it, alternated (development check)."""
import sys, time
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch
from metadamage_amd import _lib, engine
from metadamage_amd.synthetic import generate

T = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
b = generate(T, seed=1)
ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
o = _lib.default_opts()
res = engine.alloc_outputs(T, opts=o)
st = torch.cuda.current_stream()
for _ in range(3):
    engine.fit_batch_device(ty, tN, tm, o, res, stream=st)
torch.cuda.synchronize()
for rep in range(4):
    for mode in ("off", "fit_only", "all"):
        if mode != "off":
            engine.profile_enable(True, fit_only=(mode == "fit_only"))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            engine.fit_batch_device(ty, tN, tm, o, res, stream=st)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        if mode != "off":
            engine.profile_read()
            engine.profile_enable(False)
        print(f"rep {rep} {mode:9s} {ms:.4f} ms", flush=True)
