"""Development timing A/B of the fit / HPDI overlap: the MAP
call time at a batch size for several grids of the HPDI stream kernel's early
launch beside the fit kernel (MDFIT_STREAM_WAVES_PER_CU; 0 = none, the HPDI
then runs after the fit) and of the fit kernel (MDFIT_FIT_WAVES_PER_CU).
Every configuration must give the same record (checked).  One JSON line per
configuration.

    python tools/overlap_exp.py [--taxa 10000]
"""

from __future__ import annotations

import argparse
import json

import numpy as np
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", type=int, default=10_000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--configs", default="", help='JSON list of [name, {env}] (default: the stream-grid sweep)')
    a = ap.parse_args()
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(a.taxa, seed=1)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    fb = engine.alloc_outputs(a.taxa, opts=opts)
    stream = torch.cuda.current_stream()
    configs = [("default", {}), ("no_early", {"MDFIT_STREAM_WAVES_PER_CU": "0"}),
               ("early3", {"MDFIT_STREAM_WAVES_PER_CU": "3"}), ("early5", {"MDFIT_STREAM_WAVES_PER_CU": "5"}),
               ("early6", {"MDFIT_STREAM_WAVES_PER_CU": "6"}),
               ("early4_fit6", {"MDFIT_STREAM_WAVES_PER_CU": "4", "MDFIT_FIT_WAVES_PER_CU": "6"}),
               ("early4_prio0", {"MDFIT_FIT_BASE_PRIO": "0"}),
               ("default_again", {})]
    if a.configs:
        configs = [tuple(c) for c in json.loads(a.configs)]
    keys = {k for _, e in configs for k in e}
    ref = None
    for name, env in configs:
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(env)
        for _ in range(3):
            engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
        torch.cuda.synchronize()
        engine.profile_enable(True, fit_only=True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        _, fit_ms, n = engine.profile_read()
        engine.profile_enable(False)
        rec = (fb.out[:, :25].cpu().numpy(), fb.pred.cpu().numpy(), fb.status.cpu().numpy())
        if ref is None:
            ref = rec
        same = all(np.array_equal(x, y, equal_nan=True) for x, y in zip(rec, ref))
        print(json.dumps({"config": name, "env": env, "taxa": a.taxa, "call_ms": round(dt * 1e3, 4),
                          "fit_kernel_ms": round(fit_ms / n, 4), "fits_per_s": round(a.taxa / dt, 1),
                          "same_record": same}), flush=True)


if __name__ == "__main__":
    main()
