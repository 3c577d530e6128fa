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
    from metadamage_amd import _lib

    HPDI_COLS = {_lib.RESULT_FIELDS.index("D_max_lower_hpdi"), _lib.RESULT_FIELDS.index("D_max_upper_hpdi")}
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", type=int, default=10_000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--lib", default="", help="a variant build of libmdfit.so (tools/build_variant.sh)")
    ap.add_argument("--configs", default="", help='JSON list of [name, {env}] (default: the stream-grid sweep)')
    a = ap.parse_args()
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    if a.lib:
        _lib._LIB = _lib.load(a.lib)
    b = generate(a.taxa, seed=1)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    fb = engine.alloc_outputs(a.taxa, opts=opts)
    # a config whose env holds "_NOPRED" runs without the predictive columns
    # (pred = NULL: no HPDI launch) -- the floor the HPDI adds to
    fb_np = engine.alloc_outputs(a.taxa, opts=opts, with_pred=False)
    stream = torch.cuda.current_stream()
    configs = [("default", {}), ("no_early", {"MDFIT_STREAM_WAVES_PER_CU": "0"}),
               ("early3", {"MDFIT_STREAM_WAVES_PER_CU": "3"}), ("early5", {"MDFIT_STREAM_WAVES_PER_CU": "5"}),
               ("early6", {"MDFIT_STREAM_WAVES_PER_CU": "6"}),
               ("early4_fit6", {"MDFIT_STREAM_WAVES_PER_CU": "4", "MDFIT_FIT_WAVES_PER_CU": "6"}),
               ("early4_prio0", {"MDFIT_FIT_BASE_PRIO": "0"}),
               ("default_again", {})]
    if a.configs:
        configs = [tuple(c) for c in json.loads(a.configs)]
    keys = {k for _, e in configs for k in e if not k.startswith("_")}
    ref = None
    for name, env in configs:
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update({k: v for k, v in env.items() if not k.startswith("_")})
        f = fb_np if "_NOPRED" in env else fb
        for _ in range(3):
            engine.fit_batch_device(ty, tN, tm, opts, f, stream=stream)
        torch.cuda.synchronize()
        engine.profile_enable(True, fit_only=True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            engine.fit_batch_device(ty, tN, tm, opts, f, stream=stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        _, fit_ms, n = engine.profile_read()
        engine.profile_enable(False)
        rec = (f.out[:, :25].cpu().numpy(), f.status.cpu().numpy(), None if f.pred is None else f.pred.cpu().numpy())
        if ref is None and f.pred is not None:
            ref = rec
        # (without pred the HPDI columns of out are not written: compare the rest)
        cols = [c for c in range(25) if f.pred is not None or c not in HPDI_COLS]
        same = ref is None or (np.array_equal(rec[0][:, cols], ref[0][:, cols], equal_nan=True)
                               and np.array_equal(rec[1], ref[1])
                               and (rec[2] is None or np.array_equal(rec[2], ref[2], equal_nan=True)))
        print(json.dumps({"config": name, "env": env, "taxa": a.taxa, "call_ms": round(dt * 1e3, 4),
                          "fit_kernel_ms": round(fit_ms / n, 4), "fits_per_s": round(a.taxa / dt, 1),
                          "same_record": same}), flush=True)


if __name__ == "__main__":
    main()
