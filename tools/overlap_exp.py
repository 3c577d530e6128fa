"""Development timing experiment (DESIGN.md §11 lead "fit / HPDI overlap"):
the C2 call time with the fit kernel's grid capped per CU, and with K4b run
beside the fit kernel on the previous call's wide-window list
(MDFIT_EXP_OVERLAP=1, HPDI columns meaningless there).  Prints one JSON line
per configuration.

    python tools/overlap_exp.py [--taxa 10000]
"""

from __future__ import annotations

import argparse
import json
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
    a = ap.parse_args()
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(a.taxa, seed=1)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    fb = engine.alloc_outputs(a.taxa, opts=opts)
    stream = torch.cuda.current_stream()
    configs = [("base", {}), ("fit4", {"MDFIT_FIT_WAVES_PER_CU": "4"}),
               ("exp", {"MDFIT_EXP_OVERLAP": "1"}),
               ("exp_fit4_hp4", {"MDFIT_EXP_OVERLAP": "1", "MDFIT_FIT_WAVES_PER_CU": "4", "MDFIT_HPDI_WAVES_PER_CU": "4"}),
               ("exp_fit4", {"MDFIT_EXP_OVERLAP": "1", "MDFIT_FIT_WAVES_PER_CU": "4"}),
               ("exp_hp4", {"MDFIT_EXP_OVERLAP": "1", "MDFIT_HPDI_WAVES_PER_CU": "4"}),
               ("exp_fit6_hp2", {"MDFIT_EXP_OVERLAP": "1", "MDFIT_FIT_WAVES_PER_CU": "6", "MDFIT_HPDI_WAVES_PER_CU": "2"}),
               ("base_again", {})]
    keys = {k for _, e in configs for k in e}
    for name, env in configs:
        for k in keys:
            os.environ.pop(k, None)
        # one normal call first: the list the experiment drains
        engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
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
        print(json.dumps({"config": name, "env": env, "call_ms": round(dt * 1e3, 4),
                          "fit_kernel_ms": round(fit_ms / n, 4), "fits_per_s": round(a.taxa / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
