"""Print the persistent grids the library sizes (MDFIT_DEV_GRID=1) for a MAP
C2 call and a short NUTS call, and time the NUTS chain kernel at forced
waves-per-CU (MDFIT_DEV_PER_CU) -- development probe of the occupancy API.

    python tools/grid_probe.py [--nuts-taxa 100000] [--per-cu 6,12]
"""

from __future__ import annotations

import argparse
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def child(mode: str, taxa: int, steps: int) -> None:
    sys.path.insert(0, str(ROOT))
    import time

    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(taxa, seed=2 if mode == "nuts" else 1)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    o = _lib.default_opts(mode=_lib.MODE_NUTS if mode == "nuts" else _lib.MODE_MAP)
    res = engine.fit_batch_device(ty, tN, tm, o)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        engine.fit_batch_device(ty, tN, tm, o, res)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    st = res.status.cpu().numpy()
    print(f"{mode} taxa {taxa} per_cu {os.environ.get('MDFIT_DEV_PER_CU', 'api')}: {dt * 1e3:.2f} ms/call "
          f"ok {(st == 0).mean():.4f}", flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", default="")
    ap.add_argument("--nuts-taxa", type=int, default=100_000)
    ap.add_argument("--map-taxa", type=int, default=10_000)
    ap.add_argument("--per-cu", default="")
    a = ap.parse_args()
    if a.child:
        mode, taxa, steps = a.child.split(":")
        child(mode, int(taxa), int(steps))
        return
    env = dict(os.environ, MDFIT_DEV_GRID="1")
    runs = [("map", a.map_taxa, 20), ("nuts", a.nuts_taxa, 1)]
    for mode, taxa, steps in runs:
        subprocess.run([sys.executable, __file__, "--child", f"{mode}:{taxa}:{steps}"], env=env, check=True)
    for pc in [p for p in a.per_cu.split(",") if p]:
        for mode, taxa, steps in runs:
            subprocess.run([sys.executable, __file__, "--child", f"{mode}:{taxa}:{steps}"],
                           env=dict(env, MDFIT_DEV_PER_CU=pc), check=True)


if __name__ == "__main__":
    main()
