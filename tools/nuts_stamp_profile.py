"""Cycle split of the NUTS chain kernel from a -DMDFIT_STAMP build (diagnostic
only; never quote that build's run time, read its shares).

    tools/build_variant.sh nstamp -DMDFIT_STAMP
    python tools/nuts_stamp_profile.py [--taxa 10000]

Per wave: cycles in the task start, the potential (leapfrog position update +
one potential/gradient), the mode dispatch split into leaf bookkeeping, checkpoints + U-turn checks,
subtree merge, transition end (adaptation / draw) and the rest, the
begin-probe / begin-iteration block, the loop tail, and the loop trips.
"""

from __future__ import annotations

import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", type=int, default=10_000)
    ap.add_argument("--lib", default=str(ROOT / "metadamage_amd" / "libmdfit_nstamp.so"))
    a = ap.parse_args()

    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    lib = _lib.load(a.lib)
    lib.mdfit_nuts_set_stamp.argtypes = [ctypes.c_void_p]
    b = generate(a.taxa, seed=2)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    o = _lib.default_opts(mode=_lib.MODE_NUTS)
    res = engine.alloc_outputs(a.taxa, opts=o)
    stamps = torch.zeros((65536, 16), dtype=torch.int64, device="cuda")
    lib.mdfit_nuts_set_stamp(ctypes.c_void_p(stamps.data_ptr()))
    _lib.check(lib.mdfit_fit_batch(
        ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()),
        a.taxa, ctypes.byref(o), ctypes.c_void_p(res.out.data_ptr()),
        ctypes.c_void_p(res.pred.data_ptr()), ctypes.c_void_p(res.status.data_ptr()),
        ctypes.c_void_p(res.workspace.data_ptr()), None))
    torch.cuda.synchronize()
    s = stamps.cpu().numpy()
    w = s[s[:, 9] > 0]
    tot = w[:, 10].astype(float)
    trips = w[:, 9].astype(float)
    print(f"nuts_chain_kernel: waves {len(w)}  trips/wave {trips.mean():.0f}  cyc/wave {tot.mean():.3g} "
          f"(max {tot.max():.3g}, min {tot.min():.3g})  cyc/trip {tot.sum() / trips.sum():.0f}")
    for j, lab in ((0, "start"), (1, "potential"), (2, "leaf"), (5, "ckpt+uturn"), (6, "merge"),
                   (7, "transition"), (8, "dispatch-rest"), (3, "begin"), (4, "loop-tail")):
        print(f"   {lab:10s} {w[:, j].sum() / trips.sum():8.0f} cyc/trip  {100 * w[:, j].sum() / tot.sum():5.1f}%")


if __name__ == "__main__":
    main()
