"""One NUTS call (T taxa, seed 2) of a given build of libmdfit plus the
sampler's register-only probe, for rocprofv3 --pmc passes (the chain kernel's
instruction mix per wave-trip against the probe's per iteration):

    rocprofv3 --pmc <8 SQ counters> -d DIR -o run --output-format csv -- \
        python3 tools/nuts_counters.py [LIB] [--taxa 20000]
    python tools/nuts_counters.py --summary DIR...   (locally: per kernel, per wave)
"""

from __future__ import annotations

import argparse
import csv
import ctypes
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def run(lib_path, taxa):
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    lib = _lib.load(lib_path) if lib_path else _lib.load()
    b = generate(taxa, seed=2)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    o = _lib.default_opts(mode=_lib.MODE_NUTS)
    res = engine.alloc_outputs(taxa, opts=o)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.mdfit_fit_batch(ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()),
                                   ctypes.c_void_p(tm.data_ptr()), taxa, ctypes.byref(o),
                                   ctypes.c_void_p(res.out.data_ptr()), ctypes.c_void_p(res.pred.data_ptr()),
                                   ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(res.workspace.data_ptr()), s))
    torch.cuda.synchronize()
    util = res.workspace[128:144].view(torch.int64).cpu().numpy()
    n_waves, iters = 256 * 20, 32
    sink = torch.empty(n_waves * 64, dtype=torch.float64, device="cuda")
    _lib.check(lib.mdfit_nuts_peak_probe(n_waves, iters, ctypes.c_void_p(sink.data_ptr()), s))
    torch.cuda.synchronize()
    print(json.dumps({"lib": lib_path, "taxa": taxa, "wave_trips": int(util[0]), "slot_trips": int(util[1]),
                      "probe_waves": n_waves, "probe_iters": iters}), flush=True)


def summary(dirs):
    for d in dirs:
        agg = defaultdict(lambda: defaultdict(float))
        for p in Path(d).rglob("*counter_collection.csv"):
            with open(p) as f:
                for r in csv.DictReader(f):
                    k = r["Kernel_Name"]
                    k = "chain" if "nuts_chain" in k else ("probe" if "probe" in k else ("post" if "post" in k else None))
                    if k is None:
                        continue
                    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        print(d)
        for k, c in agg.items():
            w = c.get("SQ_WAVES", 0.0)
            print(" ", k, json.dumps({n: v for n, v in sorted(c.items())}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=None)
    ap.add_argument("--taxa", type=int, default=20_000)
    ap.add_argument("--summary", nargs="*")
    a = ap.parse_args()
    if a.summary:
        summary(a.summary)
    else:
        run(a.lib, a.taxa)
