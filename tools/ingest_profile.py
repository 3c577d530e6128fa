"""Stage timing of the native count ingest on one C5 file:
mdi_open, mdi_parse_into (by thread count), mdi_select, mdi_gather, the
categoricals, top-N and packing.

    python tools/ingest_profile.py [--taxa 100000] [--threads 1,4,8,16]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--taxa", type=int, default=100_000)
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--dir", default="/tmp/mdfit_ingest_prof")
    a = ap.parse_args()
    import c5_pipeline as c5

    from metadamage_amd import fits
    from metadamage_amd import ingest as I

    d = Path(a.dir)
    d.mkdir(parents=True, exist_ok=True)
    f = d / "f0.tsv"
    c5._gen((f, a.taxa, 100))
    lib = I._load()
    for nt in [int(x) for x in a.threads.split(",")]:
        best = {}
        for _ in range(3):
            s = time.perf_counter()
            h = ctypes.c_void_p()
            lib.mdi_open(str(f).encode(), nt, ctypes.byref(h))
            t_open = time.perf_counter() - s
            n = lib.mdi_rows(h)
            import numpy as np

            cols = [np.empty(n, np.int64) for _ in range(3)]
            counts = np.empty((16, n), np.int64)
            codes = [np.empty(n, np.int32) for _ in range(3)]
            s = time.perf_counter()
            lib.mdi_parse_into(h, *(c.ctypes.data for c in cols), counts.ctypes.data, *(c.ctypes.data for c in codes))
            t_parse = time.perf_counter() - s
            lib.mdi_free(h)
            for k, v in (("open", t_open), ("parse", t_parse)):
                best[k] = min(best.get(k, 1e9), v)
        print(json.dumps({"threads": nt, **{k: round(v, 4) for k, v in best.items()}}), flush=True)

    T = {}

    class P:
        def __getattr__(self, name):
            g = getattr(lib, name)

            def h(*args):
                s = time.perf_counter()
                try:
                    return g(*args)
                finally:
                    T[name] = T.get(name, 0.0) + time.perf_counter() - s
            return h

    for name in ("read_table", "_categoricals", "_frame"):
        g = getattr(I, name)

        def w(*args, _g=g, _n=name, **kw):
            s = time.perf_counter()
            try:
                return _g(*args, **kw)
            finally:
                T[_n] = T.get(_n, 0.0) + time.perf_counter() - s
        setattr(I, name, w)
    I._load = lambda: P()
    cfg = c5._cfg(d / "out", "map")
    cfg.add_filename(f)
    for _ in range(3):
        T.clear()
        s = time.perf_counter()
        df = I.compute_counts(cfg)
        T["compute_counts"] = time.perf_counter() - s
        cfg.set_number_of_fits(df)
        s = time.perf_counter()
        top = fits.get_top_max_fits(df, cfg.N_fits)
        T["top_n"] = time.perf_counter() - s
        s = time.perf_counter()
        fits.pack_counts(top, cfg)
        T["pack"] = time.perf_counter() - s
        print(json.dumps({k: round(v, 4) for k, v in T.items()}), flush=True)


if __name__ == "__main__":
    main()
