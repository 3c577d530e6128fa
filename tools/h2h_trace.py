"""Timeline of the chunked host-to-host call (run under rocprofv3
--kernel-trace --memory-copy-trace): T taxa in `n` chunks, `reps` calls."""

from __future__ import annotations

import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    T, n, reps = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (125_000, 4, 4)))
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(T, seed=3)
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    pp = engine.PinnedPack(T)
    y, N, mm = pp.views(T)
    y[:], N[:], mm[:] = b.y, b.N, b.mm
    cap = -(-T // n)
    f = engine.ChunkedFitter(cap, opts=opts)
    ch = engine.plan_chunks(T, opts, chunk_taxa=cap)
    for r in range(reps):
        t0 = time.perf_counter()
        f.run(y, N, mm, opts, pinned=pp, chunks=ch)
        print(f"call {r}: {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
