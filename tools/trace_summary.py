"""Per-kernel duration summary of rocprofv3 kernel-trace directories
(tools/trace_libs.sh): median and mean duration per kernel name.

    python tools/trace_summary.py gpurun_out/trace_*
"""

from __future__ import annotations

import csv
import sys
from pathlib import Path

import numpy as np


def main() -> None:
    for d in sys.argv[1:]:
        p = Path(d)
        if not p.is_dir():
            continue
        files = sorted(p.rglob("*kernel_trace.csv"))
        if not files:
            print(p.name, "no trace")
            continue
        durs: dict[str, list[float]] = {}
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row["Kernel_Name"].split("(")[0]
                    durs.setdefault(name, []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
        print(p.name)
        for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
            v = np.array(v)
            print(f"  {name[:60]:60s} n={len(v):4d} median {np.median(v):9.1f} us  mean {v.mean():9.1f} us")


if __name__ == "__main__":
    main()
