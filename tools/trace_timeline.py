"""Print a per-call timeline (kernels and copies, start/end relative to the
first event, ms) from a rocprofv3 --kernel-trace --memory-copy-trace CSV pair."""

from __future__ import annotations

import csv
import sys
from pathlib import Path


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    d = Path(sys.argv[1])
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    ev = []
    for p in d.rglob("*kernel_trace.csv"):
        for r in rows(p):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:40],
                       r.get("Stream_Id", r.get("Queue_Id", ""))))
    for p in d.rglob("*memory_copy_trace.csv"):
        for r in rows(p):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r.get("Direction", r.get("Operation", "")),
                       r.get("Size", r.get("Bytes", ""))))
    ev.sort()
    ev = ev[-last:]
    t0 = ev[0][0]
    for s, e, k, name, extra in ev:
        print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} {(e - s) / 1e6:8.3f} {k} {name} {extra}")


if __name__ == "__main__":
    main()
