"""Per-kernel SQ wave-cycle decomposition from a tools/sq_pass.sh directory:
per launch averages of the 8 counters, and derived shares (VALU-active,
issue-stalled and parked fractions of wave cycles; VALU instructions per wave).

    python tools/sq_summary.py gpurun_out/sq125 [...]
"""

from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def summarise(d: Path) -> dict:
    files = sorted(d.rglob("*counter_collection.csv"))
    if not files:
        return {"error": f"no counter_collection.csv under {d}"}
    acc: dict = defaultdict(lambda: defaultdict(list))
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0].replace("void ", "")
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, c in acc.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        waves = m.get("SQ_WAVES", 0.0)
        row = {"launches": len(c.get("SQ_WAVES", [])), **{n: round(v, 1) for n, v in m.items()}}
        if wc > 0:
            row["valu_active_frac"] = round(m.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4)
            row["issue_stall_frac"] = round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
            row["parked_frac"] = round(m.get("SQ_WAIT_ANY", 0) / wc, 4)
        if waves > 0:
            row["valu_per_wave"] = round(m.get("SQ_INSTS_VALU", 0) / waves, 1)
            row["salu_per_wave"] = round(m.get("SQ_INSTS_SALU", 0) / waves, 1)
        out[k] = row
    return out


def main() -> None:
    res = {Path(d).name: summarise(Path(d)) for d in sys.argv[1:]}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
