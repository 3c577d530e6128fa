"""Summarise the rocprofv3 passes of tools/profile_round.sh into profiles/.

Copies the kernel-trace stats / PMC CSVs of the named round into profiles/ and
writes profiles/pmc_fit_kernel.json (per-launch HBM bytes of fit_kernel,
corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE x2 on gfx950,
WRITE_SIZE as read; both counters are kB).

    python tools/pmc_summary.py r01 gpurun_out/prof
"""

from __future__ import annotations

import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
TAXA = 10_000
FIT_BYTES_PER_TAXON = 240 + 192 + 384  # bench.py
NUTS_TAXA = 100_000
NUTS_BYTES_PER_TAXON = 240 + 6 * 1000 * 32 + 6 * 32  # bench.py nuts_line


def rows(path: Path):
    with open(path) as f:
        yield from csv.DictReader(f)


def counter_mean(path: Path, kernel: str, name: str) -> float:
    v = [float(r["Counter_Value"]) for r in rows(path) if r["Counter_Name"] == name and kernel in r["Kernel_Name"]]
    if not v:
        raise SystemExit(f"no {name} rows for {kernel} in {path}")
    return sum(v) / len(v)


def main() -> None:
    tag, src = sys.argv[1], Path(sys.argv[2])
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    found = {}
    for sub, name, dst in (("trace", "kernel_stats.csv", "kernel_stats.csv"),
                           ("trace", "kernel_trace.csv", "kernel_trace.csv"),
                           ("fetch", "counter_collection.csv", "pmc_fetch_size.csv"),
                           ("write", "counter_collection.csv", "pmc_write_size.csv")):
        cands = sorted((src / sub).rglob(f"*{name}"))
        if not cands:
            raise SystemExit(f"missing {sub}/*{name} under {src}")
        shutil.copy(cands[0], prof / f"{tag}_{dst}")
        found[dst] = prof / f"{tag}_{dst}"
    nuts = sorted((src / "nuts_trace").rglob("*kernel_stats.csv"))
    if nuts:
        shutil.copy(nuts[0], prof / f"{tag}_nuts_kernel_stats.csv")
    for name in ("bench_trace.json", "bench_nuts_trace.json"):
        if (src / name).exists():
            shutil.copy(src / name, prof / f"{tag}_{name}")
    # the fit kernel's hand-off as the traced bench run reports it (the record
    # and the ready-list entries)
    handoff = None
    try:
        line = next(json.loads(x) for x in open(src / "bench_trace.json") if x.startswith("{"))
        handoff = line["roofline"]["hbm_intermediate"].get("bytes_per_launch")
    except Exception:
        pass
    write_summary(prof, tag, "fit_kernel", TAXA, FIT_BYTES_PER_TAXON, 448, found["kernel_stats.csv"],
                  found["pmc_fetch_size.csv"], found["pmc_write_size.csv"], "python bench.py", handoff)
    sq = sorted((src / "sq").rglob("*counter_collection.csv"))
    if sq:
        shutil.copy(sq[0], prof / f"{tag}_pmc_sq.csv")
        sq_decomposition(prof, tag, prof / f"{tag}_pmc_sq.csv")
    # the NUTS chain kernel at config C3 (optional passes)
    nf, nw = sorted((src / "nuts_fetch").rglob("*counter_collection.csv")), sorted((src / "nuts_write").rglob("*counter_collection.csv"))
    if nuts and nf and nw:
        shutil.copy(nf[0], prof / f"{tag}_nuts_pmc_fetch_size.csv")
        shutil.copy(nw[0], prof / f"{tag}_nuts_pmc_write_size.csv")
        write_summary(prof, tag, "nuts_chain_cd", NUTS_TAXA, NUTS_BYTES_PER_TAXON, 808,
                      prof / f"{tag}_nuts_kernel_stats.csv", prof / f"{tag}_nuts_pmc_fetch_size.csv",
                      prof / f"{tag}_nuts_pmc_write_size.csv", "python bench.py --mode nuts")


def sq_decomposition(prof, tag, sq_csv):
    """Per kernel: the SQ counters as fractions of SQ_WAVE_CYCLES (summed over
    dispatches), instructions per wave, SALU per VALU."""
    acc = {}
    for r in rows(sq_csv):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "mdfit" not in k:
            continue
        d = acc.setdefault(k, {"dispatches": set()})
        d["dispatches"].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = {}
    for k, d in acc.items():
        cyc = d.get("SQ_WAVE_CYCLES", 0.0)
        if cyc <= 0:
            continue
        out[k] = {"dispatches": len(d["dispatches"]),
                  **{n.replace("SQ_", "").lower(): round(d.get(n, 0.0) / cyc, 3) for n in
                     ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU")},
                  "valu_insts_per_wave": round(d.get("SQ_INSTS_VALU", 0.0) / max(d.get("SQ_WAVES", 1.0), 1.0), 1),
                  "salu_per_valu": round(d.get("SQ_INSTS_SALU", 0.0) / max(d.get("SQ_INSTS_VALU", 1.0), 1.0), 3)}
    note = ("fractions of SQ_WAVE_CYCLES (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ "
            "WAVE_CYCLES); one rocprofv3 --pmc pass of 8 SQ counters over python bench.py (C2, MAP)")
    (prof / f"{tag}_sq_decomposition.json").write_text(json.dumps({"C2 MAP": out, "note": note}, indent=1) + "\n")
    print(json.dumps(out, indent=1))


def write_summary(prof, tag, name, taxa, bytes_per_taxon, alg_per_taxon, stats_csv, fetch_csv, write_csv, cmd,
                  handoff_override=None):
    # (C2's 10k taxa run the one-point-per-lane layout, fit_kernel<1>: the bench's
    # 125k host-to-host and C4 calls, fit_kernel<2>, are other launches)
    k = f"mdfit::{name}<1>" if name == "fit_kernel" else f"mdfit::nuts::{name}"
    fetch_kb = counter_mean(fetch_csv, k, "FETCH_SIZE")
    write_kb = counter_mean(write_csv, k, "WRITE_SIZE")
    # kernel names as rocprofv3 prints them: "void mdfit::fit_kernel<1>(...)"
    fk = next((r for r in rows(stats_csv) if k in r["Name"].split("(")[0]), {})
    summary = {
        "kernel": k,
        "launches": len([1 for r in rows(fetch_csv) if r["Counter_Name"] == "FETCH_SIZE" and k in r["Kernel_Name"]]),
        "taxa_per_launch": taxa,
        "FETCH_SIZE_kB_mean": fetch_kb,
        "WRITE_SIZE_kB_mean": write_kb,
        "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md §HBM: FETCH_SIZE reports 1/2 of wide coalesced "
        "reads; this kernel's 4-B/lane and broadcast 8-B loads are uncalibrated), WRITE_SIZE x1",
        "hbm_bytes_per_launch": int(round((2 * fetch_kb + write_kb) * 1024)),
        "handoff_bytes_per_launch": handoff_override if handoff_override else bytes_per_taxon * taxa,
        "handoff_note": "what the kernel moves as built (the hand-off to the next kernels: MAP y,N + the 6 initial "
        "points in, the 6 sub-fit records and the 48-B ready-list entry per taxon out; NUTS the draws)",
        "survey_algorithmic_bytes_per_launch": alg_per_taxon * taxa,
        "survey_note": "SURVEY.md 8(d): y,N in + 26 result fields out (+ 90 prediction values for NUTS)",
        "rocprof_avg_ns": float(fk.get("AverageNs", "nan")),
        "source": f"rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; "
        f"{cmd} (profiles/{tag}_*.csv)",
    }
    (prof / f"pmc_{name}.json").write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
