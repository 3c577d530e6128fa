"""Config C5: streamed counts -> fits over several input files (SURVEY.md
§8(d): 10 files x 100k TaxIDs in the 22-column format, file i from seed
100+i, 5 % of the taxa built to fail the cuts).

Two measurements:
  * --stages: each stage of the per-file driver timed in isolation (count
    ingest + cut + sort, counts parquet, packing, GPU fit, result frames,
    result parquets) on the first files;
  * the end-to-end driver, main.main() -- reader / writer threads overlapped,
    files dealt to ranks under torchrun -- timed from the first read to the
    last parquet written (max over ranks), reported as taxa fitted per second.

    python tools/c5_pipeline.py --files 10 --taxa 100000 --inference map
    python tools/c5_pipeline.py --stages 0 --check   # + every file's frames vs the oracle

--check (MAP, after the timed run, outside it): each file's counts parquet is
packed again and fitted by the CPU oracle (oracle/, the checker only); the
driver's written result frame must keep exactly the oracle's status-0 taxa, and
every result column is compared (the frames store float32) with bench.py's
metric |gpu - cpu| / max(|cpu|, 1e-2).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from multiprocessing import Pool
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def _gen(args):
    path, taxa, seed = args
    from metadamage_amd.synthetic import generate, to_counts_table

    if not Path(path).exists():
        tmp = Path(str(path) + ".tmp")
        to_counts_table(generate(taxa, seed=seed, fail_fraction=0.05)).to_csv(tmp, sep="\t", header=False,
                                                                               index=False)
        tmp.rename(path)
    return path


def _cfg(out_dir, inference):
    from metadamage_amd import utils

    return utils.Config(out_dir=out_dir, max_fits=None, max_cores=1, min_alignments=10, min_y_sum=10,
                        substitution_bases_forward="CT", substitution_bases_reverse="GA", forced=True,
                        version="0.0.0", inference=inference)


def stages(files, out_dir, inference):
    import torch

    from metadamage_amd import counts, fits, io

    for f in files:
        cfg = _cfg(out_dir, inference)
        cfg.add_filename(f)
        t = {"file": f.name}
        c = time.process_time()
        s = time.perf_counter()
        df = counts.compute_counts(cfg)
        t["ingest_s"] = time.perf_counter() - s
        t["ingest_cpu"], c = time.process_time() - c, time.process_time()
        s = time.perf_counter()
        io.Parquet(cfg.filename_counts).save(df, metadata=cfg.to_dict())
        t["counts_parquet_s"] = time.perf_counter() - s
        t["counts_parquet_cpu"], c = time.process_time() - c, time.process_time()
        s = time.perf_counter()
        p = fits.pack_counts(df, cfg)
        t["pack_s"] = time.perf_counter() - s
        t["pack_cpu"], c = time.process_time() - c, time.process_time()
        s = time.perf_counter()
        out, pred, st = fits.fit_packed(p, fits.make_opts(cfg), shard=False)
        torch.cuda.synchronize()
        t["fit_s"] = time.perf_counter() - s
        t["fit_cpu"], c = time.process_time() - c, time.process_time()
        s = time.perf_counter()
        keep = st == 0
        dfr = fits.make_df_fit_results(p, out, keep, cfg)
        dfp = fits.make_df_fit_predictions(p, pred, keep, cfg)
        t["frames_s"] = time.perf_counter() - s
        t["frames_cpu"], c = time.process_time() - c, time.process_time()
        s = time.perf_counter()
        io.Parquet(cfg.filename_fit_results).save(dfr, metadata=cfg.to_dict())
        io.Parquet(cfg.filename_fit_predictions).save(dfp, metadata=cfg.to_dict())
        t["results_parquet_s"] = time.perf_counter() - s
        t["results_parquet_cpu"] = time.process_time() - c
        t["taxa"] = int(p.n_taxa)
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in t.items()}), flush=True)


def _trace_wrappers():
    """Wrap the pipeline's stage functions to record (thread, stage, t0, t1):
    the per-thread busy time and the critical path of main.main()."""
    import threading

    from metadamage_amd import counts, fits, ingest, io

    events = []

    def wrap(mod, name, label):
        f = getattr(mod, name)

        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                events.append((threading.current_thread().name, label, t0, time.perf_counter()))

        setattr(mod, name, g)

    wrap(counts, "compute_counts", "ingest")
    wrap(fits, "pack_counts", "pack")
    wrap(fits, "fit_packed", "fit")
    wrap(fits, "make_df_fit_results", "frame_results")
    wrap(fits, "make_df_fit_predictions", "frame_predictions")
    wrap(io.Parquet, "save", "parquet")
    wrap(fits, "get_fits", "get_fits")
    wrap(fits, "get_top_max_fits", "top_n")
    wrap(ingest, "noise", "noise")
    wrap(ingest, "read_table", "parse")
    return events


def _trace_summary(events, t_start, wall):
    by = {}
    for th, label, t0, t1 in events:
        d = by.setdefault(th, {})
        d[label] = d.get(label, 0.0) + (t1 - t0)
    return {"wall_s": round(wall, 3), "threads": {th: {k: round(v, 3) for k, v in d.items()} for th, d in by.items()},
            "timeline": [[th, label, round(t0 - t_start, 3), round(t1 - t_start, 3)] for th, label, t0, t1 in
                         sorted(events, key=lambda e: e[2])]}


def check(files, out_dir, inference, threads=16):
    """The full-size C5 run against the oracle, one JSON line per file."""
    import numpy as np

    from metadamage_amd import _lib, fits, io
    from oracle.oracle import OracleLib

    oracle = OracleLib()
    for f in files:
        cfg = _cfg(out_dir, inference)
        cfg.add_filename(f)
        dfr = io.Parquet(cfg.filename_fit_results).load()
        p = fits.pack_counts(io.Parquet(cfg.filename_counts).load(), cfg)
        t0 = time.perf_counter()
        ref, _, rst = oracle.fit_batch(p.y, p.N, p.mm, threads=threads)
        cpu_s = time.perf_counter() - t0
        keep = rst == _lib.OK
        tids = np.asarray(p.tax_id, dtype=np.int64)
        got = dfr.set_index(dfr["tax_id"].astype(np.int64))
        same_set = bool(len(got) == keep.sum() and np.array_equal(np.sort(got.index.to_numpy()), np.sort(tids[keep])))
        rows = {t: i for i, t in enumerate(tids)}
        common = tids[keep]
        ri = np.array([rows[t] for t in common], dtype=np.int64)
        worst, per = 0.0, {}
        for j, name in enumerate(_lib.RESULT_FIELDS):
            a = got.loc[common, name].to_numpy(np.float64)
            r = ref[ri, j].astype(np.float32).astype(np.float64)
            rel = np.abs(a - r) / np.maximum(np.abs(r), 1e-2)
            rel = np.where(np.isnan(a) & np.isnan(r), 0.0, rel)
            per[name] = float(np.nan_to_num(rel, nan=np.inf).max()) if rel.size else 0.0
            worst = max(worst, per[name])
        wf = max(per, key=per.get) if per else None
        print(json.dumps({"file": Path(f).name, "taxa_packed": int(p.n_taxa), "kept_gpu": int(len(got)),
                          "kept_oracle": int(keep.sum()), "same_kept_taxa": same_set, "max_rel": worst,
                          "worst_field": wf, "within_1e-4": worst < 1e-4, "oracle_s": round(cpu_s, 2),
                          "oracle_threads": threads}), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=10)
    ap.add_argument("--taxa", type=int, default=100_000)
    ap.add_argument("--inference", default="map")
    ap.add_argument("--dir", default="/tmp/mdfit_c5")
    ap.add_argument("--stages", type=int, default=2, help="files to time stage by stage first (0: none)")
    ap.add_argument("--gen-procs", type=int, default=8)
    ap.add_argument("--readers", type=int, default=0, help="files read ahead (main.N_READERS; 0: its default)")
    ap.add_argument("--arrow-threads", type=int, default=0, help="pyarrow.set_cpu_count (0: Arrow's default)")
    ap.add_argument("--trace", action="store_true", help="print the per-thread stage timeline of the driver run")
    ap.add_argument("--check", action="store_true", help="then check every file's result frame against the oracle")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    d = Path(a.dir)
    (d / "in").mkdir(parents=True, exist_ok=True)
    files = [d / "in" / f"c5_{i}.tsv" for i in range(a.files)]
    s = time.perf_counter()
    if rank == 0:
        with Pool(min(a.gen_procs, a.files)) as pool:
            pool.map(_gen, [(f, a.taxa, 100 + i) for i, f in enumerate(files)])
        print(json.dumps({"generated_s": round(time.perf_counter() - s, 1),
                          "bytes": sum(f.stat().st_size for f in files)}), flush=True)
    if world > 1:
        dist.barrier()
    torch.cuda.init()
    torch.empty(1, device="cuda")
    from metadamage_amd import engine
    from metadamage_amd import main as driver
    from metadamage_amd.synthetic import generate

    b = generate(64, seed=1)  # load the HIP library and warm the fit path outside the timed region
    engine.fit_batch(b.y, b.N, b.mm)
    if rank == 0 and a.stages:
        stages(files[: a.stages], d / "out_stages", a.inference)
    cfg = _cfg(d / "out", a.inference)
    cfg.add_filenames(files)
    if a.readers:
        driver.N_READERS = a.readers
    if a.arrow_threads:
        import pyarrow

        pyarrow.set_cpu_count(a.arrow_threads)
    if world > 1:
        dist.barrier()
    events = _trace_wrappers() if a.trace else None
    torch.cuda.synchronize()
    c = time.process_time()
    s = time.perf_counter()
    res = driver.main(files, cfg)
    torch.cuda.synchronize()
    wall = time.perf_counter() - s
    cpu = time.process_time() - c
    if events is not None and rank == 0:
        print(json.dumps({"trace": _trace_summary(events, s, wall)}), flush=True)
    taxa = sum(len(r[0]) for r in res.values() if r[0] is not None)
    if world > 1:
        t = torch.tensor([wall, float(taxa)], dtype=torch.float64, device="cuda")
        w = t.clone()
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        wall, taxa = float(w[0]), int(t[1])
    if rank == 0:
        print(json.dumps({"config": "C5", "inference": a.inference, "files": a.files, "ranks": world,
                          "taxa_fitted": taxa, "wall_s": round(wall, 3), "taxa_per_s": round(taxa / wall, 1),
                          "s_per_file": round(wall * world / a.files, 3),
                          "process_cpu_s": round(cpu, 2)}), flush=True)
    if a.check:
        from metadamage_amd.utils import extract_name

        mine = [f for f in files if extract_name(f) in res]
        check(mine, d / "out", a.inference)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
