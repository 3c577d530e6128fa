"""Benchmark: TaxID damage fits/s of the MI355X MAP fit engine (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): 10,000 synthetic TaxIDs
per GPU x 30 positions (z = +-1..15), seed 1 (+ rank), MAP beta-binomial fit of
model_PMD and model_null on all / forward / reverse positions (the 6 sub-fits
the reference runs per TaxID, fits.py:438-439, 311-313, 333-335), the record
assembly, noise estimates and per-position predictions.  One step = one
mdfit_fit_batch launch over the rank's shard with inputs already resident in HBM,
plus (N > 1) the single RCCL gather of the packed result records to rank 0
(asynchronous, overlapping the next step's fit; every gather has completed
before the clock stops).
Weak scaling: every rank fits its own 10,000 taxa.

Printed JSON (rank 0): the driver contract fields plus
  roofline          HBM roofline of the fit kernel (algorithmic bytes / kernel
                    time, HIP events on the launch stream; traffic from the
                    committed rocprofv3 PMC pass, profiles/)
  compute_roofline  useful point-evaluations/s vs the register-only probe of the
                    same point evaluation (the kernel's real bound: FP64 VALU)
  cpu_baseline      the CPU oracle (C/OpenMP restatement of the same fit,
                    oracle/mdfit_oracle.c) on the same 10k-taxon workload
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

TAXA_PER_GPU = 10_000
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# algorithmic bytes per taxon:
#  whole call: y,N 2x30x4 + mismatch 30x12x4 in, 25 result fields x8 +
#              predictions 3x30x4 + status 4 out
#  fit_kernel: y,N 2x30x4 + 6 initial points 6x4x8 in, 6 sub-fit records 6x8x8 out
CALL_BYTES_PER_TAXON = 240 + 1440 + 200 + 360 + 4
FIT_BYTES_PER_TAXON = 240 + 192 + 384
NPTS = np.array([30, 30, 15, 15, 15, 15])


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default: 20 (MAP), 1 (NUTS, ~17 s per step)")
    ap.add_argument("--warmup", type=int, default=None, help="default: 3 (MAP), 1 (NUTS)")
    ap.add_argument("--taxa", type=int, default=0, help="taxa per GPU (default: 10k MAP / 100k NUTS)")
    ap.add_argument("--mode", choices=["map", "nuts"], default="map",
                    help="map: config C2 (the headline); nuts: config C3, the reference's sampler")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = 20 if a.mode == "map" else 1
    if a.warmup is None:
        a.warmup = 3 if a.mode == "map" else 1
    return a


def pmc_traffic(kernel: str = "fit_kernel", taxa: int = TAXA_PER_GPU):
    """Per-launch HBM bytes of `kernel` from the committed rocprofv3 PMC
    summary (profiles/pmc_<kernel>.json) when it was measured at this batch
    size, else None."""
    f = ROOT / "profiles" / f"pmc_{kernel}.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return d.get("hbm_bytes_per_launch") if d.get("taxa_per_launch") == taxa else None
    except Exception:
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from metadamage_amd import _lib, engine
    from metadamage_amd.distributed import alloc_records, gather_records
    from metadamage_amd.synthetic import generate

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    # ---- synthetic shard, resident in HBM before timing -------------------
    nuts = args.mode == "nuts"
    T = args.taxa or (100_000 if nuts else TAXA_PER_GPU)
    b = generate(T, seed=(2 if nuts else 1) + rank)  # C2 seed 1, C3 seed 2
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm, device=dev)
    # N > 1: two record sets, so the gather of step i (async, on the backend's
    # stream) overlaps the fit of step i+1; a set is refilled only after its
    # previous gather has been waited for (the way a multi-batch run overlaps
    # its exchange with the next batch's fit)
    recs = [alloc_records(T, dev) for _ in range(2 if world > 1 and not nuts else 1)]
    fbs = [engine.FitBatch(r.out, r.pred, r.status) for r in recs]
    pending = [None] * len(recs)
    opts = _lib.default_opts(mode=_lib.MODE_NUTS if nuts else _lib.MODE_MAP, index_base=rank * T)
    stream = torch.cuda.current_stream(dev)
    n_step = [0]

    def step():
        k = n_step[0] % len(recs)
        n_step[0] += 1
        if pending[k] is not None:
            pending[k].wait()
            pending[k] = None
        engine.fit_batch_device(ty, tN, tm, opts, fbs[k], stream=stream)
        if world > 1:
            _, pending[k] = gather_records(recs[k].stage(), T, rank, world, async_op=True)

    def drain():
        for k, w in enumerate(pending):
            if w is not None:
                w.wait()
                pending[k] = None

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    # HIP events on the launch stream, recorded by the library around
    # fit_kernel only (torch events see only torch's stream; two more events
    # per call around the whole call cost ~1.5 % of the step, so the call time
    # is the step time)
    engine.profile_enable(True, fit_only=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    _, fit_ms_sum, n_calls = engine.profile_read()
    call_ms_sum = elapsed * 1e3 / args.steps * n_calls  # the step (one call + its gather) by the wall clock
    engine.profile_enable(False)
    assert n_calls == min(args.steps, 256), (n_calls, args.steps)  # the library keeps up to 256 calls

    # per-rank diagnostics of the last step
    last = recs[(n_step[0] - 1) % len(recs)]
    res, out, status = fbs[(n_step[0] - 1) % len(recs)], last.out, last.status
    o = out.cpu().numpy()
    st = status.cpu().numpy()
    evals = o[:, _lib.F_DIAG + 5 :: _lib.DIAG_STRIDE][:, :6]
    useful_pe = float((evals * NPTS).sum())
    # position slots the fit kernel's 32-lane groups spent: an all-position fit
    # holds 30 slots per evaluation, a fwd/rev pair 2x15 until its longer half ends
    group_evals = evals[:, 0] + evals[:, 1] + np.maximum(evals[:, 2], evals[:, 3]) + np.maximum(evals[:, 4], evals[:, 5])
    slot_pe = float(30 * group_evals.sum())

    if rank == 0 and nuts:
        smp = engine.samples_view(res, T, opts)[:64].cpu().numpy()
        print(json.dumps(nuts_line(args, T, world, elapsed, call_ms_sum, fit_ms_sum, n_calls, o, st, b, smp)),
              flush=True)
    elif rank == 0:
        total = T * world * args.steps
        value = total / elapsed
        k_avg_s = fit_ms_sum / n_calls / 1e3
        call_avg_s = call_ms_sum / n_calls / 1e3
        achieved = FIT_BYTES_PER_TAXON * T / k_avg_s / 1e9
        traffic = pmc_traffic("fit_kernel", T)
        # compute roofline: register-only probe of the same point evaluation
        n_waves, iters = 256 * 16, 64
        engine.peak_probe(n_waves, iters, stream=stream)  # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(3):
            engine.peak_probe(n_waves, iters, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        probe_rate = 3 * n_waves * 60 * iters / (e0.elapsed_time(e1) / 1e3)  # 60 points per wave-iteration
        useful_rate = useful_pe / k_avg_s
        line = {
            "metric": "TaxID damage fits/sec",
            "value": round(value, 1),
            "unit": "fits/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8(d) generator, seed 1+rank)",
            "config": {
                "workload": "C2: 10k synthetic TaxIDs x +-15 positions per GPU, MAP beta-binomial damage fit "
                "(model_PMD + model_null on all/forward/reverse = 6 sub-fits per TaxID) + record assembly",
                "taxa_per_gpu": T,
                "positions": 30,
                "parallelism": f"taxon-shard x{world}" + (" + RCCL gather" if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "fit_kernel",
                "note": "HBM fraction is structural (816 B per taxon against ~1e3 FP64 point evaluations); "
                "the kernel is FP64-VALU / latency bound: see compute_roofline (SURVEY.md 8(d), DESIGN.md 4)",
                "kernel_ms_avg": round(k_avg_s * 1e3, 4),
                "bytes_per_taxon": FIT_BYTES_PER_TAXON,
                "call_ms_avg": round(call_avg_s * 1e3, 4),
                "call_bytes_per_taxon": CALL_BYTES_PER_TAXON,
                "call_achieved": round(CALL_BYTES_PER_TAXON * T / call_avg_s / 1e9, 3),
            },
            "compute_roofline": {
                "bound": "fp64-valu",
                "achieved": round(useful_rate, 1),
                "peak": round(probe_rate, 1),
                "unit": "point-evals/s",
                "frac": useful_rate / probe_rate,
                "slot_util": useful_pe / slot_pe,
                "point_evals_per_taxon": useful_pe / T,
            },
            "status_ok_frac": float((st == 0).mean()),
        }
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N=1 figure
            line["cpu_baseline"], ref = cpu_baseline(b, args.cpu_threads)
            line["parity"] = parity(o, st, *ref[::2], kind="bitwise-algorithm (same MDFIT-MAP v1 as the oracle)")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def nuts_line(args, T, world, elapsed, call_ms_sum, fit_ms_sum, n_calls, o, st, b, smp):
    """The JSON line of config C3 (the reference's NUTS, 500 warmup + 1000 draws
    per sub-fit, 6 sub-fits per taxon)."""
    from metadamage_amd import _lib

    S, W = 1000, 500
    k_avg_s = fit_ms_sum / n_calls / 1e3
    # chain kernel: y,N in; 6 x S draws of 4 doubles + 6 x 4 diagnostics out
    bytes_per_taxon = 240 + 6 * S * 32 + 6 * 32
    achieved = bytes_per_taxon * T / k_avg_s / 1e9
    leap = o[:, _lib.F_DIAG + 5 :: _lib.DIAG_STRIDE][:, :6]  # mean leapfrogs per kept iteration
    point_evals = float((leap * NPTS).sum() * (W + S))  # (warmup iterations counted at the kept rate)
    line = {
        "metric": "TaxID damage fits/sec",
        "value": round(T * world * args.steps / elapsed, 2),
        "unit": "fits/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md §8(d) generator, seed 2+rank)",
        "config": {
            "workload": "C3: synthetic TaxIDs x +-15 positions per GPU, full Bayesian fit: NUTS 500 warmup + 1000 "
            "draws for model_PMD + model_null on all/forward/reverse (6 chains per TaxID), WAIC, predictive "
            "median/HPDI",
            "taxa_per_gpu": T,
            "positions": 30,
            "parallelism": f"taxon-shard x{world}" + (" + RCCL gather" if world > 1 else ""),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 3),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": pmc_traffic("nuts_chain_kernel", T),
            "kernel": "nuts_chain_kernel",
            "note": "HBM fraction is structural (the draws written, 192 KB per taxon, against ~2e6 leapfrog "
            "point evaluations); the kernel is FP64-VALU / latency bound (DESIGN.md 9)",
            "kernel_ms_avg": round(k_avg_s * 1e3, 3),
            "bytes_per_taxon": bytes_per_taxon,
            "call_ms_avg": round(call_ms_sum / n_calls, 3),
        },
        "leapfrog_point_evals_per_s": round(point_evals / k_avg_s, 1),
        "mean_leapfrogs_per_iteration": round(float(leap.mean()), 3),
        "status_ok_frac": float((st == 0).mean()),
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"], ref = cpu_baseline_nuts(b, args.cpu_threads)
        line["parity"] = nuts_parity(smp, st, ref)
    return line


def _mcse(x, nb=20):
    """Batch-means Monte-Carlo standard error of the mean along the last axis."""
    m = x.shape[-1] // nb
    bm = x[..., : m * nb].reshape(x.shape[:-1] + (nb, m)).mean(-1)
    return bm.std(-1, ddof=1) / np.sqrt(nb)


def nuts_parity(smp, st, ref):
    """Full-length chains agree with the CPU oracle in distribution only
    (the dual averaging amplifies last-ulp lnGamma differences
    until an accept / U-turn decision flips), so parity is measured the way
    tests/test_gpu_nuts.py does: per taxon, sub-fit and parameter, the
    difference of the posterior means in units of the combined batch-means
    MCSE of the two chains.  Same-distribution chains give |z| ~ half-normal
    (median 0.67)."""
    ro, rp, rs, rsmp = ref
    n = len(ro)
    zs = []
    for s in range(6):
        for j in ((0, 1, 2, 3) if s in (0, 2, 3) else (0, 3)):
            a, r = smp[:n, s, :, j], rsmp[:, s, :, j]
            se = np.hypot(_mcse(a), _mcse(r))
            zs.append(np.abs(a.mean(1) - r.mean(1)) / np.maximum(se, 1e-300))
    z = np.concatenate(zs)
    return {
        "kind": "distributional: |posterior mean gpu - cpu| / MCSE over 6 sub-fits x (q, A, c, phi) "
        "(same sampler and Philox streams; DESIGN.md §9)",
        "taxa": int(n),
        "status_match": float((st[:n] == rs).mean()),
        "median_z": float(np.median(z)),
        "frac_z_gt_3": float((z > 3).mean()),
        "max_z": float(z.max()),
        "within_mc_error": bool(np.median(z) < 1.2 and (z > 5).mean() < 0.03),
    }


def parity(out, st, ref_out, ref_st, kind: str, rtol: float = 1e-4):
    """max |delta param| vs the CPU oracle (the metric's second half): per
    result column |gpu - cpu| / max(|cpu|, 1e-2) over the taxa both fitted
    (NaN in both = 0), its maximum and 99.9th percentile, the worst column."""
    from metadamage_amd import _lib

    n = len(ref_out)
    a, r = out[:n, :25], ref_out[:, :25]
    both = (st[:n] == 0) & (ref_st == 0)
    rel = np.abs(a - r) / np.maximum(np.abs(r), 1e-2)
    rel = np.where(np.isnan(a) & np.isnan(r), 0.0, rel)[both]
    if rel.size == 0:
        return {"kind": kind, "taxa": 0}
    col = np.nanmax(rel, axis=0)
    return {
        "kind": kind,
        "taxa": int(both.sum()),
        "status_match": float((st[:n] == ref_st).mean()),
        "max_rel": float(np.nanmax(rel)),
        "p999_rel": float(np.nanquantile(rel.max(axis=1), 0.999)),
        "worst_field": _lib.RESULT_FIELDS[int(np.nanargmax(col))],
        "within_1e-4": bool(np.nanmax(rel) <= rtol),
        "key_fields_max_rel": {f: float(col[_lib.RESULT_FIELDS.index(f)]) for f in (
            "D_max", "q_mean", "concentration_mean", "n_sigma", "asymmetry", "D_max_forward", "D_max_reverse")},
    }


def cpu_baseline_nuts(b, threads: int):
    """The CPU oracle's sampler (oracle/mdfit_nuts.c, C + OpenMP, same
    algorithm) on the first 64 taxa of the workload."""
    from oracle.oracle import OracleLib

    lib = OracleLib()
    nthr = threads if threads > 0 else min(16, os.cpu_count() or 1)
    n = 64
    t0 = time.perf_counter()
    ref = lib.nuts_batch(b.y[:n], b.N[:n], b.mm[:n], threads=nthr, keep_samples=True)
    dt = time.perf_counter() - t0
    n1 = 4
    t1 = time.perf_counter()
    lib.nuts_batch(b.y[:n1], b.N[:n1], b.mm[:n1], threads=1)
    d1 = time.perf_counter() - t1
    return {
        "value": round(n / dt, 2),
        "unit": "fits/s",
        "cores": nthr,
        "kind": "port",
        "sample": f"first {n} taxa of the rank-0 workload on {nthr} OpenMP threads ({dt:.2f} s); "
        f"1-thread rate on the first {n1}: {n1 / d1:.2f} fits/s",
        "single_thread_value": round(n1 / d1, 2),
    }, ref


def cpu_baseline(b, threads: int):
    """The CPU oracle (oracle/libmdfit_oracle.c, C + OpenMP, same algorithm)
    on the same workload, timed on this host's cores."""
    from oracle.oracle import OracleLib

    lib = OracleLib()
    nthr = threads if threads > 0 else min(16, os.cpu_count() or 1)
    lib.fit_batch(b.y[:200], b.N[:200], b.mm[:200], threads=nthr)  # warm
    t0 = time.perf_counter()
    ref = lib.fit_batch(b.y, b.N, b.mm, threads=nthr)
    dt = time.perf_counter() - t0
    n1 = 500
    t1 = time.perf_counter()
    lib.fit_batch(b.y[:n1], b.N[:n1], b.mm[:n1], threads=1)
    d1 = time.perf_counter() - t1
    return {
        "value": round(b.n_taxa / dt, 1),
        "unit": "fits/s",
        "cores": nthr,
        "kind": "port",
        "sample": f"all {b.n_taxa} taxa of the rank-0 workload on {nthr} OpenMP threads ({dt:.2f} s); "
        f"1-thread rate on the first {n1}: {n1 / d1:.1f} fits/s",
        "single_thread_value": round(n1 / d1, 1),
    }, ref


if __name__ == "__main__":
    main()
