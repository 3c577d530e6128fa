"""Benchmark: TaxID damage fits/s of the MI355X fit engine (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

N = 1 (the headline, BASELINE.json configs[1]): 10,000
synthetic TaxIDs x 30 positions (z = +-1..15), seed 1, MAP beta-binomial fit of
model_PMD and model_null on all / forward / reverse positions (the 6 sub-fits
the reference runs per TaxID, fits.py:438-439, 311-313, 333-335), the record
assembly, noise estimates, per-position predictive medians and the exact 68 %
predictive HPDI.  One step = one mdfit_fit_batch launch with inputs resident in
HBM.

N > 1 (configs[3], C4): 1,000,000 TaxIDs in total, strong scaling: rank r fits
its contiguous 1M/N shard and every step ends with the ONE RCCL gather of the
packed result records to rank 0 (synchronous, inside the timed region; no step
overlaps another).  Global taxon i of C4 is row i % 125,000 of C4's synthetic
per-GPU share (seed 3): every rank's shard and the one-GPU base (c4_one_gpu)
fit exactly the same taxa, so value_N / (N * c4_one_gpu) is an exact
efficiency.

The N = 1 line also carries c3_nuts: BASELINE config C3 (100k TaxIDs, the
reference's own inference -- NUTS 500 warmup + 1000 draws on all 6 sub-fits,
fits.py:382-387, 792-799), one warm-up and one timed call, with its rooflines
and its distributional parity against the CPU oracle's sampler.

Printed JSON (rank 0): the driver contract fields plus
  roofline          HBM roofline of the dominant kernel (fit_kernel): SURVEY.md
                    §8(d)'s algorithmic 448 B/taxon / kernel time (HIP events
                    on the launch stream); PMC traffic from profiles/;
                    hbm_intermediate: the 816 B/taxon the kernel actually moves
                    (the K0 -> K1 -> K3 hand-off through the record)
  compute_roofline  useful point-evaluations/s vs the register-only probe of the
                    same point evaluation (the kernel's real bound: FP64 VALU)
  host_to_host      (N = 1) the product call from pinned host buffers: H2D of
                    y, N (+ the mismatch counts), the fit, D2H of the 32 record
                    columns, predictions and status
  cpu_baseline      (N = 1) the CPU oracle (C/OpenMP restatement of the same
                    fit) on the box's core share, median of 5 over the whole
                    workload, with the reference-dispatch-shape figure beside
                    it (tools/cpu_reference_dispatch.py: scipy per taxon, a Pool
                    per 1,000-taxon chunk as fits.py:692-706)
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
C4_TAXA = 1_000_000
C4_SHARE = C4_TAXA // 8  # C4's per-GPU share at N = 8 (seed 3): the rows every C4 shard is cut from
C3_TAXA = 100_000
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# bytes per taxon:
#  algorithmic: y,N 2x30x4 in + 26 numeric result fields x8 out
#  fit_kernel as built: y,N 2x30x4 + 6 initial points 6x4x8 in, 6 sub-fit records 6x8x8 out
#  whole call: y,N + mismatch 30x12x4 in, 25 result fields x8 + predictions
#              3x30x4 + status 4 out
ALG_BYTES_PER_TAXON = 240 + 208
FIT_BYTES_PER_TAXON = 240 + 192 + 384
READY_BYTES_PER_TAXON = 48
CALL_BYTES_PER_TAXON = 240 + 1440 + 200 + 360 + 4
NPTS = np.array([30, 30, 15, 15, 15, 15])
NPTS_POS = 30  # predictive windows per taxon


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default: 20 (MAP), 1 (NUTS, ~17 s per step)")
    ap.add_argument("--warmup", type=int, default=None, help="default: 3 (MAP), 1 (NUTS)")
    ap.add_argument("--taxa", type=int, default=0, help="taxa per GPU (default: 10k MAP / 100k NUTS)")
    ap.add_argument("--mode", choices=["map", "nuts"], default="map",
                    help="map: config C2 (the headline); nuts: config C3, the reference's sampler")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c4-base", action="store_true",
                    help="N=1: skip the C4-on-one-GPU strong-scaling base (c4_one_gpu)")
    ap.add_argument("--no-c3", action="store_true", help="N=1 MAP: skip the C3 NUTS leg (c3_nuts)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the process's core share (affinity, OMP_NUM_THREADS)")
    ap.add_argument("--workload", choices=["c2", "c4"], default=None,
                    help="default: c2 at N = 1 (the headline), c4 (1M taxa, strong scaling) at N > 1")
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


def c4_rows(rank: int, world: int, total: int = C4_TAXA, share: int = C4_SHARE):
    """C4's taxa of `rank`: its contiguous shard [lo, hi) of the `total`
    global taxa, and the rows of the synthetic share they are (global taxon i
    = share row i % share; 1M distinct synthetic taxa take ~1 min to generate
    on the host, the share a few seconds).  Every world size fits the same
    global taxa, so the N > 1 lines and c4_one_gpu divide like for like."""
    from metadamage_amd.distributed import shard_range

    lo, hi = shard_range(total, rank, world)
    return lo, hi, np.arange(lo, hi, dtype=np.int64) % share


def c4_counts(engine, generate, rows, dev):
    """Device y, N, mm of C4's rows (the share, seed 3, copied to the device
    once and gathered there)."""
    import torch

    b = generate(C4_SHARE, seed=3)
    sy, sN, sm = engine.to_device_counts(b.y, b.N, b.mm, device=dev)
    idx = torch.as_tensor(rows, device=dev)
    return tuple(x.index_select(0, idx).contiguous() for x in (sy, sN, sm))


def c4_one_gpu(engine, _lib, generate, dev, stream, steps: int = 3, warmup: int = 1) -> dict:
    """The strong-scaling base of the N>1 lines: C4's 1M TaxIDs fitted on ONE GPU
    in one call, inputs resident in HBM -- the taxa of every N > 1 line's
    shards together (c4_rows)."""
    import torch

    _, _, rows = c4_rows(0, 1)
    ty, tN, tm = c4_counts(engine, generate, rows, dev)
    T = rows.size
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    fb = engine.alloc_outputs(T, device=dev, opts=opts)
    for _ in range(warmup):
        engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ok = float((fb.status == 0).float().mean().item())
    del ty, tN, tm, fb
    torch.cuda.empty_cache()
    return {
        "value": round(T * steps / el, 1),
        "unit": "fits/s",
        "ms_per_step": round(el / steps * 1e3, 3),
        "taxa": T,
        "steps": steps,
        "warmup": warmup,
        "status_ok_frac": ok,
        "data": f"C4's 1M TaxIDs: global taxon i = row i % {C4_SHARE} of the synthetic share (seed 3), as in "
        "the N > 1 shards",
        "note": "the strong-scaling base for the N>1 lines (C4: 1M TaxIDs, 1M/N per rank + one gather): "
        "efficiency_N = value_N / (N * this value)",
    }


def host_cores() -> tuple[int, int]:
    """(threads to use, CPUs visible): the process's affinity set, capped by
    OMP_NUM_THREADS when the box sets it (its CPU share for one GPU)."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(visible, share) if share > 0 else visible), (os.cpu_count() or visible)


def ref_dispatch_baseline(cores: int, taxa: int = 1000) -> dict | None:
    """tools/cpu_reference_dispatch.py in a child process, started before this
    process touches the GPU (its Pool forks workers)."""
    import subprocess

    try:
        r = subprocess.run([sys.executable, str(ROOT / "tools" / "cpu_reference_dispatch.py"), "--taxa", str(taxa),
                            "--cores", str(cores)], capture_output=True, text=True, timeout=600, check=True)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # reported, never fatal: the headline does not depend on it
        return {"error": repr(e)[:200]}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    nuts = args.mode == "nuts"
    workload = args.workload or ("c4" if world > 1 and not nuts else "c2")
    cores, visible = host_cores()
    if args.cpu_threads > 0:
        cores = args.cpu_threads
    ref_dispatch = None
    if not args.no_cpu_baseline and world == 1 and not nuts:
        ref_dispatch = ref_dispatch_baseline(cores)  # before any GPU call

    import torch
    import torch.distributed as dist

    from metadamage_amd import _lib, engine
    from metadamage_amd.distributed import alloc_records, gather_records, shard_capacity, shard_range
    from metadamage_amd.synthetic import generate

    # development rehearsal of the N>1 path on a one-GPU box: every rank on
    # cuda:0, gloo instead of RCCL (the gather stages through the host); the
    # measured lines use one GPU per rank and RCCL
    share_gpu = os.environ.get("MDFIT_BENCH_SHARE_GPU") == "1"
    if share_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if share_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    red_dev = torch.device("cpu") if share_gpu else dev

    # ---- synthetic shard, resident in HBM before timing -------------------
    if workload == "c4":
        lo, hi, rows = c4_rows(rank, world)
        T, cap, total_per_step = hi - lo, shard_capacity(C4_TAXA, world), C4_TAXA
        ty, tN, tm = c4_counts(engine, generate, rows, dev)
        b = None
    else:
        T = args.taxa or (C3_TAXA if nuts else TAXA_PER_GPU)
        lo, cap, seed, total_per_step = rank * T, T, (2 if nuts else 1) + rank, T * world
        b = generate(T, seed=seed)  # C2 seed 1, C3 seed 2, C4 seed 3
        ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm, device=dev)
    rec = alloc_records(cap, dev)
    fb = engine.FitBatch(rec.out[:T], rec.pred[:T], rec.status[:T])
    opts = _lib.default_opts(mode=_lib.MODE_NUTS if nuts else _lib.MODE_MAP, index_base=lo)
    stream = torch.cuda.current_stream(dev)

    def step():
        engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
        if world > 1:  # the one gather of the packed records to rank 0 (synchronous)
            buf = rec.stage()
            gather_records(buf, cap, rank, world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # HIP events on the launch stream, recorded by the library around
    # fit_kernel only (torch events see only torch's stream)
    engine.profile_enable(True, fit_only=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    _, fit_ms_sum, n_calls = engine.profile_read()
    call_ms_sum = elapsed * 1e3 / args.steps * n_calls  # the step by the wall clock
    engine.profile_enable(False)
    assert n_calls == min(args.steps, 256), (n_calls, args.steps)  # the library keeps up to 256 calls
    ranks = None
    if world > 1:
        # per-rank split of a step (after the timed region, so its
        # synchronisations stay out of it): the fit call and the gather, by
        # the wall clock over a few extra steps; every rank's pair to rank 0
        nb = max(2, min(args.steps, 5))
        fit_s = gat_s = 0.0
        for _ in range(nb):
            dist.barrier()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
            torch.cuda.synchronize(dev)
            t2 = time.perf_counter()
            gather_records(rec.stage(), cap, rank, world)
            torch.cuda.synchronize(dev)
            fit_s += t2 - t1
            gat_s += time.perf_counter() - t2
        mine = torch.tensor([fit_s / nb * 1e3, gat_s / nb * 1e3, float(T)], dtype=torch.float64, device=red_dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        ranks = [{"rank": r, "taxa": int(v[2].item()), "fit_ms": round(float(v[0].item()), 3),
                  "gather_ms": round(float(v[1].item()), 3)} for r, v in enumerate(allr)]

    o = fb.out.cpu().numpy()
    st = fb.status.cpu().numpy()
    evals = o[:, _lib.F_DIAG + 5 :: _lib.DIAG_STRIDE][:, :6]
    useful_pe = float((evals * NPTS).sum())
    # position slots the fit kernel's 32-lane groups spent: an all-position fit
    # holds 30 slots per evaluation, a fwd/rev pair 2x15 until its longer half ends
    group_evals = evals[:, 0] + evals[:, 1] + np.maximum(evals[:, 2], evals[:, 3]) + np.maximum(evals[:, 4], evals[:, 5])
    slot_pe = float(30 * group_evals.sum())

    if rank == 0 and nuts:
        smp = engine.samples_view(fb, T, opts)[:64].cpu().numpy()
        # the chain kernel's counters of the last call (workspace header, uint64
        # at byte 128 / 136): wave-trips with a running slot, running slot-trips
        util = fb.workspace[128:144].view(torch.int64).cpu().numpy()
        # compute roofline: register-only probe of the same potential evaluation
        probe_rate = nuts_probe_rate(engine, dev, stream)
        print(json.dumps(nuts_line(args, T, world, elapsed, call_ms_sum, fit_ms_sum, n_calls, o, st, b, smp,
                                   util, probe_rate)), flush=True)
    elif rank == 0:
        value = total_per_step * args.steps / elapsed
        k_avg_s = fit_ms_sum / n_calls / 1e3
        call_avg_s = call_ms_sum / n_calls / 1e3
        achieved = ALG_BYTES_PER_TAXON * T / k_avg_s / 1e9
        # the fit kernel's hand-off as built: the record (K0 -> K1 -> K3), and
        # the ready list the HPDI stream kernel consumes beside it (one 48 B
        # entry per taxon: the PMD-all mode, the taxon index, the epoch tag)
        inter_bytes = FIT_BYTES_PER_TAXON * T + READY_BYTES_PER_TAXON * T
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
        if workload == "c4":
            wl = (f"C4: 1M synthetic TaxIDs x +-15 positions sharded over {world} GPUs ({T} on rank 0), MAP "
                  "beta-binomial damage fit (6 sub-fits per TaxID) + record assembly + predictive HPDI, then one "
                  "RCCL gather of the packed fit records to rank 0 per step")
        else:
            wl = ("C2: 10k synthetic TaxIDs x +-15 positions per GPU, MAP beta-binomial damage fit "
                  "(model_PMD + model_null on all/forward/reverse = 6 sub-fits per TaxID) + record assembly + "
                  "exact 68 % predictive HPDI")
        line = {
            "metric": "TaxID damage fits/sec",
            "value": round(value, 1),
            "unit": "fits/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if workload == "c4" else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8(d) generator; " + (
                f"C4: global taxon i = row i % {C4_SHARE} of the seed-3 share, rank r its contiguous 1M/N shard)"
                if workload == "c4" else "C2 seed 1 + rank)"),
            "config": {
                "workload": wl,
                "taxa_total": total_per_step,
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
                "bytes_per_taxon": ALG_BYTES_PER_TAXON,
                "note": "algorithmic bytes per SURVEY.md 8(d) (y,N in + 26 result fields out = 448 B/taxon); the "
                "HBM fraction is structural (~1e3 FP64 point evaluations per taxon): the kernel is FP64-VALU / "
                "latency bound, see compute_roofline (DESIGN.md 4)",
                "kernel_ms_avg": round(k_avg_s * 1e3, 4),
                "hbm_intermediate": {
                    "bytes_per_taxon": round(inter_bytes / T, 1),
                    "bytes_per_launch": inter_bytes,
                    "achieved": round(inter_bytes / k_avg_s / 1e9, 3),
                    "note": "what the kernel moves as built: y,N + the 6 initial points in, the 6 sub-fit records "
                    "out (816 B/taxon: the K0 -> K1 -> K3 hand-off through the record), plus the 48 B ready-list "
                    "entry per taxon (the PMD-all mode handed to the HPDI stream kernel running beside it)",
                },
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
            # items the HPDI stream's early waves handed to the late launch in the
            # last call (their bounded wait): 0 when undisturbed
            "hpdi_deferred_items": int(fb.workspace[128:132].view(torch.int32).item() & ~0x40000000),
        }
        if world == 1 and b is not None:
            line["host_to_host"] = host_to_host(engine, b, opts, dev, max(5, args.steps // 2), generate)
        if ranks is not None:
            from metadamage_amd.distributed import REC_BYTES

            line["per_rank"] = ranks
            # what the one gather moves into rank 0 per step: every peer's
            # padded shard of 496-B records (8 count doubles, 17 result floats,
            # 90 prediction floats, the status)
            line["gather_bytes_to_rank0"] = REC_BYTES * cap * (world - 1)
            line["gather_record_bytes"] = REC_BYTES
            line["gather_model"] = gather_model(REC_BYTES * cap, world, ranks)
            line["per_rank_note"] = ("a step split into the fit call and the one gather by the wall clock, "
                                     "measured after the timed region (synchronised per phase)")
        if (world == 1 and workload == "c2" or workload == "c4" and world > 1) and not args.no_c4_base:
            # the strong-scaling base, measured in the same run on rank 0's GPU
            # (at N > 1 the other ranks wait at the closing barrier):
            # value_N / (N * c4_one_gpu.value) is the C4 scaling efficiency
            line["c4_one_gpu"] = c4_one_gpu(engine, _lib, generate, dev, stream)
        if world == 1 and workload == "c2" and not args.no_c3:
            # config C3, the reference's own inference, in the driver's default run
            del fb, rec
            torch.cuda.empty_cache()
            line["c3_nuts"] = c3_nuts(engine, _lib, generate, dev, stream, args)
        if not args.no_cpu_baseline and world == 1 and b is not None:  # the CPU baseline is an N=1 figure
            line["cpu_baseline"], ref = cpu_baseline(b, cores, visible)
            if ref_dispatch is not None:
                line["cpu_baseline"]["reference_dispatch"] = ref_dispatch
            line["parity"] = parity(o, st, *ref[::2], kind="bitwise-algorithm (same MDFIT-MAP v1.1 as the oracle)")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


XGMI_LINK_GBS = 153.0  # per direct GPU-GPU link of an MI355X node (7 links per GPU, the node's full mesh)


def gather_model(bytes_per_peer: int, world: int, ranks) -> dict:
    """Modelled time of the one gather next to the measured one: every peer's
    shard crosses its own direct xGMI link to rank 0 at once (full mesh), so
    the transfer takes bytes_per_peer / link bandwidth; rank 0's ingress is
    (world - 1) links, never the bound at world <= 8."""
    ms = bytes_per_peer / (XGMI_LINK_GBS * 1e9) * 1e3
    meas = [r["gather_ms"] for r in ranks] if ranks else []
    return {"bytes_per_peer": bytes_per_peer, "link_GBs": XGMI_LINK_GBS, "modelled_ms": round(ms, 4),
            "measured_ms_max": max(meas) if meas else None,
            "note": "one dist.gather of the packed records to rank 0 over RCCL: modelled = bytes per peer / one "
            "xGMI link (the peers send on their own links in parallel); measured = wall clock of the gather call "
            "after the fit, per rank (includes RCCL launch and the rank-0 receive)"}


def nuts_probe_rate(engine, dev, stream) -> float:
    """Point evaluations/s of nuts_probe_kernel, the register-only loop over the
    sampler's potential at the chain kernel's occupancy (the compute ceiling)."""
    import torch

    n_waves, iters = 256 * 20, 32
    engine.peak_probe(n_waves, iters, stream=stream, nuts=True)  # warm
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(3):
        engine.peak_probe(n_waves, iters, stream=stream, nuts=True)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    return 3 * n_waves * 60 * iters / (e0.elapsed_time(e1) / 1e3)  # 60 points per wave-iteration


def c3_nuts(engine, _lib, generate, dev, stream, args) -> dict:
    """BASELINE config C3 inside the default N = 1 run: 100k synthetic TaxIDs
    (seed 2), NUTS 500 warmup + 1000 draws on all 6 sub-fits (the reference's
    inference, fits.py:382-387, 792-799), one warm-up and one timed call
    (inputs resident in HBM, HIP events on the launch stream around the chain
    kernel), with nuts_line's rooflines, CPU baseline and 64-taxon
    distributional parity."""
    import types

    import torch

    T = C3_TAXA
    b = generate(T, seed=2)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm, device=dev)
    opts = _lib.default_opts(mode=_lib.MODE_NUTS)
    fb = engine.alloc_outputs(T, device=dev, opts=opts)
    engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)  # warm-up call
    torch.cuda.synchronize(dev)
    engine.profile_enable(True, fit_only=True)
    t0 = time.perf_counter()
    engine.fit_batch_device(ty, tN, tm, opts, fb, stream=stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    _, fit_ms_sum, n_calls = engine.profile_read()
    engine.profile_enable(False)
    o = fb.out.cpu().numpy()
    st = fb.status.cpu().numpy()
    smp = engine.samples_view(fb, T, opts)[:64].cpu().numpy()
    util = fb.workspace[128:144].view(torch.int64).cpu().numpy()
    del fb, ty, tN, tm
    torch.cuda.empty_cache()
    probe_rate = nuts_probe_rate(engine, dev, stream)
    a = types.SimpleNamespace(steps=1, warmup=1, no_cpu_baseline=args.no_cpu_baseline, cpu_threads=args.cpu_threads)
    line = nuts_line(a, T, 1, elapsed, elapsed * 1e3, fit_ms_sum, n_calls, o, st, b, smp, util, probe_rate)
    for k in ("metric", "higher_is_better", "vs_baseline", "n_gpus"):
        line.pop(k, None)
    return line


def host_to_host(engine, b, opts, dev, steps: int, generate=None) -> dict:
    """The product call (fits.fit_packed -> engine.fit_batch_host: the chunked
    two-stream dispatch of engine.ChunkedFitter, chunking as its staging
    plans it) timed from the pinned host buffers the pipeline packs into
    (engine.PinnedPack) to pinned host outputs: H2D of y, N and the mismatch
    counts, the fit, D2H of the 32 record columns, predictions and status,
    synchronised per call -- at C2 (10k taxa) and at C4's per-GPU share (125k,
    seed 3), each next to the device-resident call of the same taxa.  Also
    the y, N-only variant (the noise from the host library, ingest.noise,
    timed separately)."""
    import torch

    from metadamage_amd import ingest

    out = {}
    batches = [("c2_10k", b)]
    if generate is not None:
        batches.append(("c4_share_125k", generate(C4_SHARE, seed=3)))
    for name, bb in batches:
        T = bb.n_taxa
        ty, tN, tm = engine.to_device_counts(bb.y, bb.N, bb.mm, device=dev)
        fb = engine.alloc_outputs(T, device=dev, opts=opts)
        for _ in range(2):
            engine.fit_batch_device(ty, tN, tm, opts, fb)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            engine.fit_batch_device(ty, tN, tm, opts, fb)
        torch.cuda.synchronize(dev)
        dev_dt = (time.perf_counter() - t0) / steps
        del ty, tN, tm, fb
        pp = engine.PinnedPack(T)
        y, N, mm = pp.views(T)
        y[:], N[:], mm[:] = bb.y, bb.N, bb.mm
        entry = {"taxa": T, "device_resident_fits_s": round(T / dev_dt, 1), "device_resident_ms": round(dev_dt * 1e3, 4)}
        for kind, use_mm in (("mm_shipped", True), ("y_N_only", False)):
            with engine._STAGING_LOCK:
                st = engine.staging(T, device=dev, opts=opts, with_mm=use_mm)
                chunks = engine.plan_chunks(T, opts, chunk_taxa=st.chunk_cap)
                run = lambda: st.run(y, N, mm if use_mm else None, opts, pinned=pp, chunks=chunks)  # noqa: E731
                run()
                run()
                ts = []
                for _ in range(steps):
                    t0 = time.perf_counter()
                    run()
                    ts.append(time.perf_counter() - t0)
            dt = float(np.median(ts))
            entry[kind] = {"value": round(T / dt, 1), "ms_per_call": round(dt * 1e3, 4), "chunks": len(chunks),
                           "frac_of_device_resident": round(dev_dt / dt, 3),
                           "h2d_bytes_per_taxon": 256 + (1440 if use_mm else 0), "d2h_bytes_per_taxon": 256 + 360 + 4}
        out[name] = entry
        del pp
        engine._STAGING.clear()
        torch.cuda.empty_cache()
    t0 = time.perf_counter()
    ingest.noise(b.mm)
    out["host_noise_ms_c2"] = round((time.perf_counter() - t0) * 1e3, 3)
    out["unit"] = "fits/s"
    out["note"] = ("pinned host y,N (+mm) -> H2D -> fit -> D2H of the 32 record columns, predictions, status, "
                   "median of the calls, each synchronised; chunks > 1: ChunkedFitter's two streams overlap one "
                   "chunk's copies with the other's fit (DESIGN.md 12); the PCIe-inclusive rate is never `value`")
    return out


def nuts_line(args, T, world, elapsed, call_ms_sum, fit_ms_sum, n_calls, o, st, b, smp, util, probe_rate):
    """The JSON line of config C3 (the reference's NUTS, 500 warmup + 1000 draws
    per sub-fit, 6 sub-fits per taxon)."""
    from metadamage_amd import _lib

    S, W = 1000, 500
    k_avg_s = fit_ms_sum / n_calls / 1e3
    # algorithmic bytes per SURVEY.md 8(d): y,N in + 26 result fields + the
    # predictions (30 x 3 float32) out = 808 B/taxon; what the chain kernel moves
    # as built -- y,N in, 6 x S draws of 4 doubles + 6 x 4 diagnostics out, the
    # hand-off to the post kernel -- is the hbm_intermediate figure
    bytes_per_taxon = ALG_BYTES_PER_TAXON + 30 * 3 * 4
    draws_per_taxon = 240 + 6 * S * 32 + 6 * 32
    achieved = bytes_per_taxon * T / k_avg_s / 1e9
    achieved_draws = draws_per_taxon * T / k_avg_s / 1e9
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
            "traffic": pmc_traffic("nuts_chain_cd", T),
            "kernel": "nuts_chain_cd",
            "note": "algorithmic bytes per SURVEY.md 8(d) (y,N in + 26 result fields + 90 prediction values out "
            "= 808 B/taxon); the HBM fraction is structural (~2e6 leapfrog point evaluations per taxon): the kernel "
            "is FP64-VALU / latency bound (DESIGN.md 9); traffic is the PMC-measured HBM bytes, dominated by the draws",
            "kernel_ms_avg": round(k_avg_s * 1e3, 3),
            "bytes_per_taxon": bytes_per_taxon,
            "hbm_intermediate": {
                "bytes_per_taxon": draws_per_taxon,
                "achieved": round(achieved_draws, 3),
                "note": "what the chain kernel moves as built: y,N in, the 6 x 1000 draws (q, A, c, phi) and "
                "diagnostics out -- the hand-off to nuts_post_kernel",
            },
            "call_ms_avg": round(call_ms_sum / n_calls, 3),
        },
        "compute_roofline": {
            "bound": "fp64-valu",
            "achieved": round(15.0 * float(util[1]) / k_avg_s, 1),
            "peak": round(probe_rate, 1),
            "unit": "point-evals/s",
            "frac": 15.0 * float(util[1]) / k_avg_s / probe_rate,
            "slot_util": float(util[1]) / max(1.0, 4.0 * float(util[0])),
            "point_evals_per_taxon": 15.0 * float(util[1]) / T,
            "note": "the chain kernel's potential evaluations (15 points per running chain slot per trip: "
            "leapfrogs, initial points, step-size probes; counted by the kernel) / its time, against "
            "nuts_probe_kernel, a register-only loop over the same potential_cd at the chain kernel's occupancy",
        },
        "leapfrog_point_evals_per_s": round(point_evals / k_avg_s, 1),
        "mean_leapfrogs_per_iteration": round(float(leap.mean()), 3),
        "status_ok_frac": float((st == 0).mean()),
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"], ref = cpu_baseline_nuts(b, args.cpu_threads or host_cores()[0])
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


def cpu_baseline_nuts(b, threads: int):  # threads: the core share (host_cores)
    """The CPU oracle's sampler (oracle/mdfit_nuts.c, C + OpenMP, same
    algorithm) on the first 64 taxa of the workload."""
    from oracle.oracle import OracleLib

    lib = OracleLib()
    nthr = threads if threads > 0 else host_cores()[0]
    n = 64
    t0 = time.perf_counter()
    ref = lib.nuts_batch(b.y[:n], b.N[:n], b.mm[:n], threads=nthr, keep_samples=True)
    dt = time.perf_counter() - t0
    n1 = 32  # the thread scaling on one fixed sample: its first 32 taxa on 1 and on nthr threads
    t1 = time.perf_counter()
    lib.nuts_batch(b.y[:n1], b.N[:n1], b.mm[:n1], threads=1)
    d1 = time.perf_counter() - t1
    t2 = time.perf_counter()
    lib.nuts_batch(b.y[:n1], b.N[:n1], b.mm[:n1], threads=nthr)
    d2 = time.perf_counter() - t2
    return {
        "value": round(n / dt, 2),
        "unit": "fits/s",
        "cores": nthr,
        "kind": "port",
        "sample": f"first {n} taxa of the rank-0 workload on {nthr} OpenMP threads ({dt:.2f} s)",
        "thread_curve": {"taxa": n1, "fits_per_s": {"1": round(n1 / d1, 2), str(nthr): round(n1 / d2, 2)},
                         "efficiency": round(d1 / d2 / nthr, 3)},
        "single_thread_value": round(n1 / d1, 2),
        "host": cpu_host(),
    }, ref


def cpu_host() -> dict:
    """What the CPU baseline runs on: the affinity set, the cgroup CPU quota
    (v2 cpu.max, v1 cfs quota / period), and the physical cores behind the
    affinity set (SMT siblings share one)."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = Path(path).read_text().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and txt and txt[0] != "max":
            quota = round(int(txt[0]) / int(txt[1]), 2)
        elif path.endswith("quota_us") and txt and int(txt[0]) > 0:
            per = int(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
            quota = round(int(txt[0]) / per, 2)
        break
    cores = set()
    for c in aff:
        try:
            t = Path(f"/sys/devices/system/cpu/cpu{c}/topology")
            cores.add(((t / "physical_package_id").read_text().strip(), (t / "core_id").read_text().strip()))
        except OSError:
            cores.add(("?", str(c)))
    return {"affinity_cpus": len(aff), "cgroup_cpu_quota": quota, "physical_cores_in_affinity": len(cores),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpus_in_host": os.cpu_count()}


def cpu_baseline(b, cores: int, visible: int):
    """The CPU oracle (oracle/libmdfit_oracle.c, C + OpenMP, same algorithm)
    on the whole workload, timed on this host's core share: median of 5; plus
    the thread-scaling curve on one fixed sample (the same taxa at every
    thread count)."""
    from oracle.oracle import OracleLib

    lib = OracleLib()
    lib.fit_batch(b.y[:200], b.N[:200], b.mm[:200], threads=cores)  # warm
    times, ref = [], None
    for _ in range(5):
        t0 = time.perf_counter()
        ref = lib.fit_batch(b.y, b.N, b.mm, threads=cores)
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    n_curve = min(b.n_taxa, 2000)
    curve = {}
    for th in sorted({1, 2, 4, 8, 16, cores}):
        if th > cores:
            continue
        ts = []
        for _ in range(3 if th > 1 else 1):
            t1 = time.perf_counter()
            lib.fit_batch(b.y[:n_curve], b.N[:n_curve], b.mm[:n_curve], threads=th)
            ts.append(time.perf_counter() - t1)
        curve[str(th)] = round(n_curve / float(np.median(ts)), 1)
    one = curve["1"]
    return {
        "value": round(b.n_taxa / dt, 1),
        "unit": "fits/s",
        "cores": cores,
        "host_cpus_visible": visible,
        "kind": "port",
        "sample": f"all {b.n_taxa} taxa of the rank-0 workload on {cores} OpenMP threads, median of 5 runs "
        f"({dt:.3f} s; min {min(times):.3f}, max {max(times):.3f})",
        "thread_curve": {
            "taxa": n_curve,
            "fits_per_s": curve,
            "efficiency": {k: round(v / (int(k) * one), 3) for k, v in curve.items()},
            "note": f"the first {n_curve} taxa at every thread count (1 thread: one run, others median of 3)",
        },
        "host": cpu_host(),
        "note": "cores = the process's CPU share (affinity / OMP_NUM_THREADS: 16 per GPU on the box); the "
        "oracle evaluates lnGamma with the reentrant lgamma_r (plain lgamma's global signgam made 16 threads "
        "fight over one cache line: 1.8x one thread until round 3)",
    }, ref


if __name__ == "__main__":
    main()
