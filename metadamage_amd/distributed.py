"""Taxon sharding across GPUs and the single result gather.

The fit is embarrassingly parallel over taxa (fits.py:428-469 fits one taxon
with no shared state), so the multi-GPU path is: each rank (one process per
GPU, torch.distributed over RCCL) fits a contiguous shard of taxa in df_counts
order, then ONE gather moves every rank's packed result records to rank 0,
which writes the parquet files.  There is no other collective on the data path.

Works with any torch.distributed backend: "nccl" (= RCCL on ROCm, device
tensors) on the GPU box, "gloo" (host tensors) in the CPU tests.
"""

from __future__ import annotations

import os

import numpy as np

from . import _lib

# One gathered per-taxon record: the 25 result columns of out
# (f64[NRES_GATHER]) | pred f32[3*30] | status i32 = 564 bytes.  The record's
# 7 reserved doubles and its 48 per-sub-fit diagnostic doubles stay on the
# rank that fitted them (1004 bytes per taxon otherwise).
NRES_GATHER = _lib.NRESULT
REC_PRED = _lib.NPRED * _lib.NPOS * 4
REC_RES = NRES_GATHER * 8
REC_BYTES = REC_PRED + 4 + REC_RES
REC_OUT = _lib.NOUT * 8  # the full record the kernel writes (rank-local)


def shard_range(n_taxa: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of rank `rank`: ceil-split so shards differ by
    at most one taxon."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    per = -(-n_taxa // world) if n_taxa else 0
    lo = min(rank * per, n_taxa)
    hi = min(lo + per, n_taxa)
    return lo, hi


def shard_capacity(n_taxa: int, world: int) -> int:
    """Padded shard size (every rank gathers the same number of records)."""
    return -(-n_taxa // world) if n_taxa else 0


class Records:
    """Rank-local result buffers of a shard of n taxa: `out` f64[n, NOUT] (the
    kernel's full record), and one uint8 gather buffer `buf` of n * REC_BYTES
    bytes holding res f64[n, NRES_GATHER] | pred f32[n, 3, 30] | status i32[n].
    The kernel writes pred and status in place; `stage()` copies the result
    columns of out into res (one strided device copy) before the gather."""

    def __init__(self, n: int, device):
        import torch

        self.n = n
        self.out = torch.empty((n, _lib.NOUT), dtype=torch.float64, device=device)
        self.buf = torch.empty(n * REC_BYTES, dtype=torch.uint8, device=device)
        self.pred, self.status, self.res = packed_views(self.buf, n)

    def stage(self):
        self.res.copy_(self.out[:, :NRES_GATHER])
        return self.buf


def packed_views(buf, n: int):
    """Views (pred[n, 3, 30] f32, status[n] i32, res[n, NRES_GATHER] f64) into
    one uint8 gather buffer of n * REC_BYTES bytes laid out res | pred | status
    (torch tensor; the f64 block first keeps it 8-byte aligned for any n)."""
    o1 = n * REC_RES
    o2 = o1 + n * REC_PRED
    res = buf[:o1].view(dtype=_torch_dtype("float64")).view(n, NRES_GATHER)
    pred = buf[o1:o2].view(dtype=_torch_dtype("float32")).view(n, _lib.NPRED, _lib.NPOS)
    status = buf[o2 : o2 + 4 * n].view(dtype=_torch_dtype("int32"))
    return pred, status, res


def _torch_dtype(name):
    import torch

    return getattr(torch, name)


def alloc_records(n: int, device) -> Records:
    return Records(n, device)


def gather_records(buf, n_cap: int, rank: int, world: int, group=None, async_op: bool = False):
    """Gather every rank's staged gather buffer (Records.stage(), n_cap records
    each) to rank 0.
    Returns a list of `world` buffers on rank 0, None elsewhere.  This is the
    one collective of the multi-GPU path (ncclGather semantics).  Under the
    gloo backend (CPU tests, or ranks sharing one GPU in a test) a device
    buffer is staged to host first: gloo gathers host tensors only.

    async_op=True returns (parts, work) instead: the collective is queued
    behind the work already on the current stream and runs on the backend's
    own stream, so the caller can fit the next batch into other buffers while
    it moves; `work.wait()` orders the current stream after it (and must
    precede any reuse of `buf` or any read of `parts`)."""
    import torch.distributed as dist

    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return ([buf], None) if async_op else [buf]
    if buf.is_cuda and dist.get_backend(group) == "gloo":
        buf = buf.cpu()
    parts = [buf.new_empty(buf.shape) for _ in range(world)] if rank == 0 else None
    work = dist.gather(buf, gather_list=parts, dst=0, group=group, async_op=async_op)
    return (parts, work) if async_op else parts


def all_ranks_agree(flag: bool) -> bool:
    """True iff `flag` is true on every rank (a one-int all-reduce; no process
    group: flag).
    Used so that all ranks take the same branch before a collective (e.g. a
    cache hit must skip the fit on every rank or on none)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return bool(flag)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def init_from_env(backend: str | None = None) -> tuple[int, int]:
    """Join the torch.distributed job described by the torchrun environment
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*): one process per GPU, the
    rank's GPU selected BEFORE any other device call, backend "nccl" (RCCL
    over xGMI) unless given.  WORLD_SIZE 1 (or unset): nothing to join.
    Returns (rank, world)."""
    rank, local, world = env_rank_world()
    if world <= 1:
        return 0, 1
    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    backend = backend or "nccl"
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return dist.get_rank(), dist.get_world_size()


def shutdown(ok: bool = True) -> None:
    """Leave the process group.  ok=True (the run succeeded on this rank): a
    barrier first, so no rank tears the group down under a peer's last
    collective.  ok=False (this rank raised): no barrier -- an NCCL barrier is
    itself a one-element all-reduce and could pair with a healthy peer's
    agreement all-reduce or result gather, leaving the job hung until the
    collective timeout; the group is torn down (RCCL: the communicator
    aborted) so the peers' pending collectives fail and the job exits."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return
    if ok:
        dist.barrier()
        dist.destroy_process_group()
        return
    from torch.distributed import distributed_c10d as c10d

    abort = getattr(c10d, "_abort_process_group", None)
    if dist.get_backend() == "nccl" and abort is not None:
        abort()  # tears the communicators down without waiting on peers
    if dist.is_initialized():
        dist.destroy_process_group()


def run_distributed(fn, *args, **kwargs):
    """Join the torchrun job (init_from_env), run fn, leave the group: with a
    barrier when fn returned, without one when it raised (shutdown(ok=False)),
    re-raising so the launcher tears the job down."""
    init_from_env()
    try:
        result = fn(*args, **kwargs)
    except BaseException:
        shutdown(ok=False)
        raise
    shutdown(ok=True)
    return result


def unpack_gathered(parts, n_taxa: int, world: int):
    """Concatenate gathered shards back into df_counts order (host numpy);
    the parts may be device (RCCL) or host (gloo) buffers."""
    import torch

    outs, preds, sts = [], [], []
    if parts and parts[0].is_cuda:
        # every part's D2H copy queued at once into one pinned host buffer,
        # then one synchronisation (not a blocking copy per part)
        n = sum(p.numel() for p in parts)
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        off = []
        o0 = 0
        for p in parts:
            host[o0 : o0 + p.numel()].copy_(p, non_blocking=True)
            off.append(o0)
            o0 += p.numel()
        torch.cuda.current_stream(parts[0].device).synchronize()
        parts = [host[o : o + p.numel()] for o, p in zip(off, parts)]
    for r, part in enumerate(parts):
        lo, hi = shard_range(n_taxa, r, world)
        n_cap = part.numel() // REC_BYTES
        p, s, o = packed_views(part, n_cap)
        outs.append(o[: hi - lo].numpy())
        preds.append(p[: hi - lo].numpy())
        sts.append(s[: hi - lo].numpy())
    return np.concatenate(outs), np.concatenate(preds), np.concatenate(sts)


def env_rank_world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world
