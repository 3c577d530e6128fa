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

# One gathered per-taxon record (496 bytes): the 25 result columns of out as
# the frames store them -- the 8 count columns (N_z1_*, N_sum_*, y_sum_*) as
# f64 (exact integers up to 2^53; the frames' uint32 range check runs on rank 0)
# and the 17 others rounded to f32 on the device, as downcast_dataframe rounds
# them (utils.py:329-356: make_df_fit_results writes them float32, so the
# frames are bit-identical to a single-process run) -- | pred f32[3*30] |
# status i32.  The record's 7 reserved doubles and its 48 per-sub-fit
# diagnostic doubles stay on the rank that fitted them.
NRES_GATHER = _lib.NRESULT
INT_LO, INT_HI = 7, 15  # result columns N_z1_forward .. y_sum_total (include/mdfit.h: MDFIT_F_N_Z1_FORWARD ..)
FLOAT_COLS = [j for j in range(NRES_GATHER) if not INT_LO <= j < INT_HI]
REC_INT = (INT_HI - INT_LO) * 8
REC_F32 = len(FLOAT_COLS) * 4
REC_PRED = _lib.NPRED * _lib.NPOS * 4
REC_RES = REC_INT + REC_F32
REC_BYTES = REC_RES + REC_PRED + 4
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
    bytes holding ints f64[n, 8] | floats f32[n, 17] | pred f32[n, 3, 30] |
    status i32[n].  The kernel writes pred and status in place; `stage()`
    copies the result columns of out into ints / floats (two strided device
    copies, the second rounding to f32) before the gather."""

    def __init__(self, n: int, device):
        import torch

        self.n = n
        self.out = torch.empty((n, _lib.NOUT), dtype=torch.float64, device=device)
        self.buf = torch.empty(n * REC_BYTES, dtype=torch.uint8, device=device)
        self.pred, self.status, self.ints, self.floats = packed_views(self.buf, n)
        self._fidx = torch.as_tensor(FLOAT_COLS, device=device)

    def stage(self):
        self.ints.copy_(self.out[:, INT_LO:INT_HI])
        self.floats.copy_(self.out.index_select(1, self._fidx))  # (f64 -> f32: round to nearest even, as numpy)
        return self.buf


def packed_views(buf, n: int):
    """Views (pred[n, 3, 30] f32, status[n] i32, ints[n, 8] f64, floats[n, 17]
    f32) into one uint8 gather buffer of n * REC_BYTES bytes laid out ints |
    floats | pred | status (torch tensor; the f64 block first keeps it 8-byte
    aligned for any n)."""
    o1 = n * REC_INT
    o2 = o1 + n * REC_F32
    o3 = o2 + n * REC_PRED
    ints = buf[:o1].view(dtype=_torch_dtype("float64")).view(n, INT_HI - INT_LO)
    floats = buf[o1:o2].view(dtype=_torch_dtype("float32")).view(n, len(FLOAT_COLS))
    pred = buf[o2:o3].view(dtype=_torch_dtype("float32")).view(n, _lib.NPRED, _lib.NPOS)
    status = buf[o3 : o3 + 4 * n].view(dtype=_torch_dtype("int32"))
    return pred, status, ints, floats


def round_like_gather(out: np.ndarray) -> np.ndarray:
    """The 25 result columns of host records out[T, >= 25] as the gather
    carries them (the 17 non-count columns rounded to f32), float64[T, 25]."""
    o = np.array(out[:, :NRES_GATHER], dtype=np.float64)
    o[:, FLOAT_COLS] = o[:, FLOAT_COLS].astype(np.float32).astype(np.float64)
    return o


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
        p, s, ints, floats = packed_views(part, n_cap)
        o = np.empty((hi - lo, NRES_GATHER), np.float64)
        o[:, INT_LO:INT_HI] = ints[: hi - lo].numpy()
        o[:, FLOAT_COLS] = floats[: hi - lo].numpy()
        outs.append(o)
        preds.append(p[: hi - lo].numpy())
        sts.append(s[: hi - lo].numpy())
    return np.concatenate(outs), np.concatenate(preds), np.concatenate(sts)


def env_rank_world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world
