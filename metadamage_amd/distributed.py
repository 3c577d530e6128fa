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

# bytes of one packed per-taxon record: out f64[NOUT] | pred f32[3*30] | status i32
REC_OUT = _lib.NOUT * 8
REC_PRED = _lib.NPRED * _lib.NPOS * 4
REC_BYTES = REC_OUT + REC_PRED + 4


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


def packed_views(buf, n: int):
    """Views (out[n, NOUT] f64, pred[n, 3, 30] f32, status[n] i32) into one
    uint8 record buffer of n * REC_BYTES bytes (torch tensor)."""
    o1 = n * REC_OUT
    o2 = o1 + n * REC_PRED
    out = buf[:o1].view(dtype=_torch_dtype("float64")).view(n, _lib.NOUT)
    pred = buf[o1:o2].view(dtype=_torch_dtype("float32")).view(n, _lib.NPRED, _lib.NPOS)
    status = buf[o2 : o2 + 4 * n].view(dtype=_torch_dtype("int32"))
    return out, pred, status


def _torch_dtype(name):
    import torch

    return getattr(torch, name)


def alloc_records(n: int, device):
    import torch

    return torch.empty(n * REC_BYTES, dtype=torch.uint8, device=device)


def gather_records(buf, n_cap: int, rank: int, world: int, group=None):
    """Gather every rank's record buffer (n_cap records each) to rank 0.
    Returns a list of `world` buffers on rank 0, None elsewhere.  This is the
    one collective of the multi-GPU path (ncclGather semantics)."""
    import torch.distributed as dist

    if world == 1:
        return [buf]
    if rank == 0:
        parts = [buf.new_empty(buf.shape) for _ in range(world)]
        dist.gather(buf, gather_list=parts, dst=0, group=group)
        return parts
    dist.gather(buf, dst=0, group=group)
    return None


def unpack_gathered(parts, n_taxa: int, world: int):
    """Concatenate gathered shards back into df_counts order (host numpy)."""
    outs, preds, sts = [], [], []
    for r, part in enumerate(parts):
        lo, hi = shard_range(n_taxa, r, world)
        n_cap = part.numel() // REC_BYTES
        o, p, s = packed_views(part, n_cap)
        outs.append(o[: hi - lo].cpu().numpy())
        preds.append(p[: hi - lo].cpu().numpy())
        sts.append(s[: hi - lo].cpu().numpy())
    return np.concatenate(outs), np.concatenate(preds), np.concatenate(sts)


def env_rank_world() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torch.distributed.run environment."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world
