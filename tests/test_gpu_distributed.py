"""GPU test of the product's multi-GPU branch (fits.fit_packed with
world > 1): two ranks under the gloo backend share cuda:0,
each fits its contiguous taxon shard with the HIP kernels, the packed records
are staged to the host and gathered once to rank 0 -- and the gathered
records must equal the single-process fit bit for bit (the fit of a taxon
does not depend on its batch: tests/test_gpu_parity.py's order-independence;
the sampler's streams are keyed by the global taxon index)."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from metadamage_amd.distributed import round_like_gather

pytestmark = pytest.mark.gpu


def _frames_equal(p, out, pred, st, ref_out, ref_pred, ref_st):
    """The written frames of the sharded fit (gathered f32-rounded columns) and
    of the single-process fit are identical (fits.make_df_fit_*)."""
    import types

    from metadamage_amd import fits

    cfg = types.SimpleNamespace(shortname="x")
    a = fits.make_df_fit_results(p, out, st == 0, cfg)
    b = fits.make_df_fit_results(p, ref_out, ref_st == 0, cfg)
    assert a.equals(b)
    assert fits.make_df_fit_predictions(p, pred, st == 0, cfg).equals(
        fits.make_df_fit_predictions(p, ref_pred, ref_st == 0, cfg))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, T, mode, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)  # both ranks on the one GPU of the box
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from metadamage_amd import _lib, fits
        from metadamage_amd.synthetic import generate

        b = generate(T, seed=23)
        p = fits.Packed(b.tax_id, b.tax_id.astype(str), np.full(T, "species"), b.N_alignments, b.y, b.N, b.mm)
        opts = _lib.default_opts(mode=mode, num_warmup=20, num_samples=40) if mode == _lib.MODE_NUTS else None
        res = fits.fit_packed(p, opts, shard=True)
        q.put((rank, None if res is None else [np.asarray(a) for a in res]))
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode_name", ["map", "nuts"])
def test_sharded_fit_packed_equals_single_process(mode_name):
    import torch
    import torch.multiprocessing as mp

    from metadamage_amd import _lib, fits
    from metadamage_amd.synthetic import generate

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    mode = _lib.MODE_NUTS if mode_name == "nuts" else _lib.MODE_MAP
    T = 1501 if mode == _lib.MODE_MAP else 61  # ragged shards
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, T, mode, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    got = dict(q.get(timeout=600) for _ in procs)
    for pr in procs:
        pr.join(timeout=120)
    assert got[1] is None, got[1]
    assert not isinstance(got[0], str), got[0]
    out, pred, st = got[0]
    # the single-process reference: the same packed taxa, one call
    b = generate(T, seed=23)
    p = fits.Packed(b.tax_id, b.tax_id.astype(str), np.full(T, "species"), b.N_alignments, b.y, b.N, b.mm)
    opts = _lib.default_opts(mode=mode, num_warmup=20, num_samples=40) if mode == _lib.MODE_NUTS else None
    ref_out, ref_pred, ref_st = fits.fit_packed(p, opts, shard=False)
    assert out.shape == (T, _lib.NRESULT) and ref_out.shape[0] == T  # (the gather carries the 25 result columns)
    assert np.array_equal(st, ref_st)
    assert np.array_equal(out, round_like_gather(ref_out), equal_nan=True)
    assert np.array_equal(pred, ref_pred, equal_nan=True)
    _frames_equal(p, out, pred, st, ref_out, ref_pred, ref_st)


def _rccl_rank(port, T, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        # as distributed.init_from_env joins a torchrun job: the rank's GPU
        # first, then the RCCL group bound to it
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        from metadamage_amd import distributed, fits
        from metadamage_amd.synthetic import generate

        assert dist.get_backend() == "nccl"
        agree = (distributed.all_ranks_agree(True), distributed.all_ranks_agree(False))
        b = generate(T, seed=29)
        p = fits.Packed(b.tax_id, b.tax_id.astype(str), np.full(T, "species"), b.N_alignments, b.y, b.N, b.mm)
        res = fits.fit_packed(p, None, shard=True)  # the sharded branch: device records, one RCCL gather
        q.put((agree, [np.asarray(a) for a in res]))
        distributed.shutdown(ok=True)
    except Exception as e:  # surfaced by the parent
        q.put(repr(e))


def test_rccl_path_in_a_world_of_one():
    """The RCCL ("nccl") branches of the multi-GPU path on the one GPU of the
    box: the group joined as init_from_env does, the agreement all-reduce on
    a device int, fit_packed's sharded branch with its device-buffer gather
    to rank 0 and the batched D2H of unpack_gathered, shutdown's barrier --
    bit-identical to the unsharded fit."""
    import torch
    import torch.multiprocessing as mp

    from metadamage_amd import fits
    from metadamage_amd.synthetic import generate

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    T = 777
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_rccl_rank, args=(_free_port(), T, q))
    pr.start()
    got = q.get(timeout=300)
    pr.join(timeout=120)
    assert not isinstance(got, str), got
    agree, (out, pred, st) = got
    assert agree == (True, False)
    b = generate(T, seed=29)
    p = fits.Packed(b.tax_id, b.tax_id.astype(str), np.full(T, "species"), b.N_alignments, b.y, b.N, b.mm)
    ref_out, ref_pred, ref_st = fits.fit_packed(p, None, shard=False)
    assert np.array_equal(st, ref_st)
    assert np.array_equal(out, round_like_gather(ref_out), equal_nan=True)
    assert np.array_equal(pred, ref_pred, equal_nan=True)
    _frames_equal(p, out, pred, st, ref_out, ref_pred, ref_st)
