"""GPU: the bounded-memory chunked dispatch (engine.ChunkedFitter) gives the
records of one mdfit_fit_batch call bit for bit -- MAP below and across the
60k-taxon HPDI switch, the sampler (its Philox streams keyed by index_base +
the chunk's offset), host outputs and in-place device outputs (the sharded
fit's gather records).  The reference's equivalent is its 1,000-taxon chunks
(/root/reference/metadamage/fits.py:692-706): a chunk boundary must not change
any taxon's fit."""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return torch


def _one_call(torch, b, opts):
    from metadamage_amd import engine

    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    r = engine.fit_batch_device(ty, tN, tm, opts)
    torch.cuda.synchronize()
    return r.out.cpu().numpy(), r.pred.cpu().numpy(), r.status.cpu().numpy()


@pytest.mark.parametrize("mode,T,chunk", [("map", 10_000, 3_000), ("map", 70_000, 30_000), ("nuts", 1_000, 350)])
def test_chunked_host_fit_equals_one_call(torch_dev, monkeypatch, mode, T, chunk):
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(T, seed=31)
    opts = _lib.default_opts(mode=_lib.MODE_NUTS if mode == "nuts" else _lib.MODE_MAP)
    if mode == "nuts":
        opts.num_warmup, opts.num_samples = 60, 80
    ref_out, ref_pred, ref_st = _one_call(torch, b, opts)
    monkeypatch.setenv("MDFIT_CHUNK_TAXA", str(chunk))
    assert len(engine.plan_chunks(T, opts)) == -(-T // chunk)
    out, pred, st = engine.fit_batch_host(b.y, b.N, b.mm, opts)
    assert np.array_equal(st, ref_st)
    assert out.shape[1] == 25
    assert np.array_equal(out, ref_out[:, :25], equal_nan=True)
    assert np.array_equal(pred, ref_pred, equal_nan=True)
    assert (st == 0).mean() > 0.99


def test_chunked_into_device_buffers(torch_dev):
    """run_into_device: every chunk's records written in place into the caller's
    device tensors (fits._fit_sharded's gather records), ordered before the
    caller's stream; index_base offsets the sampler's streams."""
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    T = 600
    b = generate(T, seed=32)
    opts = _lib.default_opts(mode=_lib.MODE_NUTS, num_warmup=40, num_samples=60, index_base=1234)
    ref_out, ref_pred, ref_st = _one_call(torch, b, opts)
    fitter = engine.ChunkedFitter(256, opts=opts, dest_on_device=True)
    dest = engine.alloc_outputs(T, opts=opts)
    dest.out.fill_(float("nan"))
    fitter.run_into_device(b.y, b.N, b.mm, opts, dest, chunks=engine.plan_chunks(T, opts, chunk_taxa=256))
    torch.cuda.current_stream().synchronize()
    assert np.array_equal(dest.status.cpu().numpy(), ref_st)
    assert np.array_equal(dest.out.cpu().numpy()[:, :32], ref_out[:, :32], equal_nan=True)
    assert np.array_equal(dest.pred.cpu().numpy(), ref_pred, equal_nan=True)
