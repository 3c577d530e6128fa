"""GPU tests of the MAP call's alternative paths, each against the default
call bit for bit:

  * no predictions (pred == NULL): the predictive HPDI then runs for z = +1
    only (the D_max_{lower,upper}_hpdi columns), in both lane layouts (the
    fused per-position step of the PPL-1 fit kernel, hpdi_prep_kernel after
    PPL 2);
  * the NULL (legacy default) HIP stream, and a call from another host thread
    (the record assembly forks onto the device's one side stream, the fork
    serialised by a mutex);
  * the call captured into a HIP graph and replayed;
  * garbage-filled workspace and outputs (MAP in both layouts, NUTS): every
    record column equal to a call on zeroed buffers;
  * the HPDI stream beside the fit, its defer path forced, and two calls on two
    streams at once beside unrelated kernels.
"""

from __future__ import annotations

import ctypes
import threading
import warnings

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return torch


def _call(lib, ty, tN, tm, T, opts, res, stream_handle):
    from metadamage_amd import _lib

    _lib.check(lib.mdfit_fit_batch(
        ctypes.c_void_p(ty.data_ptr()), ctypes.c_void_p(tN.data_ptr()), ctypes.c_void_p(tm.data_ptr()), T,
        ctypes.byref(opts), ctypes.c_void_p(res.out.data_ptr()),
        ctypes.c_void_p(res.pred.data_ptr()) if res.pred is not None else None,
        ctypes.c_void_p(res.status.data_ptr()), ctypes.c_void_p(res.workspace.data_ptr()), stream_handle))


@pytest.mark.parametrize("ppl", ["1", "2"])
def test_without_predictions_same_record(torch_dev, monkeypatch, ppl):
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    monkeypatch.setenv("MDFIT_FIT_PPL", ppl)
    b = generate(2_000, seed=21)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts()
    full = engine.fit_batch_device(ty, tN, tm, opts)
    bare = engine.fit_batch_device(ty, tN, tm, opts, engine.alloc_outputs(2_000, with_pred=False, opts=opts))
    torch.cuda.synchronize()
    a, c = full.out.cpu().numpy()[:, :25], bare.out.cpu().numpy()[:, :25]
    assert np.array_equal(a, c, equal_nan=True)  # the HPDI columns included
    assert np.isfinite(a[:, 2:4]).mean() > 0.99
    assert np.array_equal(full.status.cpu().numpy(), bare.status.cpu().numpy())


def test_null_stream_and_worker_thread(torch_dev):
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    T = 3_000
    b = generate(T, seed=22)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts()
    ref = engine.fit_batch_device(ty, tN, tm, opts)
    torch.cuda.synchronize()
    lib = _lib.load()
    outs = []
    # the NULL stream
    r0 = engine.alloc_outputs(T, opts=opts)
    _call(lib, ty, tN, tm, T, opts, r0, None)
    torch.cuda.synchronize()
    outs.append(r0)
    # another host thread, on a stream of its own

    def worker(box):
        try:
            s = torch.cuda.Stream()
            r = engine.alloc_outputs(T, opts=opts)
            torch.cuda.synchronize()
            _call(lib, ty, tN, tm, T, opts, r, ctypes.c_void_p(s.cuda_stream))
            s.synchronize()
            box.append(r)
        except Exception as e:  # reported in the main thread
            box.append(e)

    box: list = []
    th = threading.Thread(target=worker, args=(box,))
    th.start()
    th.join(timeout=120)
    assert box and not isinstance(box[0], Exception), box
    outs.append(box[0])
    for r in outs:
        assert np.array_equal(r.out.cpu().numpy()[:, :32], ref.out.cpu().numpy()[:, :32], equal_nan=True)
        assert np.array_equal(r.pred.cpu().numpy(), ref.pred.cpu().numpy(), equal_nan=True)
        assert np.array_equal(r.status.cpu().numpy(), ref.status.cpu().numpy())


def test_graph_capture_of_the_call(torch_dev):
    """The MAP call (with its side-stream fork / join) captured into a HIP graph
    on the caller's stream and replayed: the same record as a direct call."""
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    T = 2_000
    b = generate(T, seed=23)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts()
    ref = engine.fit_batch_device(ty, tN, tm, opts)
    torch.cuda.synchronize()
    lib = _lib.load()
    r = engine.alloc_outputs(T, opts=opts)
    s = torch.cuda.Stream()
    _call(lib, ty, tN, tm, T, opts, r, ctypes.c_void_p(s.cuda_stream))  # warm (side stream created)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        _call(lib, ty, tN, tm, T, opts, r, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    for _ in range(2):
        r.out.fill_(0.0)
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(r.out.cpu().numpy()[:, :32], ref.out.cpu().numpy()[:, :32], equal_nan=True)
        assert np.array_equal(r.pred.cpu().numpy(), ref.pred.cpu().numpy(), equal_nan=True)


@pytest.mark.parametrize("mode,ppl", [("map", "1"), ("map", "2"), ("nuts", "1")])
def test_dirty_workspace_and_outputs(torch_dev, monkeypatch, mode, ppl):
    """The library never assumes a clean workspace (torch.empty, reused across
    calls and sizes) or clean outputs: every counter, list and draw buffer it
    reads is written first in the call.  Garbage-filled workspace and outputs
    give the record of a call on zeroed ones, bit for bit."""
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    monkeypatch.setenv("MDFIT_FIT_PPL", ppl)
    T = 1_500 if mode == "map" else 96
    b = generate(T, seed=24)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts(mode=_lib.MODE_NUTS if mode == "nuts" else _lib.MODE_MAP)
    if mode == "nuts":
        opts.num_warmup, opts.num_samples = 60, 80
    lib = _lib.load()
    clean = engine.alloc_outputs(T, opts=opts)
    clean.workspace.zero_()
    clean.out.zero_()
    clean.pred.zero_()
    clean.status.zero_()
    _call(lib, ty, tN, tm, T, opts, clean, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    dirty = engine.alloc_outputs(T, opts=opts)
    g = torch.Generator(device="cpu").manual_seed(7)
    for _ in range(2):  # second round: the workspace as the first call left it, outputs re-dirtied
        dirty.out.copy_(torch.randn(dirty.out.shape, generator=g, dtype=dirty.out.dtype) * 1e30)
        dirty.pred.fill_(float("nan"))
        dirty.status.fill_(-7)
        if _ == 0:
            dirty.workspace.copy_(torch.randint(0, 256, dirty.workspace.shape, generator=g, dtype=torch.uint8))
        _call(lib, ty, tN, tm, T, opts, dirty, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        # every column of the record, the per-sub-fit diagnostics included
        assert np.array_equal(dirty.out.cpu().numpy(), clean.out.cpu().numpy(), equal_nan=True)
        assert np.array_equal(dirty.pred.cpu().numpy(), clean.pred.cpu().numpy(), equal_nan=True)
        assert np.array_equal(dirty.status.cpu().numpy(), clean.status.cpu().numpy())


@pytest.mark.parametrize("ppl", ["1", "2"])
def test_hpdi_stream_beside_the_fit_same_record(torch_dev, monkeypatch, ppl):
    """The predictive HPDI streamed beside the fit kernel (early launch on a
    side stream, waiting on the ready list) gives the record of the HPDI run
    after the fit (MDFIT_STREAM_WAVES_PER_CU=0), bit for bit, with and without
    predictions, and in both lane layouts."""
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    monkeypatch.setenv("MDFIT_FIT_PPL", ppl)
    b = generate(4_000, seed=23)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts()
    recs = []
    # "4d": the early waves defer every item they would wait on (MDFIT_STREAM_DEFER_US=0):
    # the late launch drains them from the defer list
    for early in ("0", "2", "4", "4d"):
        monkeypatch.setenv("MDFIT_STREAM_WAVES_PER_CU", early[0])
        monkeypatch.setenv("MDFIT_STREAM_DEFER_US", "0" if early == "4d" else "1000")
        for with_pred in (True, False):
            r = engine.fit_batch_device(ty, tN, tm, opts, engine.alloc_outputs(4_000, with_pred=with_pred, opts=opts))
            torch.cuda.synchronize()
            hdr = r.workspace[:256].view(torch.int32).cpu().numpy()
            assert hdr[8] == 4_000 and hdr[11] == 0  # one ready entry per taxon, no corrupt entry met
            n_def = hdr[32] & ~0x40000000
            if early != "0":
                assert hdr[32] & 0x40000000  # the late launch closed the defer list
                assert hdr[33] == n_def and hdr[34] >= n_def  # every reserved slot written, and drained
            if early == "4d":
                assert n_def > 0 and hdr[35] == 1
            recs.append((early, with_pred, r.out.cpu().numpy()[:, :32], None if r.pred is None else r.pred.cpu().numpy(),
                         r.status.cpu().numpy()))
    base = {wp: rec for e, wp, *rec in recs if e == "0"}
    for e, wp, out, pred, st in recs:
        o0, p0, s0 = base[wp]
        assert np.array_equal(out, o0, equal_nan=True), (e, wp)
        assert np.array_equal(st, s0), (e, wp)
        if wp:
            assert np.array_equal(pred, p0, equal_nan=True), (e, wp)
    assert np.isfinite(base[True][0][:, 2:4]).mean() > 0.99


def test_two_calls_on_two_streams_at_once(torch_dev):
    """Two MAP calls enqueued on two streams back to back, beside a third stream
    busy with unrelated kernels: the HPDI stream's early waves may then find
    their fit kernel short of slots, and must not wait on it indefinitely
    (bounded waits, the defer list).  Each call gives the record of
    the same call run alone, bit for bit."""
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    opts = _lib.default_opts()
    lib = _lib.load()
    cases = []
    for T, seed in ((6_000, 31), (20_000, 32)):  # both lane layouts
        b = generate(T, seed=seed)
        ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
        ref = engine.fit_batch_device(ty, tN, tm, opts)
        torch.cuda.synchronize()
        cases.append((T, ty, tN, tm, ref))
    a = torch.randn(4096, 4096, device="cuda")
    busy = torch.cuda.Stream()
    streams = [torch.cuda.Stream() for _ in cases]
    for rep in range(3):
        res = [engine.alloc_outputs(T, opts=opts) for T, *_ in cases]
        torch.cuda.synchronize()
        with torch.cuda.stream(busy):
            for _ in range(8):
                a = torch.tanh(a @ a * 1e-3)
        for (T, ty, tN, tm, _), r, s in zip(cases, res, streams):
            _call(lib, ty, tN, tm, T, opts, r, ctypes.c_void_p(s.cuda_stream))
        torch.cuda.synchronize()
        for (T, ty, tN, tm, ref), r in zip(cases, res):
            assert np.array_equal(r.out.cpu().numpy()[:, :32], ref.out.cpu().numpy()[:, :32], equal_nan=True), (rep, T)
            assert np.array_equal(r.pred.cpu().numpy(), ref.pred.cpu().numpy(), equal_nan=True), (rep, T)
            assert np.array_equal(r.status.cpu().numpy(), ref.status.cpu().numpy()), (rep, T)
            hdr = r.workspace[:256].view(torch.int32).cpu().numpy()
            assert hdr[8] == T and hdr[11] == 0


@pytest.mark.parametrize("mode,T", [("map", 1_500), ("map", 60_000), ("nuts", 96)])
def test_poisoned_lds_same_record(torch_dev, monkeypatch, mode, T):
    """No kernel of a call reads LDS it did not write: with every CU's LDS set to
    NaN before each LDS-using kernel (MDFIT_DEBUG_POISON_LDS, mdfit_poison_lds),
    the record, predictions and statuses are those of a call without -- the MAP
    streamed path, the MAP K4a / K4b path (from 60k taxa) and the sampler.  (Round
    4: the sampler's asymmetry read one unwritten LDS entry at weight 0, and a
    stale NaN there made the column NaN.)"""
    torch = torch_dev
    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(T, seed=26)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    opts = _lib.default_opts(mode=_lib.MODE_NUTS if mode == "nuts" else _lib.MODE_MAP)
    if mode == "nuts":
        opts.num_warmup, opts.num_samples = 60, 80
    recs = []
    for poison in ("0", "1"):
        monkeypatch.setenv("MDFIT_DEBUG_POISON_LDS", poison)
        r = engine.fit_batch_device(ty, tN, tm, opts)
        torch.cuda.synchronize()
        recs.append((r.out.cpu().numpy(), r.pred.cpu().numpy(), r.status.cpu().numpy()))
        if mode == "map" and T < 60_000 and int(r.workspace[48:52].view(torch.int32).item()) == 0:
            # (diagnostic only: whether the early HPDI launch claimed items before
            # the late one started is scheduling, not correctness -- it may not
            # run at all without a side fork)
            warnings.warn(f"poison={poison}: the early HPDI launch claimed no item in this call")
    for x, y in zip(*recs):
        assert np.array_equal(x, y, equal_nan=True)
    if mode == "nuts":  # (the columns test_c3_nuts_100k checks)
        assert np.isfinite(recs[1][0][recs[1][2] == 0][:, [0, 1, 4, 5, 6, 15, 18, 21]]).all()
