"""Device-side entry points: PyTorch-ROCm tensors in, C-ABI call, tensors out.

PyTorch only provides device memory and the stream; every computation runs in
the HIP kernels of libmdfit.so (metadamage_amd/csrc/mdfit.hip).  There is no
CPU fallback: without a GPU these functions raise.
"""

from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import _lib


def _torch():
    import torch

    if not torch.cuda.is_available():
        raise _lib.MdfitError("no HIP device available: the mdfit engine runs on MI355X only")
    return torch


def _stream_handle(torch, stream=None) -> ctypes.c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


@dataclass
class FitBatch:
    """Device-resident results of one mdfit_fit_batch call."""

    out: "object"  # torch.float64 [T, NOUT]
    pred: "object"  # torch.float32 [T, 3, 30]
    status: "object"  # torch.int32 [T]
    workspace: "object" = None  # torch.uint8 [mdfit_workspace_bytes(T, opts)] (work queues; NUTS: the draws)


def to_device_counts(y, N, mm=None, device="cuda"):
    """Host uint32 arrays -> device tensors in the engine's dense layout."""
    torch = _torch()
    y = np.ascontiguousarray(y, dtype=np.uint32)
    N = np.ascontiguousarray(N, dtype=np.uint32)
    if y.ndim != 2 or y.shape[1] != _lib.LD or N.shape != y.shape:
        raise ValueError(f"y, N must be uint32[T][{_lib.LD}], got {y.shape} / {N.shape}")
    ty = torch.from_numpy(y.view(np.int32)).to(device)
    tN = torch.from_numpy(N.view(np.int32)).to(device)
    tm = None
    if mm is not None:
        mm = np.ascontiguousarray(mm, dtype=np.uint32)
        if mm.shape != (y.shape[0], _lib.NPOS, _lib.NMM):
            raise ValueError(f"mm must be uint32[T][30][12], got {mm.shape}")
        tm = torch.from_numpy(mm.view(np.int32)).to(device)
    return ty, tN, tm


def alloc_outputs(n_taxa: int, device="cuda", with_pred: bool = True, opts: _lib.MdfitOpts | None = None) -> FitBatch:
    torch = _torch()
    out = torch.empty((n_taxa, _lib.NOUT), dtype=torch.float64, device=device)
    pred = (
        torch.empty((n_taxa, _lib.NPRED, _lib.NPOS), dtype=torch.float32, device=device)
        if with_pred
        else None
    )
    status = torch.empty((n_taxa,), dtype=torch.int32, device=device)
    return FitBatch(out, pred, status, alloc_workspace(n_taxa, device, opts))


def workspace_bytes(n_taxa: int, opts: _lib.MdfitOpts | None = None) -> int:
    lib = _lib.load()
    return int(lib.mdfit_workspace_bytes(int(n_taxa), ctypes.byref(opts) if opts is not None else None))


def alloc_workspace(n_taxa: int, device="cuda", opts: _lib.MdfitOpts | None = None):
    """Device scratch mdfit_fit_batch needs for n_taxa taxa under opts (work
    queues; in the sampling mode also every chain's draws)."""
    torch = _torch()
    return torch.empty((workspace_bytes(n_taxa, opts),), dtype=torch.uint8, device=device)


def samples_view(res: FitBatch, n_taxa: int, opts: _lib.MdfitOpts):
    """The sampling mode's draws in the workspace: float64 [T][6][S][4] = (q, A, c, phi)."""
    torch = _torch()
    S = int(opts.num_samples)
    n = n_taxa * 6 * S * 4
    return res.workspace[_lib.SAMPLES_OFFSET:_lib.SAMPLES_OFFSET + 8 * n].view(torch.float64).view(n_taxa, 6, S, 4)


def fit_batch_device(ty, tN, tm=None, opts: _lib.MdfitOpts | None = None, res: FitBatch | None = None,
                     stream=None) -> FitBatch:
    """Launch mdfit_fit_batch on device tensors (asynchronous on `stream`)."""
    torch = _torch()
    lib = _lib.load()
    T = int(ty.shape[0])
    for name, t in (("y", ty), ("N", tN)):
        if not (t.is_cuda and t.is_contiguous() and t.dtype == torch.int32 and tuple(t.shape) == (T, _lib.LD)):
            raise ValueError(f"{name} must be a contiguous cuda int32/uint32 view of shape [T, {_lib.LD}]")
    if tm is not None and not (tm.is_cuda and tm.is_contiguous() and tm.numel() == T * _lib.NPOS * _lib.NMM):
        raise ValueError("mm must be a contiguous cuda tensor of T*30*12 uint32")
    if res is None:
        res = alloc_outputs(T, device=ty.device, opts=opts)
    o = opts if opts is not None else _lib.default_opts()
    if res.workspace is None or res.workspace.numel() < workspace_bytes(T, o):
        res.workspace = alloc_workspace(T, ty.device, o)
    _lib.check(
        lib.mdfit_fit_batch(
            ctypes.c_void_p(ty.data_ptr()),
            ctypes.c_void_p(tN.data_ptr()),
            ctypes.c_void_p(tm.data_ptr()) if tm is not None else None,
            T,
            ctypes.byref(o),
            ctypes.c_void_p(res.out.data_ptr()),
            ctypes.c_void_p(res.pred.data_ptr()) if res.pred is not None else None,
            ctypes.c_void_p(res.status.data_ptr()),
            ctypes.c_void_p(res.workspace.data_ptr()),
            _stream_handle(torch, stream),
        )
    )
    return res


def fit_batch(y, N, mm=None, opts: _lib.MdfitOpts | None = None, device="cuda"):
    """Host arrays in, host arrays out: (out[T,80] f64, pred[T,3,30] f32, status[T] i32)."""
    torch = _torch()
    ty, tN, tm = to_device_counts(y, N, mm, device=device)
    res = fit_batch_device(ty, tN, tm, opts)
    torch.cuda.current_stream().synchronize()
    return res.out.cpu().numpy(), res.pred.cpu().numpy(), res.status.cpu().numpy()


# --------------------------------------------------------------------------
# bounded-memory chunked dispatch (the reference's 1,000-taxon chunks,
# fits.py:692-706, as device-memory-sized chunks on two streams)
# --------------------------------------------------------------------------
MAX_CALL_TAXA = 1 << 25  # mdfit_fit_batch's per-call limit (MAP: int32 position indices)
N_SETS = 2  # device buffer sets in flight: chunk k+1's H2D (and fit) beside chunk k's fit and D2H
_BUDGET_FRAC = 0.6  # default device budget of a staging: this fraction of the free device memory


def device_bytes(C: int, opts: _lib.MdfitOpts | None = None, with_mm: bool = True, with_pred: bool = True,
                 dest_on_device: bool = False) -> int:
    """Device bytes one buffer set of a C-taxon chunk takes: the inputs (y, N:
    256 B; mm: 1,440 B), the outputs (record 640 B, predictions 360 B, status 4
    B -- unless the chunk writes into the caller's device buffers) and the
    call's workspace (mdfit_workspace_bytes: MAP ~48 B below 60k taxa and
    ~4.9 KB from 60k, NUTS 6 x num_samples x 32 B, the draws)."""
    C = int(C)
    b = C * (2 * _lib.LD * 4 + (_lib.NPOS * _lib.NMM * 4 if with_mm else 0))
    if not dest_on_device:
        b += C * (_lib.NOUT * 8 + (_lib.NPRED * _lib.NPOS * 4 if with_pred else 0) + 4)
    return b + workspace_bytes(C, opts)


def plan_chunks(T: int, opts: _lib.MdfitOpts | None = None, budget_bytes: int | None = None, *,
                chunk_taxa: int = 0, n_sets: int = N_SETS, with_mm: bool = True, with_pred: bool = True,
                dest_on_device: bool = False) -> list[tuple[int, int]]:
    """Split T taxa into near-equal contiguous chunks [lo, hi) such that n_sets
    buffer sets of the largest chunk fit in budget_bytes (None: no memory
    bound), no chunk exceeds the per-call limit (2^25 taxa) or chunk_taxa (> 0;
    env MDFIT_CHUNK_TAXA when 0).  Taxa are independent and the sampler's
    streams are keyed by the global taxon index (opts.index_base + lo), so any
    split gives the records of one call bit for bit."""
    T = int(T)
    if T <= 0:
        return []
    cap = min(T, MAX_CALL_TAXA)
    if chunk_taxa <= 0:
        chunk_taxa = int(os.environ.get("MDFIT_CHUNK_TAXA", "0") or 0)
    if chunk_taxa > 0:
        cap = min(cap, int(chunk_taxa))
    if budget_bytes is not None:
        per = lambda c: n_sets * device_bytes(c, opts, with_mm, with_pred, dest_on_device)  # noqa: E731
        if per(1) > budget_bytes:
            raise _lib.MdfitError(f"device budget {budget_bytes} B below one taxon's {per(1)} B")
        if per(cap) > budget_bytes:  # largest c with per(c) <= budget (per is monotone in c)
            lo, hi = 1, cap
            while lo < hi:
                mid = (lo + hi + 1) // 2
                if per(mid) <= budget_bytes:
                    lo = mid
                else:
                    hi = mid - 1
            cap = lo
    n = -(-T // cap)
    return [(T * i // n, T * (i + 1) // n) for i in range(n)]


def default_budget(device) -> int:
    """The device budget of a staging (bytes): MDFIT_DEVICE_BUDGET_GB, else
    _BUDGET_FRAC of the device memory free now."""
    torch = _torch()
    env = os.environ.get("MDFIT_DEVICE_BUDGET_GB")
    if env:
        return int(float(env) * (1 << 30))
    free, _total = torch.cuda.mem_get_info(torch.device(device))
    return int(_BUDGET_FRAC * free)


class _Set:
    """One chunk's device buffers (the workspace is the fitter's: the calls
    run one after another on the compute stream)."""

    def __init__(self, torch, C: int, device, with_pred: bool, with_mm: bool, dest_on_device: bool):
        self.d_y = torch.empty((C, _lib.LD), dtype=torch.int32, device=device)
        self.d_N = torch.empty((C, _lib.LD), dtype=torch.int32, device=device)
        self.d_mm = torch.empty((C, _lib.NPOS, _lib.NMM), dtype=torch.int32, device=device) if with_mm else None
        self.out = self.pred = self.status = None
        if not dest_on_device:
            self.out = torch.empty((C, _lib.NOUT), dtype=torch.float64, device=device)
            self.pred = (torch.empty((C, _lib.NPRED, _lib.NPOS), dtype=torch.float32, device=device)
                         if with_pred else None)
            self.status = torch.empty((C,), dtype=torch.int32, device=device)


H_OUT_COLS = _lib.NRESULT  # record columns the host gets back: the 25 result columns


class ChunkedFitter:
    """Host-to-device fits of any number of taxa in chunks of at most
    `chunk_cap` taxa (the reference handles any number of taxa in 1,000-taxon
    chunks, fits.py:692-706; one call per file had a capacity cliff: the NUTS
    draws are 192 KB per taxon, ~1.4M taxa per GPU).  Device memory is
    N_SETS x device_bytes(chunk_cap) whatever the batch size.

    Two streams: the caller's current stream runs the calls, one after another
    (mdfit_fit_batch with mm = NULL, then mdfit_noise once the chunk's mismatch
    counts are on the device); a copy stream runs every transfer.  So the fit
    starts as soon as its y, N (256 B per taxon) are in, the mismatch counts
    (1,440 B per taxon) cross PCIe while it runs, and -- with several chunks --
    chunk k's results come back while chunk k+1 fits (N_SETS buffer sets).  The
    transfers of one chunk are ordered y, N before mm so the fit's inputs are
    not behind the bulk.  (Two streams of ours beside the library's two side
    streams: four hardware queues, GPU_MAX_HW_QUEUES on the box; more streams
    would share queues and serialise.)

    Outputs go to pinned host buffers (run: the 25 result columns, the
    predictions, the status; grown as needed and reused) or, run_into_device,
    straight into the caller's device tensors (the sharded fit's gather
    records)."""

    def __init__(self, chunk_cap: int, device="cuda", opts: _lib.MdfitOpts | None = None, with_pred: bool = True,
                 with_mm: bool = True, dest_on_device: bool = False):
        torch = _torch()
        self.chunk_cap = int(chunk_cap)
        self.device = torch.device(device)
        self.with_pred, self.with_mm, self.dest_on_device = with_pred, with_mm, dest_on_device
        self.sets = [_Set(torch, self.chunk_cap, self.device, with_pred, with_mm, dest_on_device)
                     for _ in range(N_SETS)]
        self.ws = alloc_workspace(self.chunk_cap, self.device, opts)
        self.copy = torch.cuda.Stream(device=self.device)
        self.full_cap = False  # (staging: the chunk capacity is the device budget's, not the batch's)
        self.capacity = 0  # pinned host buffers (input staging for pageable sources, outputs)
        self.h_y = self.h_N = self.h_mm = self.h_out = self.h_pred = self.h_status = None
        self._end = None  # the previous run's last event (its transfers use the pinned buffers)

    def _host(self, T: int):
        if T <= self.capacity:
            return
        torch = _torch()
        cap = int(1.25 * T) + 1
        self.h_y = torch.empty((cap, _lib.LD), dtype=torch.int32).pin_memory()
        self.h_N = torch.empty((cap, _lib.LD), dtype=torch.int32).pin_memory()
        self.h_mm = torch.empty((cap, _lib.NPOS, _lib.NMM), dtype=torch.int32).pin_memory() if self.with_mm else None
        if not self.dest_on_device:
            self.h_out = torch.empty((cap, H_OUT_COLS), dtype=torch.float64).pin_memory()
            self.h_pred = (torch.empty((cap, _lib.NPRED, _lib.NPOS), dtype=torch.float32).pin_memory()
                           if self.with_pred else None)
            self.h_status = torch.empty((cap,), dtype=torch.int32).pin_memory()
        self.capacity = cap

    def _sources(self, y, N, mm, pinned):
        """Pinned int32 views of the inputs: the PinnedPack's, or a copy into
        the staging's own pinned buffers (H2D from pageable memory would be a
        synchronous staged copy)."""
        T = int(y.shape[0])
        use_mm = mm is not None and self.with_mm
        if pinned is not None:
            return pinned.h_y[:T], pinned.h_N[:T], pinned.h_mm[:T] if use_mm else None
        if self._end is not None:  # the previous run's H2D may still read the staging buffers
            self._end.synchronize()
        self._host(T)
        self.h_y[:T].numpy()[:] = np.asarray(y, dtype=np.uint32).view(np.int32)
        self.h_N[:T].numpy()[:] = np.asarray(N, dtype=np.uint32).view(np.int32)
        if use_mm:
            self.h_mm[:T].numpy()[:] = np.asarray(mm, dtype=np.uint32).view(np.int32)
        return self.h_y[:T], self.h_N[:T], self.h_mm[:T] if use_mm else None

    def _launch(self, chunks, src, opts, dest=None):
        """Enqueue every chunk (asynchronous); returns the event after which
        every result is in place (host outputs: copied back)."""
        torch = _torch()
        lib = _lib.load()
        o0 = opts if opts is not None else _lib.default_opts()
        src_y, src_N, src_mm = src
        comp = torch.cuda.current_stream(self.device)
        cp = self.copy
        h_s = _stream_handle(torch, comp)
        start = torch.cuda.Event()
        start.record(comp)  # after the caller's prior work (and the previous run's)
        cp.wait_event(start)
        last_d2h = None
        done = []  # per chunk: its call (and noise) finished on the compute stream
        for k, (lo, hi) in enumerate(chunks):
            st = self.sets[k % N_SETS]
            n = hi - lo
            o = _lib.MdfitOpts.from_buffer_copy(o0)
            o.index_base = o0.index_base + lo  # the sampler's streams: global taxon index
            # transfers in: y, N first, then the mismatch counts (copy stream),
            # once the set's previous chunk has finished reading them
            if k >= N_SETS:
                cp.wait_event(done[k - N_SETS])
            with torch.cuda.stream(cp):
                st.d_y[:n].copy_(src_y[lo:hi], non_blocking=True)
                st.d_N[:n].copy_(src_N[lo:hi], non_blocking=True)
                ev_yn = torch.cuda.Event()
                ev_yn.record(cp)
                ev_mm = None
                if src_mm is not None:
                    st.d_mm[:n].copy_(src_mm[lo:hi], non_blocking=True)
                    ev_mm = torch.cuda.Event()
                    ev_mm.record(cp)
            if dest is not None:
                res = FitBatch(dest.out[lo:hi], dest.pred[lo:hi] if dest.pred is not None else None,
                               dest.status[lo:hi], self.ws)
            else:
                res = FitBatch(st.out[:n], st.pred[:n] if st.pred is not None else None, st.status[:n], self.ws)
            # the call (compute stream) once y, N are in; the noise once mm is
            comp.wait_event(ev_yn)
            fit_batch_device(st.d_y[:n], st.d_N[:n], None, o, res, stream=comp)
            self.ws = res.workspace
            if ev_mm is not None:
                comp.wait_event(ev_mm)
                _lib.check(lib.mdfit_noise(ctypes.c_void_p(st.d_y.data_ptr()), ctypes.c_void_p(st.d_N.data_ptr()),
                                           ctypes.c_void_p(st.d_mm.data_ptr()), n, ctypes.c_void_p(res.out.data_ptr()),
                                           h_s))
            ev_done = torch.cuda.Event()
            ev_done.record(comp)
            done.append(ev_done)
            if dest is None:  # results out on the copy stream, behind this chunk's call
                cp.wait_event(ev_done)
                with torch.cuda.stream(cp):
                    self.h_out[lo:hi].copy_(res.out[:, :H_OUT_COLS], non_blocking=True)
                    if res.pred is not None:
                        self.h_pred[lo:hi].copy_(res.pred, non_blocking=True)
                    self.h_status[lo:hi].copy_(res.status, non_blocking=True)
                last_d2h = cp
        end = torch.cuda.Event()
        end.record(cp if last_d2h is not None else comp)
        self._end = end
        return end

    def run(self, y, N, mm=None, opts: _lib.MdfitOpts | None = None, sync: bool = True,
            pinned: PinnedPack | None = None, chunks=None):
        """Fit len(y) taxa; returns numpy views (out[:, :25], pred, status) of the
        pinned buffers (valid until the next run).  pinned: y, N, mm are that
        PinnedPack's views.  chunks: the split (default plan_chunks at this
        staging's chunk_cap)."""
        T = int(y.shape[0])
        if chunks is None:
            chunks = plan_chunks(T, opts, chunk_taxa=self.chunk_cap)
        if chunks and max(hi - lo for lo, hi in chunks) > self.chunk_cap:
            raise ValueError(f"a chunk exceeds this staging's {self.chunk_cap} taxa")
        self._host(T)
        end = self._launch(chunks, self._sources(y, N, mm, pinned), opts)
        if sync:
            end.synchronize()
        pred = self.h_pred[:T].numpy() if self.h_pred is not None else None
        return self.h_out[:T].numpy(), pred, self.h_status[:T].numpy()

    def run_into_device(self, y, N, mm, opts, dest: FitBatch, chunks=None):
        """Fit len(y) taxa chunk by chunk into the caller's device tensors dest
        (out[T, NOUT], pred, status: rows written in place), ordered on the
        caller's current stream."""
        T = int(y.shape[0])
        if chunks is None:
            chunks = plan_chunks(T, opts, chunk_taxa=self.chunk_cap)
        self._launch(chunks, self._sources(y, N, mm, None), opts, dest=dest)
        return dest


class PinnedPack:
    """A pinned host buffer set for one file's packed counts (y, N: uint32
    [cap][32], mm: uint32[cap][30][12]): fits.pack_counts writes into it on a
    reader thread and ChunkedFitter.run copies it to the device directly (no
    host copy into the staging buffers: ~170 MB per 100k-taxon file)."""

    def __init__(self, capacity: int):
        torch = _torch()
        self.capacity = int(capacity)
        T = self.capacity
        self.h_y = torch.empty((T, _lib.LD), dtype=torch.int32).pin_memory()
        self.h_N = torch.empty((T, _lib.LD), dtype=torch.int32).pin_memory()
        self.h_mm = torch.empty((T, _lib.NPOS, _lib.NMM), dtype=torch.int32).pin_memory()

    def views(self, T: int):
        """numpy uint32 views (y, N, mm) of the first T taxa."""
        return (self.h_y[:T].numpy().view(np.uint32), self.h_N[:T].numpy().view(np.uint32),
                self.h_mm[:T].numpy().view(np.uint32))


_PINNED_FREE: list = []
_PINNED_N = 0
_PINNED_MAX = 3  # files in flight in main.main: N_READERS ahead + the one being fitted
_PINNED_LOCK = __import__("threading").Lock()


def acquire_pinned_pack(T: int) -> PinnedPack | None:
    """A free PinnedPack of at least T taxa (x1.25 headroom when one is made),
    or None when every set is in use (the caller then packs into pageable
    memory) or no HIP device is visible."""
    import torch

    if not torch.cuda.is_available():
        return None
    global _PINNED_N
    with _PINNED_LOCK:
        for i, pp in enumerate(_PINNED_FREE):
            if pp.capacity >= T:
                return _PINNED_FREE.pop(i)
        if _PINNED_FREE:  # too small: replaced by a larger one
            _PINNED_FREE.pop(0)
            _PINNED_N -= 1
        if _PINNED_N >= _PINNED_MAX:
            return None
        _PINNED_N += 1
    return PinnedPack(int(1.25 * T) + 1)


def release_pinned_pack(pp: PinnedPack) -> None:
    with _PINNED_LOCK:
        _PINNED_FREE.append(pp)


_STAGING: dict = {}
_STAGING_LOCK = __import__("threading").Lock()


def staging(n_taxa: int, device="cuda", opts: _lib.MdfitOpts | None = None, with_mm: bool = True,
            dest_on_device: bool = False, budget_bytes: int | None = None) -> ChunkedFitter:
    """The ChunkedFitter for batches of n_taxa on this device, reused across calls
    of this process (per device, buffer kind and sampler length): the
    multi-file pipeline fits one file after another, and pinned + device
    buffers allocated per file cost more host time than the fit.  Its chunk
    capacity is the largest chunk N_SETS buffer sets of which fit the device
    budget (default_budget), or n_taxa (x1.25 headroom) when smaller; a larger
    batch than the chunk capacity is split into chunks (plan_chunks), so the
    device memory it takes is bounded whatever the batch size.  Callers hold
    _STAGING_LOCK around its use (concurrent host threads take turns)."""
    torch = _torch()
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device(dev.type, torch.cuda.current_device())
    o = opts if opts is not None else _lib.default_opts()
    env_chunk = int(os.environ.get("MDFIT_CHUNK_TAXA", "0") or 0)
    key = (str(dev), bool(with_mm), bool(dest_on_device), int(o.mode), int(o.num_samples), env_chunk)
    st = _STAGING.get(key)
    T = max(1, int(n_taxa))
    if st is not None and (st.chunk_cap >= T or st.full_cap):
        return st
    _STAGING.pop(key, None)
    del st
    budget = budget_bytes if budget_bytes is not None else default_budget(dev)
    # the largest chunk the budget allows (x1.25 headroom over this batch: the
    # files of a run differ in taxon count by a few %)
    want = int(1.25 * T) + 1
    # (not across the library's stream / after-the-fit HPDI switch: from 60k
    # taxa the MAP workspace holds every position's wide-window record, ~4.8 KB
    # per taxon that batches below 60k never touch)
    if T < _lib.STREAM_MAX_TAXA:
        want = min(want, _lib.STREAM_MAX_TAXA - 1)
    cap = plan_chunks(want, o, budget, chunk_taxa=env_chunk, with_mm=with_mm, dest_on_device=dest_on_device)[0]
    cap = cap[1] - cap[0]
    st = ChunkedFitter(cap, device=dev, opts=o, with_mm=with_mm, dest_on_device=dest_on_device)
    # (chunk capacity below the batch: memory-bound, no regrow for larger batches)
    st.full_cap = cap < want
    _STAGING[key] = st
    return st


def fit_batch_host(y, N, mm=None, opts: _lib.MdfitOpts | None = None, noise=None, device="cuda",
                   pinned: PinnedPack | None = None):
    """The product's host-to-host fit: (out[T, 25], pred, status), chunked
    through the device budget (ChunkedFitter).  mm goes to the device (the
    assembly computes the noise columns); without it, `noise` (float64[T][3],
    ingest.noise) fills them when given.  pinned: y, N, mm are views of that
    PinnedPack (copied to the device from there)."""
    T = int(y.shape[0])
    with _STAGING_LOCK:
        st = staging(T, device=device, opts=opts, with_mm=mm is not None)
        out, pred, status = st.run(y, N, mm, opts, pinned=pinned, chunks=plan_chunks(T, opts, chunk_taxa=st.chunk_cap))
        out, pred, status = out.copy(), pred.copy(), status.copy()
    if mm is None and noise is not None:
        ok = status != _lib.INVALID
        out[ok, _lib.RESULT_FIELDS.index("normalized_noise"):_lib.NRESULT] = np.asarray(noise)[ok]
    return out, pred, status


def special(x, device="cuda"):
    """(lgamma, digamma, trigamma) of x on the device (parity tests)."""
    torch = _torch()
    lib = _lib.load()
    tx = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=device)
    o = torch.empty((tx.numel(), 3), dtype=torch.float64, device=device)
    _lib.check(lib.mdfit_special(ctypes.c_void_p(tx.data_ptr()), tx.numel(), ctypes.c_void_p(o.data_ptr()),
                                 _stream_handle(torch)))
    torch.cuda.current_stream().synchronize()
    return o.cpu().numpy()


def betabinom_logpmf(y, N, a, b, device="cuda"):
    """Pointwise beta-binomial log-pmf and (d/dalpha, d/dbeta) on the device."""
    torch = _torch()
    lib = _lib.load()
    ts = [torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64), device=device) for v in (y, N, a, b)]
    n = ts[0].numel()
    o = torch.empty(n, dtype=torch.float64, device=device)
    g = torch.empty((n, 2), dtype=torch.float64, device=device)
    _lib.check(lib.mdfit_betabinom_logpmf(*[ctypes.c_void_p(t.data_ptr()) for t in ts], n,
                                          ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(g.data_ptr()),
                                          _stream_handle(torch)))
    torch.cuda.current_stream().synchronize()
    return o.cpu().numpy(), g.cpu().numpy()


def hpdi68(N, a, b, device="cuda"):
    """68 % predictive window [lo, hi] of BetaBinomial(a, b, N) on the device
    (MDFIT-HPDI v2, mdfit_hpdi68; parity tests)."""
    torch = _torch()
    lib = _lib.load()
    shape = np.broadcast(N, a, b).shape
    # np.array copies: a broadcast view is read-only (torch warns on those)
    ts = [torch.as_tensor(np.array(np.broadcast_to(v, shape), dtype=np.float64).ravel(), device=device)
          for v in (N, a, b)]
    n = ts[0].numel()
    lo = torch.empty(n, dtype=torch.float64, device=device)
    hi = torch.empty(n, dtype=torch.float64, device=device)
    _lib.check(lib.mdfit_hpdi68(*[ctypes.c_void_p(t.data_ptr()) for t in ts], n, ctypes.c_void_p(lo.data_ptr()),
                                ctypes.c_void_p(hi.data_ptr()), _stream_handle(torch)))
    torch.cuda.current_stream().synchronize()
    return lo.cpu().numpy(), hi.cpu().numpy()


def peak_probe(n_waves: int, iters: int, stream=None, nuts: bool = False):
    """Launch the register-only point-evaluation probe (MAP: value + gradient +
    Hessian; nuts: the sampler's potential, value + gradient); returns the sink
    tensor."""
    torch = _torch()
    lib = _lib.load()
    sink = torch.empty(n_waves * 64, dtype=torch.float64, device="cuda")
    fn = lib.mdfit_nuts_peak_probe if nuts else lib.mdfit_peak_probe
    _lib.check(fn(n_waves, iters, ctypes.c_void_p(sink.data_ptr()), _stream_handle(torch, stream)))
    return sink


def nuts_potential(model, subset, y, N, v, device="cuda"):
    """Sampling-mode potential and gradient per item (mdfit_nuts_potential)."""
    torch = _torch()
    lib = _lib.load()
    n = len(model)
    tm = torch.as_tensor(np.ascontiguousarray(model, dtype=np.int32), device=device)
    ts = torch.as_tensor(np.ascontiguousarray(subset, dtype=np.int32), device=device)
    ty = torch.from_numpy(np.ascontiguousarray(y, dtype=np.uint32).view(np.int32)).to(device)
    tN = torch.from_numpy(np.ascontiguousarray(N, dtype=np.uint32).view(np.int32)).to(device)
    tv = torch.as_tensor(np.ascontiguousarray(v, dtype=np.float64), device=device)
    U = torch.empty(n, dtype=torch.float64, device=device)
    g = torch.empty((n, 4), dtype=torch.float64, device=device)
    _lib.check(lib.mdfit_nuts_potential(*(ctypes.c_void_p(t.data_ptr()) for t in (tm, ts, ty, tN, tv)), n,
                                        ctypes.c_void_p(U.data_ptr()), ctypes.c_void_p(g.data_ptr()),
                                        _stream_handle(torch)))
    torch.cuda.synchronize()
    return U.cpu().numpy(), g.cpu().numpy()


def profile_enable(on: bool = True, fit_only: bool = False) -> None:
    """Record HIP events around every following mdfit_fit_batch call (and its
    fit kernel) on the call's stream; fit_only: only the two around the fit
    kernel (profile_read's call time is then -1)."""
    _lib.check(_lib.load().mdfit_profile_enable((2 if fit_only else 1) if on else 0))


def profile_read():
    """(call_ms_sum, fit_kernel_ms_sum, n_calls) over the calls recorded since
    profile_enable / the last read (synchronises on the events)."""
    a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
    _lib.check(_lib.load().mdfit_profile_read(ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)))
    return a.value, b.value, n.value


def objective(model, subset, y, N, u, device="cuda"):
    """Per-item sub-fit objective (F, g[4], H[4,4], ell[30]) evaluated by the
    fit kernel's code path (mdfit_objective)."""
    torch = _torch()
    lib = _lib.load()
    n = len(model)
    tm = torch.as_tensor(np.ascontiguousarray(model, dtype=np.int32), device=device)
    ts = torch.as_tensor(np.ascontiguousarray(subset, dtype=np.int32), device=device)
    ty = torch.from_numpy(np.ascontiguousarray(y, dtype=np.uint32).view(np.int32)).to(device)
    tN = torch.from_numpy(np.ascontiguousarray(N, dtype=np.uint32).view(np.int32)).to(device)
    tu = torch.as_tensor(np.ascontiguousarray(u, dtype=np.float64), device=device)
    F = torch.empty(n, dtype=torch.float64, device=device)
    g = torch.empty((n, 4), dtype=torch.float64, device=device)
    H = torch.empty((n, 4, 4), dtype=torch.float64, device=device)
    ell = torch.empty((n, 30), dtype=torch.float64, device=device)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    _lib.check(lib.mdfit_objective(ptr(tm), ptr(ts), ptr(ty), ptr(tN), ptr(tu), n, ptr(F), ptr(g), ptr(H),
                                   ptr(ell), _stream_handle(torch)))
    torch.cuda.current_stream().synchronize()
    return F.cpu().numpy(), g.cpu().numpy(), H.cpu().numpy(), ell.cpu().numpy()
