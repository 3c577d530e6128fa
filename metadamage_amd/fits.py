"""The drop-in fit boundary: get_fits / compute_fits over the HIP engine.

Mirrors /root/reference/metadamage/fits.py at its operator boundary:

  get_fits(df_counts, cfg)        fits.py:754-807  (cache check, top-N, fit, save)
  get_top_max_fits                fits.py:736-751
  compute_fits(df_counts, cfg)    fits.py:709-730  -> ONE batched device call
  make_df_fit_results_*           fits.py:668-680
  make_df_fit_predictions_*       fits.py:632-665

What changes is the body of compute_fits: instead of a process pool running
numpyro NUTS per taxon (fits.py:477-626), the counts table is packed once into
the dense layout of include/mdfit.h (the batched group_to_numpyro_data,
fits.py:398-419) and fitted by mdfit_fit_batch on the GPU(s); taxa the engine
flags (status != 0) are dropped with a warning, like the reference drops taxa
whose fit timed out (fits.py:520-522, 603-606).
"""

from __future__ import annotations

import logging

import numpy as np
import pandas as pd

from . import _lib, io, utils

logger = logging.getLogger(__name__)

MM_COLUMNS = ["AC", "AG", "AT", "CA", "CG", "CT", "GA", "GC", "GT", "TA", "TC", "TG"]
POSITIONS = np.concatenate([np.arange(1, 16), -np.arange(1, 16)])

# fit_results column order (fits.py:244-293, 317-356, 374-376 + :671)
FIT_RESULT_COLUMNS = (
    ["tax_id", "tax_name", "tax_rank"]
    + _lib.RESULT_FIELDS[:7]
    + ["N_alignments"]
    + _lib.RESULT_FIELDS[7:]
    + ["shortname"]
)
INT_RESULT_FIELDS = {"N_alignments", "N_z1_forward", "N_z1_reverse", "N_sum_forward", "N_sum_reverse",
                     "N_sum_total", "y_sum_forward", "y_sum_reverse", "y_sum_total"}


# --------------------------------------------------------------------------
# packing: df_counts -> dense [T][32] tensors (batched group_to_numpyro_data)
# --------------------------------------------------------------------------
class Packed:
    def __init__(self, tax_id, tax_name, tax_rank, N_alignments, y, N, mm, cats=None, pinned=None):
        self.tax_id = tax_id
        self.tax_name = tax_name
        self.tax_rank = tax_rank
        self.N_alignments = N_alignments
        self.y = y
        self.N = N
        self.mm = mm
        # per-taxon pd.Categorical of tax_id / tax_name / tax_rank when df_counts
        # had them (sorted categories): the frames reuse their order instead of
        # re-sorting a million names
        self.cats = cats or {}
        # the engine.PinnedPack y / N / mm live in (main.main's pipeline), handed
        # back to its pool once the device has them (release_pinned)
        self.pinned = pinned

    def release_pinned(self):
        """Return the pinned buffer set; y / N / mm are gone afterwards."""
        if self.pinned is not None:
            from . import engine

            engine.release_pinned_pack(self.pinned)
            self.pinned = None
            self.y = self.N = self.mm = None

    @property
    def n_taxa(self):
        return len(self.tax_id)


def _as_u32(a: np.ndarray) -> np.ndarray:
    """uint32 view/copy of a count column, with utils.py:338-339's range check."""
    if a.dtype == np.uint32:
        return a
    if a.size and (int(a.max()) > np.iinfo(np.uint32).max or int(a.min()) < 0):
        raise AssertionError("Dataframe contains too large values.")
    return a.astype(np.uint32)


def _interleave(cols, out2d: np.ndarray) -> None:
    """out2d[:, j] = cols[j], natively over row ranges (ingest.interleave:
    numpy's strided column writes take ~0.09 s of the GIL-holding main
    thread on a 2.8 M x 12 table)."""
    from . import ingest

    ingest.interleave(cols, out2d)


def _first_values(s: pd.Series, first: np.ndarray) -> np.ndarray:
    """s.to_numpy()[first] without materialising a categorical column."""
    return np.asarray(s.array[first]) if isinstance(s.dtype, pd.CategoricalDtype) else s.to_numpy()[first]


def _first_categoricals(df: pd.DataFrame, first: np.ndarray) -> dict:
    out = {}
    for c in ("tax_id", "tax_name", "tax_rank"):
        col = df[c]
        if isinstance(col.dtype, pd.CategoricalDtype) and col.cat.categories.is_monotonic_increasing:
            out[c] = col.array[first]
    return out


def pack_counts(df: pd.DataFrame, cfg, pinned: bool = False) -> Packed:
    """Dense y/N (uint32[T][32]) and mismatch counts (uint32[T][30][12]) in
    df order (first appearance of each tax_id, i.e. the N_alignments-desc
    order of sort_by_alignments).  Column i < 15 holds z = i+1 (y = the
    forward substitution, N = its reference-base sum), i >= 15 holds
    z = -(i-14) (reverse substitution) — group_to_numpyro_data, fits.py:398-419.
    Rows are placed by their position value, so missing positions read as
    N = 0 (no information) instead of shifting the others.  The usual table
    (every taxon with its 30 rows in sort_by_alignments order) is packed by
    reshaping; anything else is scattered row by row."""
    fwd, rev = cfg.substitution_bases_forward, cfg.substitution_bases_reverse
    tax = df["tax_id"]
    # rows without a tax_id belong to no taxon: the reference's
    # groupby("tax_id", observed=True) drops missing keys (fits.py:736-744,
    # 398-419), so they are dropped here before any index is formed (a -1
    # index would scatter them onto the last taxon's row)
    missing = tax.isna().to_numpy()
    if missing.any():
        df = df[~missing]
        tax = df["tax_id"]
    codes = tax.cat.codes.to_numpy() if isinstance(tax.dtype, pd.CategoricalDtype) else None

    def packed(first, y, N, mm, pp):
        return Packed(
            tax_id=_first_values(tax, first),
            tax_name=_first_values(df["tax_name"], first),
            tax_rank=_first_values(df["tax_rank"], first),
            N_alignments=df["N_alignments"].to_numpy()[first].astype(np.int64),
            y=y,
            N=N,
            mm=mm,
            cats=_first_categoricals(df, first),
            pinned=pp,
        )

    # the usual table (counts.compute_counts: 30 rows per taxon in z order,
    # uint32 counts): one native pass writes y, N and mm and checks the layout
    pos = df["position"].to_numpy()
    n = len(tax)
    if codes is not None and n and n % _lib.NPOS == 0 and pos.dtype == np.int8 and len(tax.cat.categories) < 2**31:
        cols = [df[c].to_numpy() for c in (*MM_COLUMNS, fwd, rev, fwd[0], rev[0])]
        if all(c.dtype == np.uint32 for c in cols):
            from . import ingest

            T = n // _lib.NPOS
            y, N, mm, pp = _pack_buffers(T, pinned, zero=False)
            T = ingest.pack_dense(np.ascontiguousarray(codes, dtype=np.int32), len(tax.cat.categories), pos,
                                  [np.ascontiguousarray(c) for c in cols], y, N, mm)
            if T >= 0:
                return packed(np.arange(T, dtype=np.int64) * _lib.NPOS, y, N, mm, pp)
            if pp is not None:
                from . import engine

                engine.release_pinned_pack(pp)
    # taxon index in first-appearance order (pd.factorize) and each taxon's first row
    if codes is not None and len(tax.cat.categories) < 2**31:
        from . import ingest

        t, first = ingest.first_index(codes, len(tax.cat.categories))
    else:
        t, _ = pd.factorize(tax.to_numpy())
        t = t.astype(np.int64)
        first = np.flatnonzero(np.r_[True, t[1:] > np.maximum.accumulate(t[:-1])]) if t.size else np.zeros(0, np.int64)
    n = t.size
    T = first.size
    pos_fwd = pos > 0
    yv = _as_u32(np.where(pos_fwd, df[fwd].to_numpy(), df[rev].to_numpy()))
    Nv = _as_u32(np.where(pos_fwd, df[fwd[0]].to_numpy(), df[rev[0]].to_numpy()))
    mm_cols = [_as_u32(df[c].to_numpy()) for c in MM_COLUMNS]
    dense = n == T * _lib.NPOS and np.array_equal(
        pos.reshape(T, _lib.NPOS), np.broadcast_to(POSITIONS.astype(pos.dtype), (T, _lib.NPOS))) and np.array_equal(
        t.reshape(T, _lib.NPOS), np.broadcast_to(np.arange(T)[:, None], (T, _lib.NPOS)))
    y, N, mm, pp = _pack_buffers(T, pinned, zero=True)
    if dense:
        y[:, :_lib.NPOS] = yv.reshape(T, _lib.NPOS)
        N[:, :_lib.NPOS] = Nv.reshape(T, _lib.NPOS)
        _interleave(mm_cols, mm.reshape(-1, _lib.NMM))
    else:
        p64 = pos.astype(np.int64)
        col = np.where(p64 > 0, p64 - 1, 14 - p64)
        ok = (p64 != 0) & (np.abs(p64) <= 15)
        if not ok.all():
            logger.warning(f"{int((~ok).sum())} rows with |position| outside 1..15 ignored")
        y[t[ok], col[ok]] = yv[ok]
        N[t[ok], col[ok]] = Nv[ok]
        mm.fill(0)
        rows = np.empty((n, _lib.NMM), np.uint32)
        _interleave(mm_cols, rows)
        mm.reshape(-1, _lib.NMM)[(t * _lib.NPOS + col)[ok]] = rows[ok]
    return packed(first, y, N, mm, pp)


def _pack_buffers(T: int, pinned: bool, zero: bool):
    """y, N (uint32[T][LD]) and mm (uint32[T][30][12]) for pack_counts, in a
    pinned buffer set when pinned (main.main's reader threads: the device copy
    reads them directly); zero: y and N zero-filled."""
    pp = None
    if pinned and T > 0:
        from . import engine

        pp = engine.acquire_pinned_pack(T)
    if pp is not None:
        y, N, mm = pp.views(T)
        if zero:
            y.fill(0)
            N.fill(0)
    else:
        alloc = np.zeros if zero else np.empty
        y = alloc((T, _lib.LD), np.uint32)
        N = alloc((T, _lib.LD), np.uint32)
        mm = np.empty((T, _lib.NPOS, _lib.NMM), np.uint32)
    return y, N, mm, pp


# --------------------------------------------------------------------------
# the device call (single GPU or sharded over torch.distributed ranks)
# --------------------------------------------------------------------------
def fit_packed(p: Packed, opts=None, shard: bool = True):
    """Run mdfit_fit_batch on the packed taxa; returns host (out, pred, status)
    on rank 0 (None elsewhere in a multi-GPU job).  shard=False fits every
    taxon on this rank's GPU (main() shards whole files across ranks)."""
    import torch

    from . import engine

    if not torch.cuda.is_available():
        raise _lib.MdfitError("metadamage_amd fits run on MI355X GPUs only (no HIP device visible)")
    import torch.distributed as dist

    # the sharded branch whenever a process group is up (a world of one
    # included: one gather to itself, which is how a one-GPU box runs the
    # RCCL path, tests/test_gpu_distributed.py)
    grouped = shard and dist.is_available() and dist.is_initialized()
    world = dist.get_world_size() if grouped else 1
    rank = dist.get_rank() if grouped else 0
    dev = torch.device("cuda", torch.cuda.current_device())
    # add_noise_estimates (fits.py:359-376) runs in the assembly kernel on the
    # shipped mismatch counts: 1,440 B/taxon of asynchronous PCIe (~0.7 ms per
    # 10k taxa, bench host_to_host) costs no host time, while the host
    # statistics (ingest.noise) take ~1.5 ms of CPU per 10k taxa on the 16-thread
    # share of a multi-file pipeline that is host-bound
    if not grouped:
        try:
            return engine.fit_batch_host(p.y, p.N, p.mm, opts, pinned=p.pinned)
        finally:
            p.release_pinned()  # (the call synchronised, or raised: the pinned set goes back either way)
    try:
        return _fit_sharded(p, opts, dev, rank, world)
    finally:
        p.release_pinned()


def _fit_sharded(p: Packed, opts, dev, rank: int, world: int):
    import torch

    from . import engine
    from .distributed import alloc_records, gather_records, shard_capacity, shard_range, unpack_gathered

    lo, hi = shard_range(p.n_taxa, rank, world)
    if opts is not None:  # the sampler's streams are keyed by the global taxon index
        opts = _lib.MdfitOpts.from_buffer_copy(opts)
        opts.index_base = opts.index_base + lo
    cap = shard_capacity(p.n_taxa, world)
    rec = alloc_records(cap, dev)
    if hi > lo:
        # the shard through the bounded-memory chunked dispatch, each chunk's
        # records written in place into the gather buffers
        with engine._STAGING_LOCK:
            st = engine.staging(hi - lo, device=dev, opts=opts, with_mm=p.mm is not None, dest_on_device=True)
            st.run_into_device(p.y[lo:hi], p.N[lo:hi], p.mm[lo:hi] if p.mm is not None else None, opts,
                               engine.FitBatch(rec.out[: hi - lo], rec.pred[: hi - lo], rec.status[: hi - lo]))
            torch.cuda.synchronize(dev)  # (the chunks' pinned input staging is reused by the next call)
    p.release_pinned()
    buf = rec.stage()
    torch.cuda.synchronize(dev)
    parts = gather_records(buf, cap, rank, world)
    if rank != 0:
        return None
    return unpack_gathered(parts, p.n_taxa, world)


# --------------------------------------------------------------------------
# frames (fits.py:632-680)
# --------------------------------------------------------------------------
def _category(p: Packed, name: str, keep, repeat: int = 1) -> pd.Categorical:
    """astype("category") of np.repeat(getattr(p, name)[keep], repeat) (keep
    None: every taxon):
    categories = the sorted distinct values.  From the packed categorical when
    there is one (its categories are sorted already), else by factorising the
    per-taxon values once (the predictions repeat each taxon 30 times)."""
    cat = p.cats.get(name)
    if cat is None:
        v = getattr(p, name)
        c = pd.Categorical(v if keep is None else v[keep])
    else:
        # remove_unused_categories by a presence table instead of np.unique's
        # sort (the categories stay in their sorted order)
        codes = cat.codes if keep is None else cat.codes[keep]
        used = np.zeros(len(cat.categories), bool)
        used[codes[codes >= 0]] = True
        if used.all():
            c = pd.Categorical.from_codes(codes, dtype=cat.dtype)
        else:
            remap = (np.cumsum(used) - 1).astype(codes.dtype)
            c = pd.Categorical.from_codes(np.where(codes >= 0, remap[np.maximum(codes, 0)], -1).astype(codes.dtype),
                                          cat.categories[used])
    return pd.Categorical.from_codes(np.repeat(c.codes, repeat), dtype=c.dtype) if repeat != 1 else c


def _const_category(value, n: int) -> pd.Categorical:
    """astype("category") of a column holding one value (no categories when empty)."""
    return pd.Categorical.from_codes(np.zeros(n, np.int8), [value] if n else [])


def _uint32(v: np.ndarray) -> np.ndarray:
    if v.size and int(v.max()) > np.iinfo(np.uint32).max:
        raise AssertionError("Dataframe contains too large values.")  # utils.py:338-339
    return v.astype(np.uint32)


def _record_columns(out, keep, ncol: int, block: int = 2048) -> np.ndarray:
    """The first ncol columns of the kept rows of the row-major record as a
    column-major float64[ncol][n], transposed block by block (a column gathered
    from the 640-B record rows touches one cache line per taxon; a whole-array
    transposed copy ~4x slower than these cache-sized blocks)."""
    idx = None if keep is None else np.flatnonzero(keep)
    n = out.shape[0] if idx is None else idx.size
    cols = np.empty((ncol, n), np.float64)
    for i in range(0, n, block):
        rows = out[i:i + block, :ncol] if idx is None else out[idx[i:i + block], :ncol]
        cols[:, i:i + block] = rows.T
    return cols


def make_df_fit_results(p: Packed, out, keep, cfg) -> pd.DataFrame:
    """One row per fitted taxon in FIT_RESULT_COLUMNS order with the dtypes of
    downcast_dataframe (fits.py:668-680 + utils.py:329-356): names
    categorical, integer fields uint32, the rest float32."""
    n = int(keep.sum())
    keep = None if n == len(keep) else keep  # (every taxon kept: no row selection)
    data = {
        "tax_id": _category(p, "tax_id", keep),
        "tax_name": _category(p, "tax_name", keep),
        "tax_rank": _category(p, "tax_rank", keep),
    }
    cols = _record_columns(out, keep, _lib.NRESULT)
    for j, name in enumerate(_lib.RESULT_FIELDS):
        v = cols[j]
        data[name] = _uint32(np.rint(v).astype(np.int64)) if name in INT_RESULT_FIELDS else v.astype(np.float32)
    data["N_alignments"] = _uint32(p.N_alignments if keep is None else p.N_alignments[keep])
    data["shortname"] = _const_category(cfg.shortname, n)
    return pd.DataFrame({c: data[c] for c in FIT_RESULT_COLUMNS}, copy=False)


def make_df_fit_predictions(p: Packed, pred, keep, cfg) -> pd.DataFrame:
    """fits.py:632-665: 30 rows per fitted taxon (z = 1..15, -1..-15)."""
    n = int(keep.sum())
    kp = pred if n == len(keep) else pred[keep]
    return pd.DataFrame(
        {
            "tax_id": _category(p, "tax_id", None if n == len(keep) else keep, _lib.NPOS),
            "position": np.tile(POSITIONS.astype(np.int8), n),
            "median": np.ascontiguousarray(kp[:, 0, :], dtype=np.float32).reshape(-1),
            "hdpi_lower": np.ascontiguousarray(kp[:, 1, :], dtype=np.float32).reshape(-1),
            "hdpi_upper": np.ascontiguousarray(kp[:, 2, :], dtype=np.float32).reshape(-1),
            "shortname": _const_category(cfg.shortname, n * _lib.NPOS),
        },
        copy=False,
    )


def make_opts(cfg, mcmc_kwargs=None):
    """Engine options for cfg.inference: "nuts" (the reference's sampler,
    num_warmup / num_samples from mcmc_kwargs as fits.py:792-799 passes them)
    or "map"."""
    inference = getattr(cfg, "inference", "nuts")
    if inference == "map":
        return _lib.default_opts(mode=_lib.MODE_MAP)
    if inference != "nuts":
        raise ValueError(f"inference must be 'nuts' or 'map', got {inference!r}")
    kw = mcmc_kwargs or {}
    return _lib.default_opts(mode=_lib.MODE_NUTS, num_warmup=int(kw.get("num_warmup", 500)),
                             num_samples=int(kw.get("num_samples", 1000)))


def compute_fits(df_counts, cfg, mcmc_kwargs=None, opts=None, shard=True):
    """fits.py:709-730: (df_fit_results, df_fit_predictions) for every taxon of
    df_counts, in df_counts order, by the sampler (cfg.inference "nuts", the
    reference's NUTS with mcmc_kwargs' warmup / samples) or the MAP fit."""
    if opts is None:
        opts = make_opts(cfg, mcmc_kwargs)
    p = pack_counts(df_counts, cfg)
    res = fit_packed(p, opts, shard=shard)
    if res is None:  # non-zero rank of a multi-GPU job
        return None, None
    out, pred, status = res
    keep = status == _lib.OK
    for t in np.where(~keep)[0]:
        logger.warning(f"Fit: tax_id {p.tax_id[t]} failed (status {int(status[t])}). Skipping.")
    return make_df_fit_results(p, out, keep, cfg), make_df_fit_predictions(p, pred, keep, cfg)


def extract_top_max_fits(df_counts, max_fits):
    """fits.py:736-744: taxa with the largest summed N_alignments (ties: first
    in groupby order, i.e. ascending tax_id).

    A categorical tax_id (every counts table of counts.compute_counts) is
    summed per category code with bincount and the winners picked by a stable
    sort -- the set nlargest(keep="first") picks, ties broken by group order --
    and a selection of every taxon returns the table itself (the common case:
    max_fits unset; the groupby + isin + row copy cost ~0.15 s of the driver's
    main thread per 100k-taxon file)."""
    tax = df_counts["tax_id"]
    if isinstance(tax.dtype, pd.CategoricalDtype) and len(df_counts):
        codes = tax.cat.codes.to_numpy()
        n_cat = len(tax.cat.categories)
        from . import ingest

        used, n_missing = ingest.used_codes(codes, n_cat) if n_cat < 2**31 else (None, 1)
        if n_missing == 0:
            present = np.flatnonzero(used)
            if max_fits >= len(present):
                return df_counts
            sums = np.bincount(codes, weights=df_counts["N_alignments"].to_numpy(np.float64), minlength=n_cat)
            # groupby(observed=True) orders the groups by category code
            order = np.argsort(-sums[present], kind="stable")
            chosen = np.zeros(n_cat, bool)
            chosen[present[order[:max_fits]]] = True
            return df_counts[chosen[codes]]
    top = df_counts.groupby("tax_id", observed=True)["N_alignments"].sum().nlargest(max_fits).index
    return df_counts[df_counts["tax_id"].isin(top)]


def get_top_max_fits(df_counts, N_fits):
    if N_fits is not None and N_fits > 0:
        return extract_top_max_fits(df_counts, N_fits)
    return df_counts


def _rank() -> int:
    import torch.distributed as dist

    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


CACHE_KEYS = ["min_alignments", "min_y_sum", "substitution_bases_forward", "substitution_bases_reverse",
              "N_fits", "shortname", "filename", "inference"]


def _cache_hit(cfg) -> bool:
    """This rank's fit cache check (fits.py:767-783): both parquets exist (and
    --forced is off) with metadata equal on CACHE_KEYS."""
    parquet_fit_results = io.Parquet(cfg.filename_fit_results)
    parquet_fit_predictions = io.Parquet(cfg.filename_fit_predictions)
    if not (parquet_fit_results.exists(cfg.forced) and parquet_fit_predictions.exists(cfg.forced)):
        return False
    metadata_cfg = cfg.to_dict()
    return utils.metadata_is_similar(parquet_fit_results.load_metadata(), metadata_cfg, include=CACHE_KEYS) and \
        utils.metadata_is_similar(parquet_fit_predictions.load_metadata(), metadata_cfg, include=CACHE_KEYS)


def prepare_fits(df_counts, cfg):
    """The host work of get_fits ahead of the device call -- the top-N cut and
    the packing -- for a reader thread (main.main runs it beside the previous
    file's fit); None when this rank's fit cache is a hit (get_fits decides)."""
    if _cache_hit(cfg):
        return None
    return pack_counts(get_top_max_fits(df_counts, cfg.N_fits), cfg, pinned=True)


def get_fits(df_counts, cfg, opts=None, shard=True, writer=None, packed=None, deferred=False):
    """fits.py:754-807.  shard: split the taxa over the torch.distributed ranks
    (rank 0 gathers and saves); writer: an executor for the parquet saves;
    packed: prepare_fits(df_counts, cfg) when it ran already.  deferred: return
    a callable that builds the two frames and submits their saves (main.main
    runs it on a writer thread while the next file fits) instead of the
    frames, once the device results are on the host."""
    from .distributed import all_ranks_agree

    parquet_fit_results = io.Parquet(cfg.filename_fit_results)
    parquet_fit_predictions = io.Parquet(cfg.filename_fit_predictions)
    hit = _cache_hit(cfg)
    if shard:  # a taxon-sharded fit is collective: every rank reuses the cache or none does
        hit = all_ranks_agree(hit)
    if hit:
        if shard and _rank() != 0:
            return None, None
        logger.info("Fit: Loading fits from parquet-file.")
        return parquet_fit_results.load(), parquet_fit_predictions.load()
    logger.info("Fit: Generating fits and saving to file.")
    p = packed if packed is not None else pack_counts(get_top_max_fits(df_counts, cfg.N_fits), cfg)
    # fits.py:792-799
    mcmc_kwargs = dict(progress_bar=False, num_warmup=500, num_samples=1000, num_chains=1, chain_method="sequential")
    res = fit_packed(p, opts if opts is not None else make_opts(cfg, mcmc_kwargs), shard=shard)
    if res is None:  # non-zero rank of a multi-GPU job
        return None, None
    out, pred, status = res
    keep = status == _lib.OK
    for t in np.where(~keep)[0]:
        logger.warning(f"Fit: tax_id {p.tax_id[t]} failed (status {int(status[t])}). Skipping.")

    def finish():
        from .counts import _save

        df_fit_results = make_df_fit_results(p, out, keep, cfg)
        df_fit_predictions = make_df_fit_predictions(p, pred, keep, cfg)
        _save(writer, parquet_fit_results, df_fit_results, cfg.to_dict())
        _save(writer, parquet_fit_predictions, df_fit_predictions, cfg.to_dict())
        return df_fit_results, df_fit_predictions

    return finish if deferred else finish()
