"""Native count-table reader (libmdingest.so, include/mdingest.h) and the
vectorised count pipeline on its columns.

The reference reads each input with dask read_csv (counts.py:229-235) and runs
its per-row pandas pipeline (counts.py:86-209); for a 100k-taxon file (3 M rows,
~330 MB) that is ~9 s of host time against ~12 ms of GPU fitting.  Here the
file is memory-mapped and parsed by one thread per chunk, and every pipeline
step is a numpy expression over the parsed columns; the result is the same
DataFrame (column order, categories, dtypes) as counts.compute_counts_pandas,
the line-by-line restatement of the reference.
"""

from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import pandas as pd

LIB_PATH = Path(__file__).resolve().parent / "libmdingest.so"
_LIB = None

ACTG = "ACGT"
BASES = [r + o for r in ACTG for o in ACTG]  # AA AC .. TT, the file's column order


def _load():
    global _LIB
    if _LIB is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} not found: build it (python -c 'import __graft_entry__ as g; g.build()')")
        lib = ctypes.CDLL(str(LIB_PATH))
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.mdi_open.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(vp)]
        lib.mdi_open.restype = ctypes.c_int
        lib.mdi_parse_into.argtypes = [vp] + [vp] * 7
        lib.mdi_parse_into.restype = ctypes.c_int
        lib.mdi_format.argtypes = [vp]
        lib.mdi_format.restype = ctypes.c_int
        lib.mdi_rows.argtypes = [vp]
        lib.mdi_rows.restype = i64
        lib.mdi_n_strings.argtypes = [vp, ctypes.c_int]
        lib.mdi_n_strings.restype = i64
        lib.mdi_string_bytes.argtypes = [vp, ctypes.c_int]
        lib.mdi_string_bytes.restype = i64
        lib.mdi_strings.argtypes = [vp, ctypes.c_int, vp, vp]
        lib.mdi_strings.restype = ctypes.c_int
        lib.mdi_free.argtypes = [vp]
        lib.mdi_free.restype = None
        lib.mdi_last_error.restype = ctypes.c_char_p
        lib.mdi_select.argtypes = [i64, vp, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_char_p, ctypes.c_char_p,
                                   i64, i64, ctypes.c_int, vp, vp, vp, vp, vp]
        lib.mdi_select.restype = i64
        lib.mdi_gather.argtypes = [i64, vp, i64, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_char_p,
                                   ctypes.c_char_p, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp]
        lib.mdi_gather.restype = ctypes.c_int
        lib.mdi_counts_error.restype = ctypes.c_char_p
        lib.mdi_codes.argtypes = [i64, vp, ctypes.c_int, vp, vp, ctypes.c_int, vp, vp]
        lib.mdi_codes.restype = ctypes.c_int
        lib.mdi_remap.argtypes = [i64, ctypes.c_int, vp, vp, ctypes.c_int]
        lib.mdi_remap.restype = ctypes.c_int
        lib.mdi_noise.argtypes = [vp, i64, ctypes.c_int, vp]
        lib.mdi_noise.restype = ctypes.c_int
        lib.mdi_first_index.argtypes = [i64, vp, ctypes.c_int32, vp, vp]
        lib.mdi_first_index.restype = i64
        lib.mdi_interleave.argtypes = [i64, ctypes.c_int, vp, vp, ctypes.c_int]
        lib.mdi_interleave.restype = ctypes.c_int
        lib.mdi_pack_dense.argtypes = [i64, vp, ctypes.c_int32, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp]
        lib.mdi_pack_dense.restype = i64
        lib.mdi_used_codes.argtypes = [i64, vp, ctypes.c_int32, ctypes.c_int, vp, vp]
        lib.mdi_used_codes.restype = i64
        _LIB = lib
    return _LIB


def first_index(codes: np.ndarray, n_cat: int):
    """pd.factorize of category codes (first-appearance numbering), natively
    (mdi_first_index): (taxon int64[n], first int64[T])."""
    codes = np.ascontiguousarray(codes, dtype=np.int32)
    n = codes.size
    taxon = np.empty(n, np.int64)
    first = np.empty(n, np.int64)
    T = _load().mdi_first_index(n, codes.ctypes.data, int(n_cat), taxon.ctypes.data, first.ctypes.data)
    if T < 0:
        raise ValueError(_load().mdi_counts_error().decode())
    return taxon, first[:T]


MDI_E_LAYOUT = -5


def used_codes(codes: np.ndarray, n_cat: int, n_threads: int = 0):
    """(used bool[n_cat], n_missing) of a categorical's codes (mdi_used_codes):
    which categories occur, and how many values are missing (code -1)."""
    codes = np.ascontiguousarray(codes, dtype=np.int32)
    used = np.empty(max(1, n_cat), np.uint8)
    miss = ctypes.c_int64(0)
    lib = _load()
    if lib.mdi_used_codes(codes.size, codes.ctypes.data, int(n_cat), int(n_threads), used.ctypes.data,
                          ctypes.byref(miss)) < 0:
        raise ValueError(lib.mdi_counts_error().decode())
    return used[:n_cat].view(bool), int(miss.value)


def pack_dense(codes: np.ndarray, n_cat: int, position: np.ndarray, cols, y: np.ndarray, N: np.ndarray,
               mm: np.ndarray, n_threads: int = 0) -> int:
    """fits.pack_counts of the usual table in one native pass (mdi_pack_dense):
    codes int32[30 T] (one tax_id code per 30-row block), position int8, cols =
    16 uint32 columns (12 mismatch, y fwd / rev, N fwd / rev); fills y, N
    (uint32[T][ld]) and mm (uint32[T][30][12]).  Returns T, or -1 when the
    table is not in that layout (the outputs are then partly written)."""
    n = codes.size
    assert codes.dtype == np.int32 and position.dtype == np.int8 and len(cols) == 16
    assert all(c.dtype == np.uint32 and c.size == n and c.flags.c_contiguous for c in cols)
    T = n // 30
    assert y.shape[0] >= T and N.shape == y.shape and mm.size >= T * 360 and y.flags.c_contiguous
    assert N.flags.c_contiguous and mm.flags.c_contiguous and y.dtype == N.dtype == mm.dtype == np.uint32
    lib = _load()
    r = lib.mdi_pack_dense(n, codes.ctypes.data, int(n_cat), position.ctypes.data, _ptrs(cols, ctypes.c_void_p),
                           int(y.shape[1]), int(n_threads), y.ctypes.data, N.ctypes.data, mm.ctypes.data)
    if r == MDI_E_LAYOUT:
        return -1
    if r < 0:
        raise ValueError(lib.mdi_counts_error().decode())
    return int(r)


def interleave(cols, out2d: np.ndarray, n_threads: int = 0) -> None:
    """out2d[:, j] = cols[j] for uint32 columns (mdi_interleave)."""
    cols = [np.ascontiguousarray(c, dtype=np.uint32) for c in cols]
    n = out2d.shape[0]
    if out2d.dtype != np.uint32 or not out2d.flags.c_contiguous or out2d.shape[1] != len(cols) or \
            any(c.shape != (n,) for c in cols):
        raise ValueError("interleave: shapes / dtypes")
    ptrs = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    if _load().mdi_interleave(n, len(cols), ptrs, out2d.ctypes.data, int(n_threads)) != 0:
        raise ValueError(_load().mdi_counts_error().decode())


def noise(mm: np.ndarray, n_threads: int = 0) -> np.ndarray:
    """add_noise_estimates (fits.py:359-376) of packed taxa on the host
    (mdi_noise): mm uint32[T][30][12] -> float64[T][3] (normalized_noise,
    _forward, _reverse).  The fit then needs no mismatch counts on the GPU."""
    mm = np.ascontiguousarray(mm, dtype=np.uint32)
    T = mm.shape[0]
    if mm.shape != (T, 30, 12):
        raise ValueError(f"mm must be uint32[T][30][12], got {mm.shape}")
    out = np.empty((T, 3))
    rc = _load().mdi_noise(mm.ctypes.data, T, int(n_threads), out.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"mdi_noise failed ({rc})")
    return out


@dataclass
class Table:
    format: int  # 22 (reference table) or 20 (data/input table)
    tax_id: np.ndarray  # int64[rows]
    n_alignments: np.ndarray
    position: np.ndarray  # as in the file (0-indexed)
    counts: np.ndarray  # int64[16][rows], AA .. TT
    name_code: np.ndarray  # int32[rows] into names
    names: np.ndarray  # object[n]
    rank_code: np.ndarray
    ranks: np.ndarray
    strand_code: np.ndarray
    strands: np.ndarray

    @property
    def rows(self) -> int:
        return len(self.tax_id)


_SCRATCH = threading.local()


def _scratch(name: str, shape, dtype) -> np.ndarray:
    """A per-thread array reused across calls: compute_counts' intermediates
    (the parsed columns, the cut's index arrays; ~0.5 GB per 100k-taxon file)
    are dropped once the output columns are gathered, and refilling mapped
    pages spares the kernel's zeroing of fresh ones -- the pipeline's reader
    threads are bound by host memory traffic."""
    d = _SCRATCH.__dict__.setdefault("arrays", {})
    n = int(np.prod(shape))
    a = d.get(name)
    if a is None or a.size < n or a.dtype != np.dtype(dtype):
        a = d[name] = np.empty(n + n // 8, dtype)
    return a[:n].reshape(shape)


def read_table(path, n_threads: int = 0, scratch: bool = False) -> Table:
    """Parse a count table with the native reader.  scratch: the numeric
    columns live in this thread's reused buffers (valid until its next
    scratch call; compute_counts)."""
    lib = _load()
    h = ctypes.c_void_p()
    rc = lib.mdi_open(os.fsencode(str(path)), int(n_threads), ctypes.byref(h))
    if rc != 0:
        raise FileNotFoundError(f"{path}: {lib.mdi_last_error().decode()}")
    alloc = _scratch if scratch else (lambda name, shape, dtype: np.empty(shape, dtype))
    try:
        n = int(lib.mdi_rows(h))
        cols = [alloc(f"col{i}", n, np.int64) for i in range(3)]
        counts = alloc("counts", (16, n), np.int64)  # column-major: one contiguous array per base pair
        codes = [alloc(f"code{i}", n, np.int32) for i in range(3)]
        # (no pre-fault: the parser threads first-touch their own row ranges in
        # parallel -- faulting ~470 MB here on one thread cost more than the parse)
        rc = lib.mdi_parse_into(h, *(c.ctypes.data for c in cols), counts.ctypes.data,
                                *(c.ctypes.data for c in codes))
        if rc != 0:
            raise ValueError(f"{path}: {lib.mdi_last_error().decode()}")
        tables = []
        for which in range(3):
            k = int(lib.mdi_n_strings(h, which))
            nb = int(lib.mdi_string_bytes(h, which))
            buf = ctypes.create_string_buffer(max(nb, 1))
            off = np.empty(k + 1, np.int64)
            lib.mdi_strings(h, which, buf, off.ctypes.data)
            tables.append(_split_strings(buf.raw, off, k))
        fmt = int(lib.mdi_format(h))
    finally:
        lib.mdi_free(h)
    return Table(fmt, cols[0], cols[1], cols[2], counts, codes[0], tables[0], codes[1], tables[1], codes[2],
                 tables[2])


def _split_strings(raw: bytes, off: np.ndarray, k: int) -> np.ndarray:
    """The k strings raw[off[i]:off[i+1]] (UTF-8) as an object array: newlines
    inserted at the offsets, one decode and one split in C -- a string field
    of the table never holds a newline -- instead of k slices and decodes in
    Python (~0.1 s of a reader thread per 100k-taxon file)."""
    out = np.empty(k, dtype=object)
    if k == 0:
        return out
    b = np.frombuffer(raw, np.uint8, count=int(off[k]))
    if k > 1:
        b = np.insert(b, off[1:k], 10)
    parts = b.tobytes().decode().split("\n")
    if len(parts) != k:  # (a newline inside a field: impossible from the parser; keep the slow form)
        parts = [raw[off[i]:off[i + 1]].decode() for i in range(k)]
    out[:] = parts
    return out


def _categorical_from_codes(codes: np.ndarray, table: np.ndarray) -> pd.Categorical:
    """astype('category') of table[codes] (categories = the sorted distinct
    values present) without materialising a value per row."""
    used = np.flatnonzero(np.bincount(codes, minlength=len(table)))
    vals = table[used]
    order = np.argsort(vals.astype(str) if vals.dtype == object else vals, kind="stable")
    remap = np.zeros(len(table), np.int32)
    remap[used[order]] = np.arange(len(used), dtype=np.int32)
    return pd.Categorical.from_codes(remap[codes], vals[order])


def _ptrs(arrays, ctype):
    return (ctype * len(arrays))(*[a.ctypes.data for a in arrays])


def _categoricals(perm: np.ndarray, columns, n_threads: int = 0) -> list:
    """[astype("category") of table[codes[perm]] for (codes, table) in columns]
    (categories = the sorted distinct values present) with the per-row passes
    -- gather through perm, usage, the remap to category order -- in the native
    library, parallel over row ranges (mdi_codes / mdi_remap); only the used
    values are sorted here."""
    lib = _load()
    k = len(perm)
    ins = [np.ascontiguousarray(c, dtype=np.int32) for c, _ in columns]
    sizes = np.array([len(tbl) for _, tbl in columns], np.int32)
    outs = [np.empty(k, np.int32) for _ in columns]
    used = [np.empty(max(1, len(tbl)), np.uint8) for _, tbl in columns]
    perm = np.ascontiguousarray(perm, dtype=np.int64)
    if lib.mdi_codes(k, perm.ctypes.data, len(columns), _ptrs(ins, ctypes.c_void_p), sizes.ctypes.data,
                     int(n_threads), _ptrs(outs, ctypes.c_void_p), _ptrs(used, ctypes.c_void_p)) != 0:
        raise ValueError(lib.mdi_counts_error().decode())
    remaps, cats = [], []
    for (_, tbl), u in zip(columns, used):
        idx = np.flatnonzero(u[: len(tbl)])
        vals = tbl[idx]
        order = np.argsort(vals.astype(str) if vals.dtype == object else vals, kind="stable")
        remap = np.zeros(max(1, len(tbl)), np.int32)
        remap[idx[order]] = np.arange(len(idx), dtype=np.int32)
        remaps.append(remap)
        cats.append(vals[order])
    if lib.mdi_remap(k, len(columns), _ptrs(outs, ctypes.c_void_p), _ptrs(remaps, ctypes.c_void_p),
                     int(n_threads)) != 0:
        raise ValueError(lib.mdi_counts_error().decode())
    return [pd.Categorical.from_codes(o, dtype=pd.CategoricalDtype(c), validate=False) for o, c in zip(outs, cats)]


def _const_category(value, n: int) -> pd.Categorical:
    """astype("category") of a column holding one value (no categories when empty)."""
    return pd.Categorical.from_codes(np.zeros(n, np.int32), np.array([value] if n else [], object))


def _row_order(taxon, nal, tax_id, order) -> np.ndarray:
    """Row permutation of sort_by_alignments (counts.py:167-172): N_alignments,
    tax_id, order, all descending.  Fast path for the usual layout -- each
    taxon's rows contiguous, already in order, with one N_alignments -- sorts
    the taxa only; anything else takes the full three-key sort."""
    n = len(taxon)
    if n == 0:
        return np.zeros(0, np.int64)
    starts = np.flatnonzero(np.r_[True, taxon[1:] != taxon[:-1]])
    block = np.repeat(np.arange(len(starts)), np.diff(np.r_[starts, n]))
    contiguous = len(starts) == len(np.unique(taxon[starts]))
    if contiguous:
        same_block = block[1:] == block[:-1]
        contiguous = bool(np.all(order[1:][same_block] < order[:-1][same_block])) and bool(
            np.all(nal == nal[starts][block]))
    if not contiguous:
        return np.lexsort((-order, -tax_id, -nal))
    bs = np.lexsort((-tax_id[starts], -nal[starts]))  # blocks: N_alignments, tax_id descending
    lens = np.diff(np.r_[starts, n])[bs]
    first = starts[bs]
    offs = np.repeat(first - np.r_[0, np.cumsum(lens)[:-1]], lens)
    return np.arange(n) + offs


def _frame(cols: dict) -> pd.DataFrame:
    """DataFrame over the given arrays without copying them into a
    consolidated block."""
    return pd.DataFrame(cols, copy=False)


def compute_counts(cfg, table: Table | None = None, n_threads: int = 0) -> pd.DataFrame:
    """counts.py:212-273 on the parsed columns: the cut, the sort and every
    numeric column by the native pipeline (mdi_select / mdi_gather,
    csrc/counts.cpp); the categoricals from the interned string codes.  Same
    frame as compute_counts_numpy and counts.compute_counts_pandas."""
    lib = _load()
    t = read_table(cfg.filename, n_threads, scratch=True) if table is None else table
    fwd, rev = cfg.substitution_bases_forward, cfg.substitution_bases_reverse
    n = t.rows
    is_fwd = np.ascontiguousarray(t.strands == "5'", dtype=np.uint8)
    taxon = _scratch("taxon", n, np.int32)
    ysum = _scratch("ysum", n, np.int64)
    perm = _scratch("perm", n, np.int64)
    common = (t.position.ctypes.data, t.counts.ctypes.data, t.strand_code.ctypes.data, is_fwd.ctypes.data,
              len(is_fwd), fwd.encode(), rev.encode())
    uniq = _scratch("uniq", n, np.int64)
    n_taxa = ctypes.c_int64(0)
    k = lib.mdi_select(n, t.tax_id.ctypes.data, t.n_alignments.ctypes.data, *common, int(cfg.min_alignments),
                       int(cfg.min_y_sum), int(n_threads), taxon.ctypes.data, ysum.ctypes.data, perm.ctypes.data,
                       uniq.ctypes.data, ctypes.byref(n_taxa))
    if k < 0:
        raise ValueError(lib.mdi_counts_error().decode())
    uniq = uniq[:n_taxa.value].copy()
    perm = perm[:k]
    nal = np.empty(k, np.uint32)
    pos = np.empty(k, np.int8)
    c16 = np.empty((16, k), np.uint32)
    ref2 = np.empty((2, k), np.uint32)
    f2 = np.empty((2, k), np.float32)
    ys = np.empty(k, np.uint32)
    rc = lib.mdi_gather(n, perm.ctypes.data, k, t.n_alignments.ctypes.data, *common, ysum.ctypes.data,
                        int(n_threads), nal.ctypes.data, pos.ctypes.data, c16.ctypes.data, ref2.ctypes.data,
                        f2.ctypes.data, ys.ctypes.data)
    if rc != 0:
        raise AssertionError(lib.mdi_counts_error().decode())
    if t.format == 22:
        cat_id, cat_name, cat_rank, cat_strand = _categoricals(
            perm, [(taxon, uniq), (t.name_code, t.names), (t.rank_code, t.ranks), (t.strand_code, t.strands)],
            n_threads)
    else:  # the data/input adapter of counts.read_counts_file: "taxid_<id>", "unknown"
        cat_id, cat_name, cat_strand = _categoricals(
            perm, [(taxon, uniq), (taxon, np.array([f"taxid_{v}" for v in uniq], dtype=object)),
                   (t.strand_code, t.strands)], n_threads)
        cat_rank = _const_category("unknown", k)
    data = {"tax_id": cat_id, "tax_name": cat_name, "tax_rank": cat_rank}
    data["N_alignments"] = nal
    data["strand"] = cat_strand
    data["position"] = pos
    for j, b in enumerate(BASES):
        data[b] = c16[j]
    data[fwd[0]] = ref2[0]
    data[rev[0]] = ref2[1]  # same key as the forward one when both start with one base: the later wins
    data[f"f_{fwd}"] = f2[0]
    data[f"f_{rev}"] = f2[1]
    data["y_sum_total"] = ys
    data["shortname"] = _const_category(cfg.shortname, k)
    return _frame(data)


def compute_counts_numpy(cfg, table: Table | None = None) -> pd.DataFrame:
    """counts.py:212-273 as numpy expressions over the parsed columns (the
    cross-check of compute_counts' native pipeline; see
    counts.compute_counts_pandas for the step-by-step restatement and its
    reference line numbers)."""
    t = read_table(cfg.filename) if table is None else table
    fwd, rev = cfg.substitution_bases_forward, cfg.substitution_bases_reverse
    col = {b: t.counts[j] for j, b in enumerate(BASES)}
    # add_reference_counts (counts.py:86-89), in pipeline order
    extra = {}
    for ref in (fwd[0], rev[0]):
        b4 = [b for b in BASES if b[0] == ref]
        extra[ref] = col[b4[0]] + col[b4[1]] + col[b4[2]] + col[b4[3]]
    # add_error_rates (counts.py:109-114); fillna(0) turns 0/0 into 0, x/0 stays inf
    for sub in (fwd, rev):
        with np.errstate(divide="ignore", invalid="ignore"):
            f = col[sub] / extra[sub[0]]
        f[np.isnan(f)] = 0.0
        extra[f"f_{sub}"] = f
    # positions: 1-indexed, reverse strand negative (counts.py:117-126)
    is_fwd = (t.strands == "5'")[t.strand_code]
    pos = np.where(is_fwd, t.position + 1, -(t.position + 1))
    # y_sum_total per taxon (counts.py:179-204), then the frozen cut (:207-209)
    y = np.where(pos > 0, col[fwd], 0) + np.where(pos < 0, col[rev], 0)
    taxon, uniq = pd.factorize(t.tax_id)
    ysum = np.zeros(len(uniq), np.int64)
    np.add.at(ysum, taxon, y)
    y_sum_total = ysum[taxon]
    keep = np.flatnonzero((t.n_alignments >= cfg.min_alignments) & (y_sum_total >= cfg.min_y_sum))
    # sort_by_alignments (counts.py:167-172): N_alignments, tax_id, z = 1..15, -1..-15 (all descending)
    p = pos[keep]
    order = np.where(p > 0, 1.0 / np.where(p > 0, p, 1), p)
    perm = keep[_row_order(taxon[keep], t.n_alignments[keep], t.tax_id[keep], order)]

    tax = taxon[perm]
    data = {"tax_id": _categorical_from_codes(tax, np.asarray(uniq))}
    if t.format == 22:
        data["tax_name"] = _categorical_from_codes(t.name_code[perm], t.names)
        data["tax_rank"] = _categorical_from_codes(t.rank_code[perm], t.ranks)
    else:  # the data/input adapter of counts.read_counts_file: "taxid_<id>", "unknown"
        names = np.array([f"taxid_{v}" for v in uniq], dtype=object)
        data["tax_name"] = _categorical_from_codes(tax, names)
        data["tax_rank"] = _const_category("unknown", len(perm))
    # downcast_dataframe (utils.py:329-356): ints -> uint32 (position int8), floats -> float32
    ints = [t.n_alignments, *col.values(), *(v for k, v in extra.items() if not k.startswith("f_")), y_sum_total]
    big = np.iinfo(np.uint32).max
    if len(perm) and any(int(a.max()) > big for a in ints):  # exact check on the kept rows only if needed
        if max(int(a[perm].max()) for a in ints) > big:
            raise AssertionError("Dataframe contains too large values.")
    data["N_alignments"] = t.n_alignments[perm].astype(np.uint32)
    data["strand"] = _categorical_from_codes(t.strand_code[perm], t.strands)
    data["position"] = pos[perm].astype(np.int8)
    for b in BASES:
        data[b] = col[b][perm].astype(np.uint32)
    for k, v in extra.items():
        data[k] = v[perm].astype(np.float32 if k.startswith("f_") else np.uint32)
    data["y_sum_total"] = y_sum_total[perm].astype(np.uint32)
    data["shortname"] = _const_category(cfg.shortname, len(perm))
    return pd.DataFrame(data)
