"""Parquet persistence with the reference's metadata contract.

Mirror of /root/reference/metadamage/io.py:19-91: the config dict is stored as
JSON under the schema-metadata key "metadamage" so that cache checks
(fits.py:759-786, counts.py:281-299) and the dashboard read the files as-is.
The one deliberate difference: the reference writes format version "2.0",
which the installed pyarrow rejects; we write "2.6".
"""

from __future__ import annotations

import ctypes
import json
import os
import threading
from pathlib import Path

import pyarrow as pa
import pyarrow.parquet as pq

from . import utils

PARQUET_VERSION = "2.6"
PQ_LIB = Path(__file__).resolve().parent / "libmdpq.so"
_PQ = None


def _native_writer():
    """libmdpq.so (csrc/pqwrite.cpp): the same file as pq.write_table with the
    columns of each row group encoded in parallel on Arrow's CPU pool.  Two
    handles on the library: mdpq_unwrap through PyDLL (it touches the pyarrow
    object, GIL held), mdpq_write through CDLL (GIL released while encoding, so
    main()'s writer threads and the reader thread run beside it).  None when
    the library is not built (pq.write_table then writes the same file on one
    core)."""
    global _PQ
    if _PQ is None:
        if not PQ_LIB.exists():
            _PQ = False
        else:
            py, c = ctypes.PyDLL(str(PQ_LIB)), ctypes.CDLL(str(PQ_LIB))
            py.mdpq_unwrap.argtypes = [ctypes.py_object]
            py.mdpq_unwrap.restype = ctypes.c_void_p
            c.mdpq_write.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_int, ctypes.c_int64]
            c.mdpq_write.restype = ctypes.c_int
            c.mdpq_last_error.restype = ctypes.c_char_p
            py.mdpq_last_error.restype = ctypes.c_char_p
            _PQ = (py, c)
    return _PQ or None


def write_table(table: "pa.Table", path, dict_cols, stat_cols=None, compression: str = "snappy") -> None:
    """pq.write_table(table, path, version="2.6", use_dictionary=dict_cols,
    write_statistics=stat_cols (default: dict_cols), compression=compression)
    -- natively when libmdpq.so is built."""
    if compression not in ("snappy", "none"):
        raise ValueError(f"compression must be 'snappy' or 'none', got {compression!r}")
    stat_cols = list(dict_cols) if stat_cols is None else list(stat_cols)
    nat = _native_writer()
    if nat is None:
        pq.write_table(table, path, version=PARQUET_VERSION, use_dictionary=list(dict_cols) or False,
                       write_statistics=stat_cols or False, compression=compression)
        return
    py, c = nat
    h = py.mdpq_unwrap(table)
    if not h:
        raise RuntimeError(f"mdpq_unwrap: {py.mdpq_last_error().decode()}")
    names = (ctypes.c_char_p * max(1, len(dict_cols)))(*[n.encode() for n in dict_cols])
    stats = (ctypes.c_char_p * max(1, len(stat_cols)))(*[n.encode() for n in stat_cols])
    if c.mdpq_write(h, os.fsencode(str(path)), names, len(dict_cols), stats, len(stat_cols),
                    int(compression == "snappy"), 0) != 0:
        raise OSError(f"{path}: {c.mdpq_last_error().decode()}")


# tables of at least this many rows (the counts cache, the per-position
# predictions: 30 rows per taxon) are written uncompressed with statistics on
# tax_id only (the key io.Parquet.load filters on): their count / float columns
# compress ~2x at best under snappy, which costs half the encoding CPU of the
# host-bound multi-file pipeline
PLAIN_MIN_ROWS = 1_000_000


class Parquet:
    def __init__(self, filename):
        self.filename = Path(filename)
        self.custom_meta_key = "metadamage"

    def __str__(self):
        return f"Parquet file: '{self.filename}'"

    def __repr__(self):
        return f"Parquet('{self.filename}')"

    def load_metadata(self):
        schema = pq.read_schema(self.filename)
        return json.loads(schema.metadata[self.custom_meta_key.encode()])

    def _load_table(self, shortname=None, tax_id=None, columns=None):
        filename = self.filename
        if shortname is not None:
            filename = filename / f"{shortname}.parquet"
        filters = None if tax_id is None else [("tax_id", "==", tax_id)]
        if isinstance(columns, str):
            columns = [columns]
        return pq.read_table(filename, filters=filters, columns=columns)

    def _table_to_pandas(self, table):
        df = table.to_pandas()
        if "tax_id" in df.columns:
            df = df.astype({"tax_id": "category"})
        return df

    def load(self, shortname=None, tax_id=None, columns=None):
        return self._table_to_pandas(self._load_table(shortname, tax_id=tax_id, columns=columns))

    def _add_metadata_to_table(self, table, metadata):
        meta = {self.custom_meta_key.encode(): json.dumps(metadata or {}).encode(), **(table.schema.metadata or {})}
        return table.replace_schema_metadata(meta)

    def save(self, df, metadata=None):
        """Same schema and metadata as the reference's save; the encoding keeps
        dictionaries and column statistics to the categorical columns (the ones
        readers filter on), which writes a counts table ~1.6x faster than
        dictionary-encoding every numeric column too; tables of PLAIN_MIN_ROWS
        rows and more go uncompressed with statistics on tax_id only.  Plain
        pages (snappy or none) read back with any pyarrow, including the
        reference's ^2.0 pin."""
        utils.init_parent_folder(self.filename)
        table = self._add_metadata_to_table(pa.Table.from_pandas(df), metadata)
        cats = [f.name for f in table.schema if pa.types.is_dictionary(f.type)]
        big = table.num_rows >= PLAIN_MIN_ROWS
        stats = ([c for c in cats if c == "tax_id"] if big else cats)
        comp = "none" if big else "snappy"
        # written next to the target and renamed into place: a reader (another
        # rank's cache check, a writer thread of the next file) sees either no
        # file or a complete one, never a half-written parquet
        tmp = self.filename.with_name(f".{self.filename.name}.{os.getpid()}.{threading.get_ident()}.tmp")
        try:
            write_table(table, tmp, cats, stats, comp)
            os.replace(tmp, self.filename)
        finally:
            if tmp.exists():
                tmp.unlink()

    def exists(self, forced=False):
        return self.filename.exists() and not forced
