"""The native parquet writer (libmdpq.so, csrc/pqwrite.cpp: column-parallel
encoding through libparquet) writes the file pq.write_table writes: same
schema and key-value metadata (the "metadamage" config, pandas' own, the
stored Arrow schema), format 2.6, the same row groups, dictionaries and
statistics on the categorical columns only -- and it reads back equal."""

from __future__ import annotations

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from metadamage_amd import io


def _frame(n):
    rng = np.random.default_rng(0)
    return pd.DataFrame({
        "tax_id": pd.Categorical(rng.integers(0, 500, n)),
        "tax_name": pd.Categorical([f"taxon_{i}" for i in rng.integers(0, 500, n)]),
        "N_alignments": rng.integers(0, 2**32 - 1, n, dtype=np.uint32),
        "position": rng.integers(-15, 16, n).astype(np.int8),
        "f_CT": rng.random(n).astype(np.float32),
        "D_max": rng.random(n),
        "shortname": pd.Categorical(["c5_0"] * n),
    })


@pytest.mark.skipif(io._native_writer() is None, reason="libmdpq.so not built")
@pytest.mark.parametrize("n,comp", [(0, "snappy"), (1, "snappy"), (1000, "snappy"), (1_300_000, "snappy"),
                                    (1000, "none"), (1_300_000, "none")])
def test_native_writer_matches_write_table(tmp_path, n, comp):
    df = _frame(n)
    meta = {"out_dir": "x", "N_fits": 3}
    table = io.Parquet(tmp_path / "a")._add_metadata_to_table(pa.Table.from_pandas(df), meta)
    cats = [f.name for f in table.schema if pa.types.is_dictionary(f.type)]
    stats = cats if comp == "snappy" else ["tax_id"]
    io.write_table(table, tmp_path / "native.parquet", cats, stats, comp)
    pq.write_table(table, tmp_path / "pyarrow.parquet", version="2.6", use_dictionary=cats or False,
                   write_statistics=stats or False, compression=comp)
    a, b = pq.read_table(tmp_path / "native.parquet"), pq.read_table(tmp_path / "pyarrow.parquet")
    assert a.equals(b) and a.schema.equals(b.schema, check_metadata=True)
    ma, mb = pq.ParquetFile(tmp_path / "native.parquet").metadata, pq.ParquetFile(tmp_path / "pyarrow.parquet").metadata
    assert ma.format_version == mb.format_version == "2.6"
    assert [ma.row_group(i).num_rows for i in range(ma.num_row_groups)] == \
        [mb.row_group(i).num_rows for i in range(mb.num_row_groups)]
    for i in range(ma.num_row_groups):
        for j in range(ma.num_columns):
            ca, cb = ma.row_group(i).column(j), mb.row_group(i).column(j)
            assert set(ca.encodings) == set(cb.encodings), (ca.path_in_schema, ca.encodings, cb.encodings)
            assert (ca.statistics is None) == (cb.statistics is None), ca.path_in_schema
            assert ca.compression == cb.compression == ("SNAPPY" if comp == "snappy" else "UNCOMPRESSED")
    # the reference's reader path (io.Parquet.load) gives the same frame (save:
    # uncompressed from io.PLAIN_MIN_ROWS rows)
    io.Parquet(tmp_path / "c.parquet").save(df, metadata=meta)
    big = n >= io.PLAIN_MIN_ROWS
    mc = pq.ParquetFile(tmp_path / "c.parquet").metadata
    if mc.num_row_groups:
        assert mc.row_group(0).column(0).compression == ("UNCOMPRESSED" if big else "SNAPPY")
    back = io.Parquet(tmp_path / "c.parquet").load()
    assert back.equals(io.Parquet(tmp_path / "pyarrow.parquet").load())
    assert io.Parquet(tmp_path / "c.parquet").load_metadata() == meta


def test_native_writer_reports_errors(tmp_path):
    if io._native_writer() is None:
        pytest.skip("libmdpq.so not built")
    table = pa.table({"x": [1, 2, 3]})
    with pytest.raises(OSError):
        io.write_table(table, tmp_path / "no_such_dir" / "x.parquet", [])
