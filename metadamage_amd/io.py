"""Parquet persistence with the reference's metadata contract.

Mirror of /root/reference/metadamage/io.py:19-91: the config dict is stored as
JSON under the schema-metadata key "metadamage" so that cache checks
(fits.py:759-786, counts.py:281-299) and the dashboard read the files as-is.
The one deliberate difference: the reference writes format version "2.0",
which the installed pyarrow rejects; we write "2.6".
"""

from __future__ import annotations

import json
import os
import threading
from pathlib import Path

import pyarrow as pa
import pyarrow.parquet as pq

from . import utils

PARQUET_VERSION = "2.6"


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
        dictionary-encoding every numeric column too.  Plain + snappy pages
        read back with any pyarrow, including the reference's ^2.0 pin."""
        utils.init_parent_folder(self.filename)
        table = self._add_metadata_to_table(pa.Table.from_pandas(df), metadata)
        cats = [f.name for f in table.schema if pa.types.is_dictionary(f.type)]
        # written next to the target and renamed into place: a reader (another
        # rank's cache check, a writer thread of the next file) sees either no
        # file or a complete one, never a half-written parquet
        tmp = self.filename.with_name(f".{self.filename.name}.{os.getpid()}.{threading.get_ident()}.tmp")
        try:
            pq.write_table(table, tmp, version=PARQUET_VERSION, use_dictionary=cats,
                           write_statistics=cats or False)
            os.replace(tmp, self.filename)
        finally:
            if tmp.exists():
                tmp.unlink()

    def exists(self, forced=False):
        return self.filename.exists() and not forced
