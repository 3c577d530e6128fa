"""Configuration and helpers of the fit pipeline (host side).

Mirrors the parts of /root/reference/metadamage/utils.py that define the
output contract of `metadamage fit`: the Config dataclass whose asdict() is
embedded as parquet metadata (utils.py:43-137), the substitution-base enum
(utils.py:186-201), file/name helpers (utils.py:219-246, 254-263), the
dataframe downcast (utils.py:329-356), the cache-metadata comparison
(utils.py:362-377) and the empty-table check (utils.py:565-573).
PDF/LaTeX/plot helpers of the reference are out of scope.
"""

from __future__ import annotations

import logging
import shutil
from dataclasses import asdict, dataclass, field
from enum import Enum
from pathlib import Path
from typing import Optional

import numpy as np
import pandas as pd

logger = logging.getLogger(__name__)


def _cpu_count() -> int:
    try:
        from psutil import cpu_count

        return int(cpu_count(logical=True))
    except Exception:  # psutil absent
        import os

        return os.cpu_count() or 1


@dataclass
class Config:
    """utils.py:43-137: field names, order and defaults are the parquet
    metadata contract (io.py:64-72)."""

    out_dir: Path
    #
    max_fits: Optional[int]
    max_cores: int
    #
    min_alignments: int
    min_y_sum: int
    #
    substitution_bases_forward: str
    substitution_bases_reverse: str
    #
    forced: bool
    version: str
    #
    filename: Optional[Path] = None
    shortname: Optional[str] = None

    N_filenames: Optional[int] = None
    N_fits: Optional[int] = None
    # this engine's addition: "nuts" samples like the reference (fits.py:382-387),
    # "map" is the frequentist MAP fit (BASELINE config 2); saved in the parquet
    # metadata and part of the cache key
    inference: str = "nuts"
    N_cores: int = field(init=False)

    def __post_init__(self):
        self._set_N_cores()

    def _set_N_cores(self):
        """utils.py:70-85: too large -> available-1, negative -> available-|n|."""
        available_cores = _cpu_count()
        if self.max_cores > available_cores:
            self.N_cores = available_cores - 1
            logger.info(f"'max_cores' larger than available: clipping to {self.N_cores} (available-1) cores")
        elif self.max_cores < 0:
            self.N_cores = available_cores - abs(self.max_cores)
            logger.info(f"'max-cores' negative: using {self.N_cores} (available-max_cores) cores")
        else:
            self.N_cores = self.max_cores

    def add_filenames(self, filenames):
        self.N_filenames = len(filenames)

    def add_filename(self, filename):
        self.filename = filename
        self.shortname = extract_name(filename)

    def _require_shortname(self, what):
        if self.shortname is None:
            raise AssertionError(
                f"Shortname has to be set before {what} is defined: cfg.add_filename(filename) "
            )

    @property
    def filename_counts(self):
        self._require_shortname("filename_counts")
        return Path(self.out_dir) / "counts" / f"{self.shortname}.parquet"

    @property
    def filename_fit_results(self):
        self._require_shortname("filename_fit_results")
        return Path(self.out_dir) / "fit_results" / f"{self.shortname}.parquet"

    @property
    def filename_fit_predictions(self):
        self._require_shortname("filename_fit_predictions")
        return Path(self.out_dir) / "fit_predictions" / f"{self.shortname}.parquet"

    def set_number_of_fits(self, df_counts):
        """utils.py:121-130.  The distinct tax_ids (a missing value counts as
        one, as in pd.unique) of a categorical column by one native pass over
        its codes (ingest.used_codes)."""
        tax = df_counts.tax_id
        if isinstance(tax.dtype, pd.CategoricalDtype) and len(tax.cat.categories) < 2**31:
            from . import ingest

            used, n_missing = ingest.used_codes(tax.cat.codes.to_numpy(), len(tax.cat.categories))
            self.N_tax_ids = int(used.sum()) + (n_missing > 0)
        else:
            self.N_tax_ids = len(pd.unique(tax))
        if self.max_fits is not None and self.max_fits > 0:
            self.N_fits = min(self.max_fits, self.N_tax_ids)
        else:
            self.N_fits = self.N_tax_ids
        logger.info(f"Setting number_of_fits to {self.N_fits}")

    def to_dict(self):
        d_out = asdict(self)
        for key, val in d_out.items():
            if isinstance(val, Path):
                d_out[key] = str(val)
        return d_out


class SubstitutionBases(str, Enum):
    """utils.py:186-201."""

    AC = "AC"
    AG = "AG"
    AT = "AT"

    CA = "CA"
    CG = "CG"
    CT = "CT"

    GA = "GA"
    GC = "GC"
    GT = "GT"

    TA = "TA"
    TC = "TC"
    TG = "TG"


def extract_name(filename, max_length=60):
    """utils.py:219-224."""
    shortname = Path(filename).stem.split(".")[0]
    if len(shortname) > max_length:
        shortname = shortname[:max_length] + "..."
    logger.info(f"Running new file: {shortname}")
    return shortname


def file_is_valid(filename):
    """utils.py:227-239.  As in the reference, a missing file raises
    FileNotFoundError (from Path.stat) rather than returning False."""
    if Path(filename).exists() and Path(filename).stat().st_size > 0:
        return True
    exists = Path(filename).exists()
    valid_size = Path(filename).stat().st_size > 0
    logger.error(f"{filename} is not a valid file. {exists=} and {valid_size=}. Skipping for now.")
    return False


def delete_folder(path):
    try:
        shutil.rmtree(path)
    except OSError:
        logger.exception(f"Could not delete folder, {path}")


def init_parent_folder(filename):
    Path(filename).parent.mkdir(parents=True, exist_ok=True)


def is_forward(df):
    """utils.py:254-255."""
    return df["strand"] == "5'"


def downcast_dataframe(df, categories, fully_automatic=False):
    """utils.py:329-356 with the dtypes it produced under its pinned pandas
    (^1.2): listed columns -> category, integer columns -> uint32 (position ->
    int8), float columns -> float32; raises if an integer exceeds uint32."""
    categories = [c for c in categories if c in df.columns]
    df2 = df.astype({c: "category" for c in categories})
    int_cols = df2.select_dtypes(include=["integer"]).columns
    if len(int_cols) and df2[int_cols].max().max() > np.iinfo("uint32").max:
        raise AssertionError("Dataframe contains too large values.")
    conv = {}
    for col in int_cols:
        if fully_automatic:
            conv[col] = pd.to_numeric(df2[col], downcast="integer").dtype
        else:
            conv[col] = "int8" if col == "position" else "uint32"
    for col in df2.select_dtypes(include=["float"]).columns:
        conv[col] = pd.to_numeric(df2[col], downcast="float").dtype if fully_automatic else "float32"
    return df2.astype(conv)


def metadata_is_similar(metadata_file, metadata_cfg, include=None):
    """utils.py:362-377."""
    if include is None:
        if set(metadata_file.keys()) != set(metadata_cfg.keys()):
            return False
        include = set(metadata_file.keys())
    equals = {key: metadata_file.get(key) == metadata_cfg.get(key) for key in include}
    if not all(equals.values()):
        diff = {key: val for key, val in equals.items() if val is False}
        logger.info(f"The files' metadata are not the same, differing here: {diff}")
        return False
    return True


def is_df_counts_accepted(df_counts, cfg):
    """utils.py:565-573."""
    if len(df_counts) > 0:
        return True
    logger.warning(f"{cfg.shortname}: Length of dataframe was 0. Stopping any further operations on this file.")
    return False
