"""Count ingest + cuts: the input side of the fit boundary.

Restates /root/reference/metadamage/counts.py:212-306 without dask (the
reference's LocalCluster is process plumbing, not semantics); every step keeps
the reference's meaning and column order:

  read (counts.py:229-235)            22 headerless columns, or the shipped
                                      20-column headed format via the adapter
                                      
  add_reference_counts (:86-89)       C = sum(C*), G = sum(G*) (per cfg bases)
  add_error_rates (:109-114)          f_CT = CT / C, f_GA = GA / G
  make_position_1_indexed (:117-120)  position += 1
  make_reverse_position_negative      position = -position on the 3' strand
  replace_nans_with_zeroes (:175-176)
  add_y_sum_counts (:179-204)         y_sum_total = sum CT (z>0) + sum GA (z<0)
  filter_cut_based_on_cfg (:207-209)  N_alignments >= min_alignments and
                                      y_sum_total >= min_y_sum   (unchanged)
  sort_by_alignments (:167-172)       N_alignments, tax_id desc; z = 1..15, -1..-15
  downcast_dataframe                  utils.py:329-356
  load_counts (:276-306)              parquet cache keyed on 6 config fields
"""

from __future__ import annotations

import logging
from pathlib import Path

import numpy as np
import pandas as pd

from . import io, utils

logger = logging.getLogger(__name__)

ACTG = ["A", "C", "G", "T"]
ref_obs_bases = [f"{r}{o}" for r in ACTG for o in ACTG]
columns = ["tax_id", "tax_name", "tax_rank", "N_alignments", "strand", "position", *ref_obs_bases]


def get_base_columns(df):
    return [c for c in df.columns if len(c) == 2 and c[0] in ACTG and c[1] in ACTG]


def add_reference_counts(df, ref):
    df[ref] = df[[c for c in get_base_columns(df) if c[0] == ref]].sum(axis=1)
    return df


def add_error_rates(df, ref, obs):
    with np.errstate(divide="ignore", invalid="ignore"):
        df[f"f_{ref}{obs}"] = df[ref + obs] / df[ref]
    return df


def make_position_1_indexed(df):
    df["position"] += 1
    return df


def make_reverse_position_negative(df):
    is_reverse = ~utils.is_forward(df)
    df["position"] = df["position"].mask(is_reverse, -df["position"])
    return df


def replace_nans_with_zeroes(df):
    return df.fillna(0)


def compute_y_sum_total(df, cfg):
    """Per-taxon y_sum_total (counts.py:179-189), vectorised over taxa."""
    fwd = cfg.substitution_bases_forward
    rev = cfg.substitution_bases_reverse
    y = np.where(df["position"] > 0, df[fwd], 0) + np.where(df["position"] < 0, df[rev], 0)
    return pd.Series(y, index=df.index).groupby(df["tax_id"], sort=True).sum().rename("y_sum_total")


def add_y_sum_counts(df, cfg):
    ys = compute_y_sum_total(df, cfg).reset_index()
    return pd.merge(df, ys, on=["tax_id"])


def filter_cut_based_on_cfg(df, cfg):
    """counts.py:207-209 — the frozen cut."""
    return df[(df["N_alignments"] >= cfg.min_alignments) & (df["y_sum_total"] >= cfg.min_y_sum)]


def sort_by_alignments(df):
    pos = df["position"]
    df = df.assign(order=pos.mask(pos > 0, 1 / pos))
    return df.sort_values(by=["N_alignments", "tax_id", "order"], ascending=False).drop(columns=["order"])


def _is_headed_20col(filename) -> bool:
    with open(filename, "r") as fh:
        first = fh.readline()
    return first.startswith("#") or len(first.rstrip("\n").split("\t")) == 20


def read_counts_file(filename) -> pd.DataFrame:
    """The reference's 22-column headerless table (counts.py:37-45, 230-235),
    or the 20-column headed files shipped in data/input/ (#taxid Nalignments
    Direction Pos AA..TT; 0-indexed positions) through an adapter that
    synthesises tax_name = "taxid_<id>" and tax_rank = "unknown"."""
    if not _is_headed_20col(filename):
        return pd.read_csv(filename, sep="\t", header=None, names=columns)
    raw = pd.read_csv(filename, sep="\t")
    df = pd.DataFrame(
        {
            "tax_id": raw["#taxid"].astype(np.int64),
            "tax_name": raw["#taxid"].map(lambda t: f"taxid_{t}"),
            "tax_rank": "unknown",
            "N_alignments": raw["Nalignments"].astype(np.int64),
            "strand": raw["Direction"].astype(str),
            "position": raw["Pos"].astype(np.int64),
        }
    )
    for b in ref_obs_bases:
        df[b] = raw[b].astype(np.int64)
    return df


def compute_counts(cfg, df_raw: pd.DataFrame | None = None) -> pd.DataFrame:
    """counts.compute_counts_with_dask (counts.py:212-273): the native reader +
    vectorised pipeline (metadamage_amd/ingest.py) for a file, the pandas
    restatement for an in-memory table."""
    if df_raw is not None:
        return compute_counts_pandas(cfg, df_raw)
    from . import ingest

    return ingest.compute_counts(cfg)


def compute_counts_pandas(cfg, df_raw: pd.DataFrame | None = None) -> pd.DataFrame:
    """counts.compute_counts_with_dask (counts.py:212-273), the step-by-step
    pandas restatement (kept as the readable statement of the semantics; tests
    hold the native path to it)."""
    fwd, rev = cfg.substitution_bases_forward, cfg.substitution_bases_reverse
    df = read_counts_file(cfg.filename) if df_raw is None else df_raw.copy()
    df = (
        df.pipe(add_reference_counts, ref=fwd[0])
        .pipe(add_reference_counts, ref=rev[0])
        .pipe(add_error_rates, ref=fwd[0], obs=fwd[1])
        .pipe(add_error_rates, ref=rev[0], obs=rev[1])
        .pipe(make_position_1_indexed)
        .pipe(make_reverse_position_negative)
        .pipe(replace_nans_with_zeroes)
        .pipe(add_y_sum_counts, cfg=cfg)
        .pipe(filter_cut_based_on_cfg, cfg)
        .reset_index(drop=True)
        .pipe(sort_by_alignments)
        .reset_index(drop=True)
    )
    df["shortname"] = cfg.shortname
    categories = ["tax_id", "tax_name", "tax_rank", "strand", "shortname"]
    return utils.downcast_dataframe(df, categories, fully_automatic=False)


CACHE_KEYS = ["min_alignments", "min_y_sum", "substitution_bases_forward", "substitution_bases_reverse",
              "shortname", "filename"]


def load_counts(cfg, writer=None, save=True):
    """counts.py:276-306: reuse counts/<shortname>.parquet when its metadata
    matches on CACHE_KEYS and --forced is off; else compute and save (on the
    `writer` executor when one is given: main() overlaps the write with the
    next stages).  save=False computes without writing (the ranks of a
    taxon-sharded job other than rank 0 need the table, not another copy of
    the file)."""
    parquet = io.Parquet(cfg.filename_counts)
    if parquet.exists(cfg.forced):
        if utils.metadata_is_similar(parquet.load_metadata(), cfg.to_dict(), include=CACHE_KEYS):
            logger.info("Loading DataFrame from parquet-file.")
            df_counts = parquet.load()
            cfg.set_number_of_fits(df_counts)
            return df_counts
    logger.info("Creating DataFrame, please wait.")
    df_counts = compute_counts(cfg)
    if save:
        _save(writer, parquet, df_counts, cfg.to_dict())
    cfg.set_number_of_fits(df_counts)
    return df_counts


def _save(writer, parquet, df, metadata):
    if writer is None:
        parquet.save(df, metadata=metadata)
    else:
        writer.submit(parquet.save, df, metadata)


def input_is_file(path) -> bool:
    return Path(path).is_file()
