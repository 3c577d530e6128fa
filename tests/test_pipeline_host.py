"""CPU tests of the host side of the per-file driver (main.py) and of the
packing fast path: file-sharding over gloo ranks, the overlapped reader /
writer threads, and the reshape vs row-scatter packing paths agreeing with a
row-by-row restatement of group_to_numpyro_data (fits.py:398-419)."""

from __future__ import annotations

import multiprocessing as mp
import os
import shutil
import socket

import numpy as np
import pandas as pd
import pytest

from metadamage_amd import counts, fits, io, utils
from metadamage_amd import main as main_mod
from tests.helpers import GOLDEN


def _cfg(out_dir, **kw):
    return utils.Config(out_dir=out_dir, max_fits=None, max_cores=1, min_alignments=10, min_y_sum=10,
                        substitution_bases_forward=kw.get("fwd", "CT"), substitution_bases_reverse=kw.get("rev", "GA"),
                        forced=kw.get("forced", True), version="0.0.0", inference="map")


def _pack_rows(df, cfg):
    """Row-by-row packing: taxa in first-appearance order, each row's counts at
    its position's column."""
    fwd, rev = cfg.substitution_bases_forward, cfg.substitution_bases_reverse
    order = list(dict.fromkeys(df["tax_id"].tolist()))
    idx = {t: i for i, t in enumerate(order)}
    y = np.zeros((len(order), 32), np.uint32)
    N = np.zeros((len(order), 32), np.uint32)
    mm = np.zeros((len(order), 30, 12), np.uint32)
    for r in df.itertuples(index=False):
        r = r._asdict()
        z = int(r["position"])
        c = z - 1 if z > 0 else 14 - z
        t = idx[r["tax_id"]]
        y[t, c] = r[fwd] if z > 0 else r[rev]
        N[t, c] = r[fwd[0]] if z > 0 else r[rev[0]]
        mm[t, c] = [r[k] for k in fits.MM_COLUMNS]
    return order, y, N, mm


@pytest.mark.parametrize("how", ["dense", "shuffled", "missing_rows", "empty"])
def test_pack_paths_match_row_restatement(how):
    cfg = _cfg("/tmp/mdfit_unused")
    df = pd.read_parquet(GOLDEN / "counts_synthetic.parquet")
    rng = np.random.default_rng(5)
    if how == "shuffled":
        df = df.iloc[rng.permutation(len(df))]
    elif how == "missing_rows":
        df = df.iloc[np.sort(rng.choice(len(df), len(df) * 2 // 3, replace=False))]
    elif how == "empty":
        df = df.iloc[:0]
    p = fits.pack_counts(df, cfg)
    order, y, N, mm = _pack_rows(df, cfg)
    assert list(p.tax_id) == order
    assert p.y.dtype == p.N.dtype == p.mm.dtype == np.uint32
    np.testing.assert_array_equal(p.y, y)
    np.testing.assert_array_equal(p.N, N)
    np.testing.assert_array_equal(p.mm, mm)
    first = ~pd.Series(df["tax_id"].to_numpy()).duplicated().to_numpy()
    np.testing.assert_array_equal(p.N_alignments, df["N_alignments"].to_numpy()[first].astype(np.int64))
    np.testing.assert_array_equal(p.tax_name, df["tax_name"].to_numpy()[first])


def _files(tmp_path, n):
    out = []
    for i in range(n):
        f = tmp_path / f"sample{i}.txt"
        shutil.copy(GOLDEN / "data_ancient.txt", f)
        out.append(f)
    return out


def _fake_get_fits(log):
    def get_fits(df_counts, cfg, opts=None, shard=True, writer=None, packed=None, deferred=False):
        log.append((cfg.shortname, shard, len(df_counts)))
        # the reader thread packed the file (every taxon: max_fits unset)
        assert packed is not None and packed.n_taxa == df_counts["tax_id"].nunique()
        if deferred:
            return lambda: (cfg.shortname, shard)
        return cfg.shortname, shard
    return get_fits


def test_main_overlaps_reads_and_writes(tmp_path, monkeypatch):
    files = _files(tmp_path, 3)
    log = []
    monkeypatch.setattr(fits, "get_fits", _fake_get_fits(log))
    cfg = _cfg(tmp_path / "out")
    res = main_mod.main(files, cfg)
    assert list(res) == ["sample0", "sample1", "sample2"]
    assert res["sample1"] == ("sample1", True)  # the deferred frames resolved
    assert [s for s, _, _ in log] == ["sample0", "sample1", "sample2"] and all(sh for _, sh, _ in log)
    assert cfg.shortname == "sample2"  # the caller's cfg follows the files
    for f in files:  # the counts parquet written on the writer threads is the computed table
        c = _cfg(tmp_path / "out")
        c.add_filename(f)
        back = io.Parquet(c.filename_counts).load()
        want = counts.compute_counts(c)
        pd.testing.assert_frame_equal(back, want)


def test_main_surfaces_failed_writes(tmp_path, monkeypatch):
    files = _files(tmp_path, 2)
    monkeypatch.setattr(fits, "get_fits", _fake_get_fits([]))

    def boom(self, df, metadata=None):
        raise OSError("disk full")

    monkeypatch.setattr(io.Parquet, "save", boom)
    with pytest.raises(OSError, match="disk full"):
        main_mod.main(files, _cfg(tmp_path / "out"))


def test_main_all_bad_files(tmp_path):
    empty = tmp_path / "empty.txt"
    empty.write_text("")
    with pytest.raises(Exception, match="All files were bad"):  # reference main.py:72-74
        main_mod.main([empty], _cfg(tmp_path / "out"))
    with pytest.raises(FileNotFoundError):  # a missing file raises, as utils.py:227-239
        main_mod.main([tmp_path / "missing.txt"], _cfg(tmp_path / "out"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_worker(rank, world, port, files, out_dir, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log = []
        fits.get_fits = _fake_get_fits(log)
        main_mod.main(files, _cfg(out_dir))
        q.put((rank, log))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_files,world", [(5, 2), (1, 2), (3, 3), (10, 8)])
def test_main_deals_files_to_ranks(tmp_path, n_files, world):
    """At least as many files as ranks: files round-robin, fitted unsharded on
    the owning rank.  Fewer: every rank reads every file and the fit shards
    the taxa (fit_packed)."""
    files = _files(tmp_path, n_files)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_worker, args=(r, world, port, files, tmp_path / "out", q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    names = [f"sample{i}" for i in range(n_files)]
    for r in range(world):
        if n_files >= world:
            assert [(s, sh) for s, sh, _ in got[r]] == [(s, False) for s in names[r::world]]
        else:
            assert [(s, sh) for s, sh, _ in got[r]] == [(s, True) for s in names]
