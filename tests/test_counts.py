"""CPU tests: count ingest + cuts + packing vs the reference's own pipeline
(golden tables made by tests/golden/make_golden_reference.py)."""

from __future__ import annotations

import numpy as np
import pandas as pd
import pytest

from metadamage_amd import counts, fits, ingest, utils
from tests.helpers import GOLDEN, MM_COLUMNS

CASES = {
    "data_ancient": "data_ancient.txt",
    "data_control": "data_control.txt",
    "synthetic": "synthetic_counts_22col.tsv",
    "synthetic_strict": "synthetic_counts_22col.tsv",
    "synthetic_CA_GT": "synthetic_counts_22col.tsv",
}


def cfg_for(meta_case, path, out_dir="/tmp/mdfit_unused"):
    c = meta_case["cfg"]
    cfg = utils.Config(out_dir=out_dir, max_fits=None, max_cores=1, min_alignments=c["min_alignments"],
                       min_y_sum=c["min_y_sum"], substitution_bases_forward=c["substitution_bases_forward"],
                       substitution_bases_reverse=c["substitution_bases_reverse"], forced=False, version="0.0.0")
    cfg.add_filename(path)
    cfg.shortname = c["shortname"]
    return cfg


@pytest.mark.parametrize("name", list(CASES))
def test_counts_pipeline_matches_reference(name, ref_meta):
    cfg = cfg_for(ref_meta["cases"][name], GOLDEN / CASES[name])
    df = counts.compute_counts(cfg)
    ref = pd.read_parquet(GOLDEN / f"counts_{name}.parquet")
    assert list(df.columns) == list(ref.columns) == ref_meta["cases"][name]["columns"]
    assert len(df) == len(ref)
    for col in ref.columns:
        if isinstance(ref[col].dtype, pd.CategoricalDtype) or ref[col].dtype == object:
            assert (df[col].astype(str).to_numpy() == ref[col].astype(str).to_numpy()).all(), col
        else:
            assert np.array_equal(df[col].to_numpy().astype(float), ref[col].to_numpy().astype(float)), col
    # pandas-1.x dtypes of the reference's downcast (utils.py:329-356)
    assert df["position"].dtype == np.int8
    assert df["N_alignments"].dtype == np.uint32
    assert isinstance(df["tax_id"].dtype, pd.CategoricalDtype)


@pytest.mark.parametrize("name", list(CASES))
def test_packing_matches_group_to_numpyro_data(name, ref_meta, ref_golden):
    cfg = cfg_for(ref_meta["cases"][name], GOLDEN / CASES[name])
    df = pd.read_parquet(GOLDEN / f"counts_{name}.parquet")
    p = fits.pack_counts(df, cfg)
    assert (p.tax_id == ref_golden[f"{name}__tax_id"]).all()
    assert (p.y[:, :30] == ref_golden[f"{name}__y"]).all()
    assert (p.N[:, :30] == ref_golden[f"{name}__N"]).all()
    assert (p.y[:, 30:] == 0).all() and (p.N[:, 30:] == 0).all()
    mm = df[MM_COLUMNS].to_numpy().reshape(-1, 30, 12)
    assert (p.mm == mm).all()


def _general_pack(df, cfg):
    """pack_counts through its general path (an int16 position column skips
    the native dense pass)."""
    d = df.copy()
    d["position"] = d["position"].astype(np.int16)
    return fits.pack_counts(d, cfg)


def _same_pack(a, b):
    assert a.n_taxa == b.n_taxa
    assert (a.y == b.y).all() and (a.N == b.N).all() and (a.mm == b.mm).all()
    assert [str(x) for x in a.tax_id] == [str(x) for x in b.tax_id]
    assert (a.N_alignments == b.N_alignments).all()


@pytest.mark.parametrize("name", list(CASES))
def test_native_dense_pack_equals_general_path(name, ref_meta):
    """ingest.pack_dense (mdi_pack_dense) packs the usual table exactly as the
    general path; tables out of that layout (a taxon short of a row, a taxon
    split in two blocks, positions out of z order) fall back to it."""
    cfg = cfg_for(ref_meta["cases"][name], GOLDEN / CASES[name])
    df = counts.compute_counts(cfg)
    assert df["position"].dtype == np.int8 and df["AC"].dtype == np.uint32
    _same_pack(fits.pack_counts(df, cfg), _general_pack(df, cfg))
    if len(df) < 90:
        return
    short = df.drop(index=df.index[5]).reset_index(drop=True)  # ragged: 29 rows for the first taxon
    _same_pack(fits.pack_counts(short, cfg), _general_pack(short, cfg))
    split = pd.concat([df.iloc[:15], df.iloc[30:60], df.iloc[15:30], df.iloc[60:]]).reset_index(drop=True)
    _same_pack(fits.pack_counts(split, cfg), _general_pack(split, cfg))
    swapped = df.copy()
    p = swapped["position"].to_numpy().copy()
    p[[0, 1]] = p[[1, 0]]
    swapped["position"] = p
    _same_pack(fits.pack_counts(swapped, cfg), _general_pack(swapped, cfg))


def test_packing_categorical_with_a_missing_tax_id(ref_meta):
    """Rows whose tax_id is missing (a categorical's code -1, or NaN in a plain
    column) belong to no taxon -- the reference's groupby(observed=True) drops
    missing keys -- so both forms pack exactly like the table without those
    rows: no extra taxon, and no other taxon's counts overwritten."""
    name = list(CASES)[0]
    cfg = cfg_for(ref_meta["cases"][name], GOLDEN / CASES[name])
    df = pd.read_parquet(GOLDEN / f"counts_{name}.parquet")
    df["tax_id"] = df["tax_id"].astype(str).astype(object)
    full = fits.pack_counts(df, cfg)
    assert full.n_taxa >= 2
    for rows in (slice(-30, None), slice(0, 30)):  # the last taxon's rows, then the first's
        d = df.copy()
        d.loc[d.index[rows], "tax_id"] = np.nan
        ref = fits.pack_counts(d[d["tax_id"].notna()], cfg)
        kept = list(range(1, full.n_taxa)) if rows.start == 0 else list(range(full.n_taxa - 1))
        assert ref.n_taxa == full.n_taxa - 1
        assert (ref.y == full.y[kept]).all() and (ref.N == full.N[kept]).all()
        cat = d.copy()
        cat["tax_id"] = cat["tax_id"].astype("category")
        assert cat["tax_id"].cat.codes.min() == -1
        for frame in (d, cat):
            p = fits.pack_counts(frame, cfg)
            assert p.n_taxa == ref.n_taxa
            assert (p.y == ref.y).all() and (p.N == ref.N).all() and (p.mm == ref.mm).all()
            assert [str(x) for x in p.tax_id] == [str(x) for x in ref.tax_id]


def test_top_max_fits_matches_reference(ref_meta):
    for name in CASES:
        df = pd.read_parquet(GOLDEN / f"counts_{name}.parquet")
        df["tax_id"] = df["tax_id"].astype("category")
        for k, expect in ref_meta["cases"][name]["top_max_fits"].items():
            got = [int(t) for t in pd.unique(fits.get_top_max_fits(df, int(k)).tax_id)]
            assert got == expect, (name, k)


@pytest.mark.parametrize("sorted_cats", [True, False])
def test_top_max_fits_fast_path_equals_groupby(sorted_cats):
    """The bincount selection picks nlargest(keep="first")'s set on tied sums
    and unsorted / unobserved categories, and returns the table itself when
    every taxon is selected."""
    rng = np.random.default_rng(5)
    n = 4000
    cats = np.arange(300) * 7 + 11
    if not sorted_cats:
        cats = rng.permutation(cats)
    codes = rng.integers(0, 250, n)  # categories 250.. never observed
    df = pd.DataFrame({"tax_id": pd.Categorical.from_codes(codes, categories=cats),
                       "N_alignments": rng.integers(1, 4, n), "x": np.arange(n)})
    n_taxa = len(np.unique(codes))
    for k in [1, 2, 17, 100, n_taxa - 1]:
        top = df.groupby("tax_id", observed=True)["N_alignments"].sum().nlargest(k).index
        want = df[df["tax_id"].isin(top)]
        got = fits.extract_top_max_fits(df, k)
        assert got.index.equals(want.index), k
    assert fits.extract_top_max_fits(df, n_taxa) is df
    assert fits.extract_top_max_fits(df, n_taxa + 5) is df


def test_cut_semantics_are_frozen(tmp_path):
    """N_alignments >= min_alignments AND y_sum_total >= min_y_sum (counts.py:207-209),
    y_sum_total = sum of the forward substitution at z > 0 + reverse at z < 0."""
    from metadamage_amd.synthetic import generate, to_counts_table

    b = generate(30, seed=21, fail_fraction=0.5)
    table = to_counts_table(b)
    f = tmp_path / "cut.tsv"
    table.to_csv(f, sep="\t", header=False, index=False)
    cfg = utils.Config(out_dir=tmp_path, max_fits=None, max_cores=1, min_alignments=50, min_y_sum=25,
                       substitution_bases_forward="CT", substitution_bases_reverse="GA", forced=False,
                       version="0.0.0")
    cfg.add_filename(f)
    df = counts.compute_counts(cfg)
    ysum = b.y[:, :15].sum(1) + b.y[:, 15:30].sum(1)
    keep = (b.N_alignments >= 50) & (ysum >= 25)
    assert set(int(t) for t in pd.unique(df.tax_id)) == set(int(t) for t in b.tax_id[keep])
    g = df.groupby("tax_id", observed=True)["y_sum_total"].first()
    for t, v in g.items():
        assert v == ysum[list(b.tax_id).index(int(t))]
    # sort: N_alignments desc, then z = 1..15, -1..-15 within each taxon
    first = df.groupby("tax_id", observed=True, sort=False).head(1)
    assert (np.diff(first["N_alignments"].to_numpy().astype(np.int64)) <= 0).all()
    assert (df["position"].to_numpy()[:30] == np.r_[np.arange(1, 16), -np.arange(1, 16)]).all()


def test_load_counts_cache(tmp_path, ref_meta):
    cfg = cfg_for(ref_meta["cases"]["data_ancient"], GOLDEN / "data_ancient.txt", out_dir=tmp_path)
    df1 = counts.load_counts(cfg)
    assert cfg.filename_counts.exists()
    meta = __import__("metadamage_amd.io", fromlist=["Parquet"]).Parquet(cfg.filename_counts).load_metadata()
    assert meta["shortname"] == cfg.shortname and meta["min_y_sum"] == 10
    df2 = counts.load_counts(cfg)  # cache hit
    assert len(df1) == len(df2) == 90
    assert cfg.N_fits == 3


def test_config_n_cores_rules():
    avail = utils._cpu_count()
    mk = lambda n: utils.Config(out_dir=".", max_fits=None, max_cores=n, min_alignments=10, min_y_sum=10,  # noqa
                                substitution_bases_forward="CT", substitution_bases_reverse="GA",
                                forced=False, version="0.0.0")
    assert mk(1).N_cores == 1
    assert mk(avail + 5).N_cores == avail - 1
    assert mk(-2).N_cores == avail - 2


def test_downcast_raises_on_uint32_overflow():
    df = pd.DataFrame({"a": np.array([2**33], dtype=np.int64)})
    with pytest.raises(AssertionError):
        utils.downcast_dataframe(df, [])


# --------------------------------------------------------------------------
# the native reader (include/mdingest.h) + vectorised pipeline
# --------------------------------------------------------------------------
def _cfg(path, fwd="CT", rev="GA", min_alignments=10, min_y_sum=10):
    cfg = utils.Config(out_dir="/tmp/mdfit_unused", max_fits=None, max_cores=1, min_alignments=min_alignments,
                       min_y_sum=min_y_sum, substitution_bases_forward=fwd, substitution_bases_reverse=rev,
                       forced=False, version="0.0.0")
    cfg.add_filename(path)
    return cfg


@pytest.mark.parametrize("shuffle,bases", [(False, ("CT", "GA")), (True, ("CA", "GT")), (True, ("CT", "CT"))])
def test_native_pipeline_equals_pandas_restatement(tmp_path, shuffle, bases):
    """Frame-identical to counts.compute_counts_pandas, on the usual layout (fast
    row order) and on shuffled rows (full sort), with other substitution bases."""
    from metadamage_amd import ingest
    from metadamage_amd.synthetic import generate, to_counts_table

    table = to_counts_table(generate(400, seed=31, fail_fraction=0.2))
    if shuffle:
        table = table.sample(frac=1, random_state=1)
    f = tmp_path / "t.tsv"
    table.to_csv(f, sep="\t", header=False, index=False)
    cfg = _cfg(f, *bases)
    pd.testing.assert_frame_equal(ingest.compute_counts(cfg), counts.compute_counts_pandas(cfg))


def test_native_reader_threads_and_line_endings(tmp_path):
    from metadamage_amd import ingest
    from metadamage_amd.synthetic import generate, to_counts_table

    table = to_counts_table(generate(3000, seed=32))
    f = tmp_path / "t.tsv"
    table.to_csv(f, sep="\t", header=False, index=False)
    a = ingest.read_table(f, 1)
    b = ingest.read_table(f, 7)
    for k in ("tax_id", "n_alignments", "position", "counts", "name_code", "strand_code"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    g = tmp_path / "crlf.tsv"
    g.write_bytes(f.read_bytes().replace(b"\n", b"\r\n") + b"\r\n")
    c = ingest.read_table(g, 4)
    assert np.array_equal(a.counts, c.counts) and list(c.names[c.name_code]) == list(a.names[a.name_code])


def test_native_reader_errors(tmp_path):
    from metadamage_amd import ingest

    with pytest.raises(FileNotFoundError):
        ingest.read_table(tmp_path / "missing.tsv")
    f = tmp_path / "bad.tsv"
    good = "7\tname\tspecies\t100\t5'\t0" + "\t1" * 16 + "\n"
    f.write_text(good * 3 + "7\tname\tspecies\t100\t5'\tx" + "\t1" * 16 + "\n")
    with pytest.raises(ValueError, match="line 4, column 6"):
        ingest.read_table(f)


@pytest.mark.parametrize("newline_at_end", [True, False])
def test_native_reader_integer_widths(tmp_path, newline_at_end):
    """The 8-digits-at-a-time integer scan: every width 1..18, signs, "12.0",
    names that only share a prefix with the previous row's, and a last field
    within 8 bytes of the end of the file (read with the byte-wise scan)."""
    from metadamage_amd import ingest

    rng = np.random.default_rng(3)
    rows, want = [], []
    names = ["taxon_a", "taxon_ab", "taxon_a", "taxon_", "x"]
    for i in range(400):
        w = 1 + i % 18
        v = [int(rng.integers(10 ** (w - 1) if w > 1 else 0, 10 ** w)) for _ in range(16)]
        pos = int(rng.integers(0, 15))
        nal = int(rng.integers(0, 10 ** (1 + i % 12)))
        tid = int(rng.integers(1, 10 ** (1 + i % 17)))
        sv = [str(x) for x in v]
        if i % 7 == 0:
            sv[3] = f"+{v[3]}"
        if i % 11 == 0:
            sv[5] = f"{v[5]}.000"
        rows.append("\t".join([str(tid), names[i % 5], "species", str(nal), "5'" if i % 2 else "3'", str(pos), *sv]))
        want.append((tid, names[i % 5], nal, pos, v))
    rows.append("\t".join(["5", "x", "genus", "1", "5'", "-3"] + ["1"] * 15 + ["7"]))
    want.append((5, "x", 1, -3, [1] * 15 + [7]))
    f = tmp_path / "w.tsv"
    f.write_text("\n".join(rows) + ("\n" if newline_at_end else ""))
    for nt in (1, 3):
        t = ingest.read_table(f, nt)
        assert t.rows == len(want)
        assert list(t.tax_id) == [w[0] for w in want]
        assert list(t.names[t.name_code]) == [w[1] for w in want]
        assert list(t.n_alignments) == [w[2] for w in want]
        assert list(t.position) == [w[3] for w in want]
        assert np.array_equal(t.counts.T, np.array([w[4] for w in want], dtype=np.int64))


def test_native_reader_on_the_shipped_headed_files():
    from metadamage_amd import ingest

    for name in ("data_ancient.txt", "data_control.txt"):
        t = ingest.read_table(GOLDEN / name)
        raw = pd.read_csv(GOLDEN / name, sep="\t")
        assert t.format == 20 and t.rows == len(raw)
        assert np.array_equal(t.tax_id, raw["#taxid"].to_numpy())
        assert np.array_equal(t.counts.T, raw[[r + o for r in "ACGT" for o in "ACGT"]].to_numpy())


@pytest.mark.parametrize("layout", ["reversed_within_taxon", "split_runs", "zero_rows", "empty_after_cut"])
def test_native_pipeline_edge_layouts(tmp_path, layout):
    """The native select/gather (csrc/counts.cpp) and the numpy restatement
    agree with the pandas restatement off the usual layout: rows of a taxon out
    of z order, a taxon's rows in two runs, all-zero rows (0/0 error rates),
    and a cut that keeps nothing."""
    from metadamage_amd import ingest
    from metadamage_amd.synthetic import generate, to_counts_table

    table = to_counts_table(generate(60, seed=33, fail_fraction=0.2))
    if layout == "reversed_within_taxon":
        table = table.iloc[::-1]
    elif layout == "split_runs":
        table = pd.concat([table.iloc[: len(table) // 2 + 7], table.iloc[len(table) // 2 + 7:]]).iloc[
            np.r_[np.arange(15), np.arange(len(table) - 20, len(table)), np.arange(15, len(table) - 20)]]
    elif layout == "zero_rows":
        table = table.copy()
        table.iloc[::7, 6:] = 0
    f = tmp_path / "t.tsv"
    table.to_csv(f, sep="\t", header=False, index=False)
    cfg = _cfg(f, min_y_sum=10**12 if layout == "empty_after_cut" else 10)
    want = counts.compute_counts_pandas(cfg)
    if layout == "empty_after_cut":
        assert len(want) == 0
    pd.testing.assert_frame_equal(ingest.compute_counts(cfg), want)
    pd.testing.assert_frame_equal(ingest.compute_counts_numpy(cfg), want)


@pytest.fixture(scope="module")
def table_9000():
    from metadamage_amd.synthetic import generate, to_counts_table

    return to_counts_table(generate(9000, seed=34, fail_fraction=0.1))


@pytest.mark.parametrize("layout", ["usual", "shuffled", "split_runs"])
def test_native_pipeline_threads(tmp_path, layout, table_9000):
    """mdi_select / mdi_gather over several row ranges (>= 65,536 rows per
    thread): runs of a taxon cut by a range boundary, a taxon in two runs far
    apart, and the full sort -- frame-identical to the numpy restatement and to
    the one-thread call."""
    from metadamage_amd import ingest

    table = table_9000
    if layout == "shuffled":
        table = table.sample(frac=1, random_state=2)
    elif layout == "split_runs":
        n = len(table)
        table = table.iloc[np.r_[np.arange(0, 45), np.arange(n // 2, n), np.arange(45, n // 2)]]
    f = tmp_path / "t.tsv"
    table.to_csv(f, sep="\t", header=False, index=False)
    cfg = _cfg(f)
    t = ingest.read_table(f, 3)
    assert t.rows >= 4 * 65536
    many = ingest.compute_counts(cfg, table=t, n_threads=4)
    _assert_frames_identical(many, ingest.compute_counts(cfg, table=t, n_threads=1))
    _assert_frames_identical(many, ingest.compute_counts_numpy(cfg, table=t))


def _assert_frames_identical(a, b):
    """assert_frame_equal for large frames: categoricals by categories + codes
    (pandas boxes every value of a categorical column when comparing)."""
    assert list(a.columns) == list(b.columns) and a.index.equals(b.index)
    for c in a.columns:
        x, y = a[c], b[c]
        assert x.dtype == y.dtype, c
        if isinstance(x.dtype, pd.CategoricalDtype):
            assert x.cat.categories.equals(y.cat.categories), c
            assert np.array_equal(x.cat.codes.to_numpy(), y.cat.codes.to_numpy()), c
        else:
            assert np.array_equal(x.to_numpy(), y.to_numpy(), equal_nan=x.dtype.kind == "f"), c


def test_native_pipeline_uint32_overflow(tmp_path):
    """A kept count above uint32 raises as utils.py:338-339; in a row the cut
    drops it does not."""
    from metadamage_amd import ingest

    row = lambda tid, nal, pos, big: "\t".join(  # noqa: E731
        [str(tid), "n", "species", str(nal), "5'", str(pos)] + [str(big)] + ["30"] * 15) + "\n"
    f = tmp_path / "big.tsv"
    f.write_text(row(1, 100, 0, 2**32) + row(1, 100, 1, 1))
    with pytest.raises(AssertionError, match="too large"):
        ingest.compute_counts(_cfg(f))
    g = tmp_path / "dropped.tsv"
    g.write_text(row(1, 100, 0, 5) + row(2, 3, 0, 2**32))  # taxon 2 fails min_alignments
    df = ingest.compute_counts(_cfg(g))
    assert list(df["tax_id"].astype(int).unique()) == [1]


def test_native_noise_matches_the_reference_restatement():
    """ingest.noise (mdi_noise, the host form of add_noise_estimates,
    fits.py:359-376) against the numpy restatement pinned to the reference's
    own add_noise_estimates (oracle.noise): zero columns, an all-zero taxon,
    a zero half."""
    from metadamage_amd import ingest
    from metadamage_amd.synthetic import generate
    from oracle import oracle as orc

    b = generate(300, seed=8)
    b.mm[5] = 0
    b.mm[6, :, 3] = 0
    b.mm[7, :15, :] = 0
    b.mm[8, :, 5] = 0
    nz = ingest.noise(b.mm)
    ref = np.array([orc.noise(b.mm[i]) for i in range(b.n_taxa)])
    assert np.array_equal(np.isnan(nz), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert (np.abs(nz[ok] - ref[ok]) <= 1e-13 * np.abs(ref[ok])).all()


@pytest.mark.parametrize("n_cat,missing", [(5, False), (5, True), (40_000, False), (40_000, True)])
def test_number_of_fits_counts_distinct_tax_ids_like_pd_unique(n_cat, missing):
    """utils.Config.set_number_of_fits on a categorical tax_id (native
    ingest.used_codes) counts the distinct values as len(pd.unique(...)): unused
    categories left out, a missing value counted once."""
    rng = np.random.default_rng(n_cat)
    vals = rng.choice(n_cat, size=3 * n_cat, replace=True)
    cat = pd.Categorical(vals, categories=np.arange(n_cat + 3))
    if missing:
        cat[[1, 7]] = np.nan
    df = pd.DataFrame({"tax_id": cat})
    cfg = utils.Config(out_dir="/tmp/mdfit_unused", max_fits=None, max_cores=1, min_alignments=10, min_y_sum=10,
                       substitution_bases_forward="CT", substitution_bases_reverse="GA", forced=False,
                       version="0.0.0")
    cfg.set_number_of_fits(df)
    assert cfg.N_tax_ids == len(pd.unique(df.tax_id))
    used, n_missing = ingest.used_codes(cat.codes, n_cat + 3)
    assert n_missing == (2 if missing else 0)
    assert (np.flatnonzero(used) == np.unique(cat.codes[cat.codes >= 0])).all()


@pytest.mark.parametrize("strings", [[], ["a"], ["", "x", ""], ["Escherichia coli", "Bacillus", "β-proteobacterium", "日本"],
                                     [f"taxon {i} sp." for i in range(1000)]])
def test_string_table_split_matches_per_string_decode(strings):
    """ingest._split_strings (one decode and split) gives the string table the
    per-string slices gave, empty and non-ASCII names included."""
    enc = [s.encode() for s in strings]
    raw = b"".join(enc) + b"\0"
    off = np.concatenate([[0], np.cumsum([len(e) for e in enc])]).astype(np.int64)
    got = ingest._split_strings(raw, off, len(strings))
    assert got.dtype == object and list(got) == strings
