"""Bounded-memory chunked dispatch (engine.plan_chunks): the
split logic on CPU (the library's host-side mdfit_workspace_bytes, no GPU).
The reference fits any number of taxa in 1,000-taxon chunks
(/root/reference/metadamage/fits.py:692-706); here a batch is split into
chunks whose N_SETS device buffer sets fit a device budget, each chunk at most
the C-ABI's 2^25 taxa per call.  GPU equality of chunked and one-call records:
tests/test_gpu_chunks.py."""

from __future__ import annotations

import pytest

from metadamage_amd import _lib, engine


def _check_cover(chunks, T):
    assert chunks[0][0] == 0 and chunks[-1][1] == T
    for (a, b), (c, d) in zip(chunks, chunks[1:]):
        assert b == c
    assert all(b > a for a, b in chunks)
    sizes = [b - a for a, b in chunks]
    assert max(sizes) - min(sizes) <= 1  # near-equal


def test_no_budget_one_chunk():
    assert engine.plan_chunks(10_000) == [(0, 10_000)]
    assert engine.plan_chunks(0) == []


def test_forced_chunk_taxa(monkeypatch):
    ch = engine.plan_chunks(10_000, chunk_taxa=3_000)
    assert len(ch) == 4 and max(b - a for a, b in ch) <= 3_000
    _check_cover(ch, 10_000)
    monkeypatch.setenv("MDFIT_CHUNK_TAXA", "3000")
    assert engine.plan_chunks(10_000) == ch


def test_map_beyond_the_call_limit():
    """More than 2^25 MAP taxa: chunks of at most 2^25, no error."""
    T = (1 << 25) + 12_345
    ch = engine.plan_chunks(T, _lib.default_opts(mode=_lib.MODE_MAP))
    assert len(ch) == 2 and max(b - a for a, b in ch) <= engine.MAX_CALL_TAXA
    _check_cover(ch, T)


@pytest.mark.parametrize("T", [1_400_000, 3_000_000, 10_000_000])
def test_nuts_taxa_beyond_one_gpu_in_one_call(T):
    """The sampler keeps every draw (192 KB per taxon at 1,000 draws): ~1.4M
    taxa filled 60 % of an MI355X's 288 GB in one call.  Chunked, two buffer
    sets of the largest chunk stay within the budget at any T."""
    opts = _lib.default_opts(mode=_lib.MODE_NUTS)
    budget = int(0.6 * 288e9)
    ch = engine.plan_chunks(T, opts, budget)
    _check_cover(ch, T)
    big = max(b - a for a, b in ch)
    assert engine.N_SETS * engine.device_bytes(big, opts) <= budget
    assert engine.device_bytes(big, opts) >= 192_000 * big
    # the largest chunk is within one taxon of the budget's maximum
    assert len(ch) == -(-T // big) or engine.N_SETS * engine.device_bytes(big + 1, opts) > budget


def test_map_budget_across_the_workspace_switch():
    """The MAP workspace grows by ~4.8 KB per taxon from 60k taxa: a budget that
    a 59,999-taxon chunk fits but a 60k one does not gives chunks below 60k."""
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    b59 = engine.N_SETS * engine.device_bytes(59_999, opts)
    b60 = engine.N_SETS * engine.device_bytes(60_000, opts)
    assert b60 > b59 + 60_000 * 4_000
    ch = engine.plan_chunks(200_000, opts, b59 + 1)
    assert max(b - a for a, b in ch) < 60_000
    _check_cover(ch, 200_000)


def test_budget_too_small_raises():
    with pytest.raises(_lib.MdfitError):
        engine.plan_chunks(10, _lib.default_opts(mode=_lib.MODE_NUTS), 1_000)


def test_device_bytes_dest_on_device_smaller():
    opts = _lib.default_opts(mode=_lib.MODE_MAP)
    a = engine.device_bytes(1000, opts)
    b = engine.device_bytes(1000, opts, dest_on_device=True)
    assert a - b == 1000 * (640 + 360 + 4)
