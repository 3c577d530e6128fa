"""CPU tests of the C-ABI boundary: the in-tree libmdfit.so loads without a GPU
and exports every function include/mdfit.h declares (no compute calls)."""

from __future__ import annotations

import ctypes
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "mdfit.h"


def declared_functions():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mdfit_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_the_documented_entry_points():
    names = declared_functions()
    for required in ("mdfit_fit_batch", "mdfit_default_opts", "mdfit_last_error", "mdfit_abi_version"):
        assert required in names


def test_library_loads_and_exports_every_declared_symbol():
    from metadamage_amd import _lib

    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (mdfit_[a-z_0-9]+)", out))
    assert set(declared_functions()) <= exported
    assert set(_lib.EXPORTED_SYMBOLS) == set(declared_functions())


def test_abi_version_and_defaults_without_gpu():
    from metadamage_amd import _lib

    lib = _lib.load()
    assert lib.mdfit_abi_version() == _lib.ABI_VERSION
    o = _lib.default_opts()
    assert (o.mode, o.max_iter, o.tol_step) == (_lib.MODE_MAP, 200, 1e-9)
    assert (o.seed, o.num_warmup, o.num_samples, o.index_base) == (0, 500, 1000, 0)  # fits.py:792-799
    # the ctypes mirror of mdfit_opts has the C layout (int32, int32, double, uint64, int32, int32, int64)
    assert ctypes.sizeof(_lib.MdfitOpts) == 40
    # workspace: MAP = the per-XCD queue counters; NUTS adds 6 x S x 4 doubles of draws per taxon
    assert lib.mdfit_workspace_bytes(1000, None) >= 4 * 8
    nuts = _lib.default_opts(mode=_lib.MODE_NUTS, num_samples=100)
    assert lib.mdfit_workspace_bytes(1000, ctypes.byref(nuts)) == _lib.SAMPLES_OFFSET + 1000 * 6 * 100 * 4 * 8


def test_argument_errors_need_no_device():
    from metadamage_amd import _lib

    lib = _lib.load()
    assert lib.mdfit_fit_batch(None, None, None, -1, None, None, None, None, None, None) == -1
    assert b"n_taxa" in lib.mdfit_last_error()
    assert lib.mdfit_fit_batch(None, None, None, 0, None, None, None, None, None, None) == 0
    bad = _lib.default_opts(mode=7)
    dummy = ctypes.c_void_p(16)
    assert lib.mdfit_fit_batch(dummy, dummy, None, 1, ctypes.byref(bad), dummy, None, dummy, None, None) == -1


def test_record_layout_constants_match_header():
    from metadamage_amd import _lib

    text = HEADER.read_text()
    assert f"#define MDFIT_LD {_lib.LD}" in text
    assert f"#define MDFIT_NPOS {_lib.NPOS}" in text
    assert f"MDFIT_F_DIAG = {_lib.F_DIAG}" in text
    assert f"MDFIT_NOUT = {_lib.NOUT}" in text
    enum = re.search(r"enum mdfit_field \{(.*?)MDFIT_NRESULT", text, re.S).group(1)
    fields = re.findall(r"MDFIT_F_([A-Z0-9_]+)", enum)
    assert [f.lower() for f in fields] == [f.lower() for f in _lib.RESULT_FIELDS]


def test_ingest_library_exports_every_declared_symbol():
    """include/mdingest.h (native count reader + pipeline) against libmdingest.so."""
    from metadamage_amd import ingest

    text = re.sub(r"/\*.*?\*/", "", (ROOT / "include" / "mdingest.h").read_text(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(mdi_[a-z_0-9]+)\s*\(", text)))
    assert {"mdi_open", "mdi_parse_into", "mdi_select", "mdi_gather"} <= set(declared)
    lib = ingest._load()
    for name in declared:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(ingest.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    assert set(declared) <= set(re.findall(r"\bT (mdi_[a-z_0-9]+)", out))
