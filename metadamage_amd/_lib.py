"""ctypes binding of the engine's C-ABI (include/mdfit.h, libmdfit.so).

The shared library is built in-tree by __graft_entry__.build() (hipcc, gfx950)
and loaded from this package directory.  There is no fallback: if the library
or a GPU is missing, the product path raises.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libmdfit.so"

# mirrors of include/mdfit.h
ABI_VERSION = 2
NPOS = 30
NHALF = 15
LD = 32
NMM = 12
NPRED = 3
MODE_MAP = 0  # (MODE_NUTS below)
OK, MAXITER, NONFINITE, INVALID = 0, 1, 2, 3
NRESULT = 25
F_DIAG = 32
NOUT = 80
NSUBFIT = 6
DIAG_STRIDE = 8

# output record field order (enum mdfit_field) == fit_results numeric columns
RESULT_FIELDS = [
    "D_max",
    "n_sigma",
    "D_max_lower_hpdi",
    "D_max_upper_hpdi",
    "q_mean",
    "concentration_mean",
    "D_max_marginalized_mean",
    "N_z1_forward",
    "N_z1_reverse",
    "N_sum_forward",
    "N_sum_reverse",
    "N_sum_total",
    "y_sum_forward",
    "y_sum_reverse",
    "y_sum_total",
    "n_sigma_forward",
    "D_max_forward",
    "q_mean_forward",
    "n_sigma_reverse",
    "D_max_reverse",
    "q_mean_reverse",
    "asymmetry",
    "normalized_noise",
    "normalized_noise_forward",
    "normalized_noise_reverse",
]
SUBFITS = ["PMD", "null", "PMD_forward", "PMD_reverse", "null_forward", "null_reverse"]
DIAG_FIELDS = ["q", "A", "c", "phi", "objective", "evals", "status"]

# C-ABI symbols declared in include/mdfit.h
EXPORTED_SYMBOLS = [
    "mdfit_default_opts",
    "mdfit_fit_batch",
    "mdfit_workspace_bytes",
    "mdfit_noise",
    "mdfit_betabinom_logpmf",
    "mdfit_special",
    "mdfit_hpdi68",
    "mdfit_peak_probe",
    "mdfit_nuts_peak_probe",
    "mdfit_poison_lds",
    "mdfit_objective",
    "mdfit_nuts_potential",
    "mdfit_profile_enable",
    "mdfit_profile_read",
    "mdfit_last_error",
    "mdfit_abi_version",
]


class MdfitOpts(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int32),
        ("max_iter", ctypes.c_int32),
        ("tol_step", ctypes.c_double),
        ("seed", ctypes.c_uint64),
        ("num_warmup", ctypes.c_int32),
        ("num_samples", ctypes.c_int32),
        ("index_base", ctypes.c_int64),
    ]


MODE_MAP, MODE_NUTS = 0, 1
# MAP: below this many taxa per call the predictive HPDI streams beside the fit
# kernel; from it the workspace also holds the wide-window records
# (kStreamMaxTaxa, csrc/mdfit.hip)
STREAM_MAX_TAXA = 60_000
SAMPLES_OFFSET = 256  # NUTS workspace: double[T][6][S][4] draws after the queue counters


class MdfitError(RuntimeError):
    pass


_LIB = None


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load libmdfit.so (in-tree) and declare the C-ABI signatures."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise MdfitError(
            f"{p} not found: build the HIP extension first (python -c "
            "'import __graft_entry__ as g; g.build()')"
        )
    lib = ctypes.CDLL(str(p))
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    lib.mdfit_default_opts.argtypes = [ctypes.POINTER(MdfitOpts)]
    lib.mdfit_default_opts.restype = None
    lib.mdfit_fit_batch.argtypes = [vp, vp, vp, i64, ctypes.POINTER(MdfitOpts), vp, vp, vp, vp, vp]
    lib.mdfit_fit_batch.restype = ctypes.c_int
    lib.mdfit_workspace_bytes.argtypes = [i64, ctypes.c_void_p]
    if hasattr(lib, "mdfit_nuts_potential"):
        lib.mdfit_nuts_potential.argtypes = [vp, vp, vp, vp, vp, i64, vp, vp, vp]
        lib.mdfit_nuts_potential.restype = ctypes.c_int
    if hasattr(lib, "mdfit_profile_enable"):  # (absent from older dev builds loaded by tools/)
        lib.mdfit_profile_enable.argtypes = [ctypes.c_int]
        lib.mdfit_profile_enable.restype = ctypes.c_int
        lib.mdfit_profile_read.argtypes = [vp, vp, vp]
        lib.mdfit_profile_read.restype = ctypes.c_int
    lib.mdfit_workspace_bytes.restype = i64
    lib.mdfit_noise.argtypes = [vp, vp, vp, i64, vp, vp]
    lib.mdfit_noise.restype = ctypes.c_int
    lib.mdfit_betabinom_logpmf.argtypes = [vp, vp, vp, vp, i64, vp, vp, vp]
    lib.mdfit_betabinom_logpmf.restype = ctypes.c_int
    lib.mdfit_special.argtypes = [vp, i64, vp, vp]
    lib.mdfit_special.restype = ctypes.c_int
    lib.mdfit_hpdi68.argtypes = [vp, vp, vp, i64, vp, vp, vp]
    lib.mdfit_hpdi68.restype = ctypes.c_int
    lib.mdfit_peak_probe.argtypes = [i64, i32, vp, vp]
    lib.mdfit_peak_probe.restype = ctypes.c_int
    if hasattr(lib, "mdfit_poison_lds"):
        lib.mdfit_poison_lds.argtypes = [vp]
        lib.mdfit_poison_lds.restype = ctypes.c_int
    if hasattr(lib, "mdfit_nuts_peak_probe"):  # (absent from round-3 builds loaded by tools/ for A/B)
        lib.mdfit_nuts_peak_probe.argtypes = [i64, i32, vp, vp]
        lib.mdfit_nuts_peak_probe.restype = ctypes.c_int
    lib.mdfit_objective.argtypes = [vp, vp, vp, vp, vp, i64, vp, vp, vp, vp, vp]
    lib.mdfit_objective.restype = ctypes.c_int
    lib.mdfit_last_error.argtypes = []
    lib.mdfit_last_error.restype = ctypes.c_char_p
    lib.mdfit_abi_version.argtypes = []
    lib.mdfit_abi_version.restype = ctypes.c_int
    if lib.mdfit_abi_version() != ABI_VERSION:
        raise MdfitError(f"ABI mismatch: library {lib.mdfit_abi_version()} != {ABI_VERSION}")
    if path is None:
        _LIB = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().mdfit_last_error().decode(errors="replace")
        raise MdfitError(f"mdfit call failed (rc={rc}): {msg}")


def default_opts(**overrides) -> MdfitOpts:
    o = MdfitOpts()
    load().mdfit_default_opts(ctypes.byref(o))
    for k, v in overrides.items():
        setattr(o, k, v)
    return o
