"""metadamage_amd — MI355X-native per-TaxID ancient-DNA damage fits.

A drop-in for the fits.py hot path of genomewalker/metadamage: the per-taxon
beta-binomial / exponential-decay damage model is fitted for a whole batch of
taxa by hand-written HIP kernels (metadamage_amd/csrc/mdfit.hip) behind a C-ABI
(include/mdfit.h).  Host modules mirror the reference's operator interface:
counts.load_counts, fits.get_fits / compute_fits, io.Parquet, utils.Config,
main.main and the `metadamage fit` CLI.
"""

from .__version__ import __version__  # noqa: F401
