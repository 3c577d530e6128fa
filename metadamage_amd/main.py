"""Per-file driver (mirror of /root/reference/metadamage/main.py:28-74).

For every input file: validate, load (or compute) the counts table with the
frozen cuts, then get_fits.  The reference dispatched fits to a process pool
per file; here get_fits issues one batched GPU call (sharded over ranks when
torch.distributed is initialised).
"""

from __future__ import annotations

import logging

from . import counts, fits, utils

logger = logging.getLogger(__name__)


def main(filenames, cfg, opts=None):
    N_files = len(filenames)
    bad_files = 0
    results = {}
    for filename in filenames:
        if not utils.file_is_valid(filename):
            bad_files += 1
            continue
        cfg.add_filename(filename)
        df_counts = counts.load_counts(cfg)
        if not utils.is_df_counts_accepted(df_counts, cfg):
            continue
        results[cfg.shortname] = fits.get_fits(df_counts, cfg, opts=opts)
        logger.debug("End of loop\n")
    if bad_files == N_files:
        raise Exception("All files were bad!")
    return results
