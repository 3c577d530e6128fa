"""Per-file driver (mirror of /root/reference/metadamage/main.py:28-74).

For every input file: validate, load (or compute) the counts table with the
frozen cuts, then get_fits.  The reference ran the files one after another and
dispatched each file's fits to a process pool; here

  * the stages of consecutive files overlap: reader threads ingest files
    i+1 and i+2 and pack them for the fit (the native reader releases the
    GIL) while file i is fitted, and the parquet writes (counts, fit_results, fit_predictions) run
    on writer threads (pyarrow releases the GIL while encoding);
  * in a multi-GPU job (torch.distributed initialised) with at least as many
    files as ranks, whole files are dealt round-robin to the ranks and each
    rank fits its files on its own GPU -- no collective, nothing replicated;
    with fewer files than ranks every rank reads every file and the taxa of
    each are sharded over the ranks (fits.fit_packed, one RCCL gather).
"""

from __future__ import annotations

import copy
import logging
from collections import deque
from concurrent.futures import Future, ThreadPoolExecutor

from . import counts, fits, utils

logger = logging.getLogger(__name__)

N_WRITERS = 3
# files read ahead of the one being fitted, each on its own reader thread: the
# count ingest of one file (~0.2 s on a 16-core share) has serial stretches
# (the cut + sort, the categoricals) that a second file's parse fills
N_READERS = 2


def _world():
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return 1, 0
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


class _Writer:
    """Executor front that remembers its futures so main() can surface a
    failed write."""

    def __init__(self, pool):
        self.pool = pool
        self.futures = []

    def submit(self, fn, *args):
        self.futures.append(self.pool.submit(fn, *args))

    def drain(self):
        for f in self.futures:
            f.result()
        self.futures.clear()


def _load(filename, cfg, writer, save=True):
    """Reader thread: the counts table of one file, then the host work of its
    fit ahead of the device call (fits.prepare_fits: top-N, packing)."""
    cfg_f = copy.copy(cfg)
    cfg_f.add_filename(filename)
    df_counts = counts.load_counts(cfg_f, writer=writer, save=save)
    packed = fits.prepare_fits(df_counts, cfg_f) if len(df_counts) > 0 else None
    return cfg_f, df_counts, packed


def main(filenames, cfg, opts=None):
    """Fit every file; returns {shortname: (df_fit_results, df_fit_predictions)}
    for the files this rank fitted (rank 0 holds the gathered frames of
    taxon-sharded files)."""
    N_files = len(filenames)
    valid = [f for f in filenames if utils.file_is_valid(f)]
    if N_files and not valid:
        raise Exception("All files were bad!")
    world, rank = _world()
    shard_files = world > 1 and len(valid) >= world
    mine = valid[rank::world] if shard_files else valid
    # taxon-sharded files are read by every rank (each packs its own shard);
    # only rank 0 writes their counts parquet (atomically, io.Parquet.save)
    save = shard_files or rank == 0
    results = {}
    with ThreadPoolExecutor(N_READERS) as reader, ThreadPoolExecutor(N_WRITERS) as pool:
        writer = _Writer(pool)
        ahead = deque(reader.submit(_load, f, cfg, writer, save) for f in mine[:N_READERS])
        for i in range(len(mine)):
            cfg_f, df_counts, packed = ahead.popleft().result()
            if i + N_READERS < len(mine):
                ahead.append(reader.submit(_load, mine[i + N_READERS], cfg, writer, save))
            cfg.add_filename(cfg_f.filename)  # the caller's cfg follows the files as in the reference
            cfg.N_tax_ids, cfg.N_fits = getattr(cfg_f, "N_tax_ids", None), cfg_f.N_fits
            accepted = utils.is_df_counts_accepted(df_counts, cfg_f)
            if not shard_files:  # every rank must skip (or fit) the file together
                from .distributed import all_ranks_agree

                accepted = all_ranks_agree(accepted)
            if not accepted:
                if packed is not None:
                    packed.release_pinned()
                continue
            try:
                r = fits.get_fits(df_counts, cfg_f, opts=opts, shard=not shard_files, writer=writer, packed=packed,
                                  deferred=True)
            finally:
                if packed is not None:  # (a cache hit never fits it; a failed fit returns it too)
                    packed.release_pinned()
            # the frames are built (and their saves submitted) on a writer
            # thread while the next file fits
            results[cfg_f.shortname] = pool.submit(r) if callable(r) else r
            logger.debug("End of loop\n")
        results = {k: (v.result() if isinstance(v, Future) else v) for k, v in results.items()}
        writer.drain()
    return results
