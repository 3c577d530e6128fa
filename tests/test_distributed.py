"""CPU tests of the multi-GPU path with the gloo backend (world size 2 and 3):
contiguous taxon shards + the single gather of packed result records.  The
per-shard fit is done by the CPU oracle here (a stand-in for the kernel; the
GPU runs the same code path with the nccl/RCCL backend)."""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from metadamage_amd.distributed import (FLOAT_COLS, INT_HI, INT_LO, NRES_GATHER, REC_BYTES, alloc_records,
                                        gather_records, round_like_gather, shard_capacity, shard_range,
                                        unpack_gathered)


def test_shard_ranges_cover_in_order():
    for T in (0, 1, 2, 7, 10, 10_001):
        for world in (1, 2, 3, 8):
            spans = [shard_range(T, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == T
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and a <= b
            assert all(b - a <= shard_capacity(T, world) for a, b in spans)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, T, q, async_op=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from metadamage_amd.synthetic import generate
        from oracle.oracle import OracleLib

        b = generate(T, seed=8)
        lo, hi = shard_range(T, rank, world)
        cap = shard_capacity(T, world)
        rec = alloc_records(cap, "cpu")
        rec.buf.zero_()
        rec.out.zero_()
        if hi > lo:
            o, p, s = OracleLib().fit_batch(b.y[lo:hi], b.N[lo:hi], b.mm[lo:hi], threads=1)
            rec.out[: hi - lo] = torch.from_numpy(o)
            rec.pred[: hi - lo] = torch.from_numpy(p)
            rec.status[: hi - lo] = torch.from_numpy(s)
        if async_op:
            # bench.py's double-buffered steps: the gather of one batch is in
            # flight while the next batch is written into a second record set
            parts, work = gather_records(rec.stage(), cap, rank, world, async_op=True)
            rec2 = alloc_records(cap, "cpu")
            rec2.buf.copy_(rec.buf)
            rec2.out.copy_(rec.out)
            parts2, work2 = gather_records(rec2.stage(), cap, rank, world, async_op=True)
            work2.wait()
            work.wait()
            if rank == 0:
                for a, b2 in zip(parts, parts2):
                    assert torch.equal(a, b2)
        else:
            parts = gather_records(rec.stage(), cap, rank, world)
        if rank == 0:
            q.put(unpack_gathered(parts, T, world))
        else:
            assert parts is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,T,async_op", [(2, 37, False), (3, 20, False), (2, 1, False), (2, 37, True)])
def test_gloo_shard_and_gather_reproduce_single_process(world, T, async_op):
    from metadamage_amd.synthetic import generate
    from oracle.oracle import OracleLib

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, T, q, async_op)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b = generate(T, seed=8)
    o, pr, s = OracleLib().fit_batch(b.y, b.N, b.mm, threads=1)
    # the diagnostic columns stay on the fitting rank: the 25 result columns
    # only, the non-count ones rounded to f32 as the frames store them
    assert got[0].shape == (T, NRES_GATHER)
    np.testing.assert_array_equal(got[0], round_like_gather(o))
    np.testing.assert_array_equal(got[1], pr)
    np.testing.assert_array_equal(got[2], s)


def _c4_worker(rank, world, port, total, share, q):
    """bench.py's C4 step at world size `world` on gloo: this rank's C4 rows
    (bench.c4_rows), the fit (the CPU oracle standing in for the kernel),
    stage, the one gather, unpack on rank 0."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from metadamage_amd.synthetic import generate
        from oracle.oracle import OracleLib

        b = generate(share, seed=3)
        lo, hi, rows = bench.c4_rows(rank, world, total=total, share=share)
        cap = shard_capacity(total, world)
        rec = alloc_records(cap, "cpu")
        rec.buf.zero_()
        rec.out.zero_()
        if hi > lo:
            o, p, s = OracleLib().fit_batch(b.y[rows], b.N[rows], b.mm[rows], threads=1)
            rec.out[: hi - lo] = torch.from_numpy(o)
            rec.pred[: hi - lo] = torch.from_numpy(p)
            rec.status[: hi - lo] = torch.from_numpy(s)
        parts = gather_records(rec.stage(), cap, rank, world)
        if rank == 0:
            q.put(unpack_gathered(parts, total, world))
        else:
            assert parts is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,share", [(8, 64, 16), (8, 61, 16), (4, 64, 16)])
def test_bench_c4_step_rehearsal(world, total, share):
    """The C4 bench step (shard -> stage -> gather -> unpack) at 8 ranks on
    gloo reproduces the one-process fit of the same global taxa (global taxon
    i = share row i % share, what c4_one_gpu fits), ragged totals included."""
    import bench
    from metadamage_amd.synthetic import generate
    from oracle.oracle import OracleLib

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, total, share, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, _, rows = bench.c4_rows(0, 1, total=total, share=share)
    assert rows.size == total and (rows == np.arange(total) % share).all()
    b = generate(share, seed=3)
    o, pr, s = OracleLib().fit_batch(b.y[rows], b.N[rows], b.mm[rows], threads=1)
    np.testing.assert_array_equal(got[0], round_like_gather(o))
    np.testing.assert_array_equal(got[1], pr)
    np.testing.assert_array_equal(got[2], s)


@pytest.mark.parametrize("n", [5, 6])
def test_record_views_layout(n):
    rec = alloc_records(n, "cpu")
    assert REC_BYTES == 496 and rec.buf.numel() == n * REC_BYTES
    assert rec.out.shape == (n, 80) and rec.ints.shape == (n, INT_HI - INT_LO)
    assert rec.floats.shape == (n, len(FLOAT_COLS)) and len(FLOAT_COLS) + INT_HI - INT_LO == NRES_GATHER
    assert rec.pred.shape == (n, 3, 30) and rec.status.shape == (n,)
    for t in (rec.ints, rec.floats, rec.pred, rec.status):
        assert t.is_contiguous()
    assert rec.ints.data_ptr() == rec.buf.data_ptr()
    assert rec.floats.data_ptr() - rec.buf.data_ptr() == n * 8 * 8
    assert rec.pred.data_ptr() - rec.floats.data_ptr() == n * 17 * 4
    assert rec.status.data_ptr() - rec.pred.data_ptr() == n * 360
    g = torch.Generator().manual_seed(n)
    rec.out.copy_(torch.rand((n, 80), generator=g, dtype=torch.float64) * 1e3)
    rec.out[:, INT_LO:INT_HI] = torch.randint(0, 2**32, (n, INT_HI - INT_LO), generator=g).double()
    rec.out[0, 0] = float("nan")
    rec.stage()
    rec.pred.zero_()
    rec.status.zero_()
    got, _, _ = unpack_gathered([rec.buf], n, 1)
    np.testing.assert_array_equal(got, round_like_gather(rec.out.numpy()))
    # the counts exact, the rest as the frames' float32 cast rounds them
    np.testing.assert_array_equal(got[:, INT_LO:INT_HI], rec.out[:, INT_LO:INT_HI].numpy())
    np.testing.assert_array_equal(got[:, FLOAT_COLS].astype(np.float32),
                                  rec.out.numpy()[:, FLOAT_COLS].astype(np.float32))


def _failing_worker(rank, world, port, q):
    """The `metadamage fit` wrapper (distributed.run_distributed) where rank 1
    raises before the collective rank 0 is about to enter."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    from metadamage_amd.distributed import all_ranks_agree, init_from_env, run_distributed

    init_from_env_gloo = lambda: init_from_env("gloo")  # noqa: E731

    def body():
        if rank == 1:
            raise RuntimeError("bad input file on rank 1")
        return all_ranks_agree(True)  # rank 0 waits here for its peer

    import metadamage_amd.distributed as d

    d.init_from_env = init_from_env_gloo  # CPU test: gloo instead of RCCL
    try:
        run_distributed(body)
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, type(e).__name__))


def test_a_failing_rank_does_not_hang_the_job():
    """a rank that raises leaves the group without a barrier, so
    the healthy rank's pending collective fails instead of pairing with it and
    hanging; both processes exit promptly."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=90)
    alive = [p.is_alive() for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not any(alive), "a rank is still waiting in a collective"
    got = dict(q.get(timeout=5) for _ in range(2))
    assert got[1] == "RuntimeError"
    assert got[0] != "ok"  # the healthy rank's collective failed (peer gone) rather than completing
