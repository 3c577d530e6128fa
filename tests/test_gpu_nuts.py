"""GPU parity of the sampling mode (MDFIT-NUTS v1) against the CPU oracle.

The kernel draws the oracle's Philox numbers in the oracle's order, so short
chains reproduce the oracle draw for draw; over the reference's full 500 + 1000
iterations the step-size adaptation amplifies the ~1e-9 differences of the
lnGamma sums (|U| ~ 1e7) until a decision flips, so full-length parity is
distributional (posterior means within Monte-Carlo error).
"""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def nuts_engine():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    from metadamage_amd import engine

    return engine


def _run(engine, b, warmup, samples, index_base=0, keep=False):
    import torch

    from metadamage_amd import _lib

    opts = _lib.default_opts(mode=_lib.MODE_NUTS, num_warmup=warmup, num_samples=samples, index_base=index_base)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    res = engine.alloc_outputs(len(b.y), opts=opts)
    engine.fit_batch_device(ty, tN, tm, opts, res)
    torch.cuda.synchronize()
    out = (res.out.cpu().numpy(), res.pred.cpu().numpy(), res.status.cpu().numpy())
    if keep:
        out = out + (engine.samples_view(res, len(b.y), opts).cpu().numpy(),)
    return out


def test_potential_matches_oracle(nuts_engine, oracle_lib):
    from metadamage_amd.synthetic import generate

    b = generate(40, seed=3)
    rng = np.random.default_rng(0)
    items = [(t, m, s) for t in range(40) for m in (0, 1) for s in (0, 1, 2)]
    model = np.array([m for _, m, _ in items])
    subset = np.array([s for _, _, s in items])
    y = b.y[[t for t, _, _ in items]]
    N = b.N[[t for t, _, _ in items]]
    v = rng.uniform(-2, 2, (len(items), 4))
    v[model == 1, 1:3] = 0
    v[5] = [0.0, 3.0, 3.0, 5.0]  # infeasible A + c >= 1
    U, g = nuts_engine.nuts_potential(model, subset, y, N, v)
    for k, (t, m, s) in enumerate(items):
        Uo, go = oracle_lib.nuts_potential(m, s, y[k, :30], N[k, :30], v[k])
        if not np.isfinite(Uo):
            assert U[k] == np.inf and (g[k] == 0).all()
            continue
        assert abs(U[k] - Uo) <= 1e-13 * abs(Uo) + 1e-9, (k, U[k], Uo)
        assert np.abs(g[k] - go).max() <= 1e-9 * max(1.0, np.abs(go).max()), (k, g[k], go)


def test_short_chains_follow_the_oracle_draw_for_draw(nuts_engine, oracle_lib):
    from metadamage_amd.synthetic import generate

    b = generate(32, seed=2)
    out, pred, st, smp = _run(nuts_engine, b, 1, 100, keep=True)
    ro, rp, rs, rsmp = oracle_lib.nuts_batch(b.y, b.N, b.mm, num_warmup=1, num_samples=100, threads=8,
                                             keep_samples=True)
    assert (st == 0).all() and (rs == 0).all()
    d = np.abs(smp - rsmp).max(axis=(2, 3))  # [T, 6]
    assert (d < 1e-6).mean() >= 0.95, d
    same = (d < 1e-6).all(1)
    rel = np.abs(out[same, :25] - ro[same, :25]) / np.maximum(np.abs(ro[same, :25]), 1e-2)
    assert np.nanmax(rel) < 1e-6, np.nanmax(rel, 0)
    # diagnostics: the adapted step size (exp of the dual-averaging mean, which
    # amplifies the ~1e-9 energy differences) and the leapfrog counts
    np.testing.assert_allclose(out[same, 36::8][:, :6], ro[same, 36::8][:, :6], rtol=1e-6)
    # (a tree may stop one doubling apart and still pick the same draw: a few
    # iterations of a few chains, by up to a depth-4 doubling's 16 leaves in
    # one of the 100 iterations)
    dl = np.abs(out[same, 37::8][:, :6] - ro[same, 37::8][:, :6])
    assert dl.max() <= 0.16 + 1e-9, dl.max()
    assert (dl > 1e-9).mean() <= 0.05, (dl > 1e-9).mean()


def test_register_sort_path_follows_the_oracle(nuts_engine, oracle_lib):
    """600 draws: the post kernel sorts the predictive counts in registers
    (513..1024 draws; 100 take the LDS sort above).  Chains that match the
    oracle draw for draw must give its records -- predictive medians, HPDI
    bounds and WAIC columns -- to 1e-6."""
    from metadamage_amd.synthetic import generate

    b = generate(16, seed=5)
    out, pred, st, smp = _run(nuts_engine, b, 1, 600, keep=True)
    ro, rp, rs, rsmp = oracle_lib.nuts_batch(b.y, b.N, b.mm, num_warmup=1, num_samples=600, threads=8,
                                             keep_samples=True)
    assert (st == 0).all() and (rs == 0).all()
    same = (np.abs(smp - rsmp).max(axis=(2, 3)) < 1e-6).all(1)
    assert same.mean() >= 0.5, same.mean()
    rel = np.abs(out[same, :25] - ro[same, :25]) / np.maximum(np.abs(ro[same, :25]), 1e-2)
    assert np.nanmax(rel) < 1e-6, np.nanmax(rel, 0)
    prel = np.abs(pred[same] - rp[same]) / np.maximum(np.abs(rp[same]), 1e-2)
    assert np.nanmax(prel) < 1e-6, np.nanmax(prel)


def _mcse(x, nb=20):
    m = x.shape[-1] // nb
    bm = x[..., : m * nb].reshape(x.shape[:-1] + (nb, m)).mean(-1)
    return bm.std(-1, ddof=1) / np.sqrt(nb)


def test_full_length_chains_agree_in_distribution(nuts_engine, oracle_lib):
    """The reference's settings (500 warmup, 1000 draws): posterior means of
    every parameter of every sub-fit agree with the oracle's within Monte-Carlo
    error (batch-means MCSE of both chains)."""
    from metadamage_amd.synthetic import generate

    b = generate(48, seed=4)
    out, pred, st, smp = _run(nuts_engine, b, 500, 1000, keep=True)
    ro, rp, rs, rsmp = oracle_lib.nuts_batch(b.y, b.N, b.mm, threads=8, keep_samples=True)
    assert (st == 0).all() and (rs == 0).all()
    zs = []
    for s in range(6):
        for j in ((0, 1, 2, 3) if s in (0, 2, 3) else (0, 3)):
            a, r = smp[:, s, :, j], rsmp[:, s, :, j]
            se = np.hypot(_mcse(a), _mcse(r))
            zs.append(np.abs(a.mean(1) - r.mean(1)) / np.maximum(se, 1e-300))
    z = np.concatenate(zs)
    assert np.median(z) < 1.2, np.median(z)
    assert (z > 5).mean() < 0.03, np.sort(z)[-10:]
    # adapted step sizes: chain-to-chain scatter of dual averaging (~10-30 %),
    # no systematic offset
    lr = np.log(out[:, 36::8][:, :6] / ro[:, 36::8][:, :6])
    assert abs(np.median(lr)) < 0.1 and np.median(np.abs(lr)) < 0.3


def test_sampling_is_deterministic_and_keyed_by_index_base(nuts_engine):
    from metadamage_amd.synthetic import generate

    b = generate(8, seed=6)
    a = _run(nuts_engine, b, 60, 80)
    c = _run(nuts_engine, b, 60, 80)
    np.testing.assert_array_equal(a[0], c[0])
    np.testing.assert_array_equal(a[1], c[1])

    class Part:
        y, N, mm = b.y[3:], b.N[3:], b.mm[3:]

    p = _run(nuts_engine, Part, 60, 80, index_base=3)
    np.testing.assert_array_equal(a[0][3:], p[0])


def test_records_do_not_depend_on_which_wave_runs_a_chain(nuts_engine, monkeypatch):
    """The chain kernel's scheduling -- per-XCD queues, stealing across them,
    the long-chain issue priority -- decides only which wave runs a chain and
    when: the streams are keyed by (taxon, sub-fit), so a grid of 1 wave per CU
    (every wave runs many chains, the queues drain in another order) gives the
    default grid's records bit for bit."""
    from metadamage_amd.synthetic import generate

    b = generate(600, seed=9)
    a = _run(nuts_engine, b, 40, 60)
    monkeypatch.setenv("MDFIT_DEV_PER_CU", "1")
    c = _run(nuts_engine, b, 40, 60)
    for x, y in zip(a, c):
        np.testing.assert_array_equal(x.view(np.uint8), y.view(np.uint8))


def test_invalid_and_empty_positions(nuts_engine):
    from metadamage_amd.synthetic import generate

    b = generate(4, seed=8)
    b.y[1, 3] = b.N[1, 3] + 1  # y > N -> status 3
    b.N[2, 5] = 0
    b.y[2, 5] = 0  # N = 0 -> NaN predictions there (0/0 draws)
    out, pred, st = _run(nuts_engine, b, 30, 50)
    assert st[1] == 3 and np.isnan(out[1]).all()
    assert st[0] == 0 and st[2] == 0
    assert np.isnan(pred[2, :, 5]).all() and np.isfinite(pred[2, :, 4]).all()
    assert np.isfinite(out[2, :22]).all()
