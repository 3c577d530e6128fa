"""GPU: the library's HIP-event profiling hooks (bench.py's kernel timing),
both modes: events around the call and the fit kernel, or the fit kernel only."""

from __future__ import annotations

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fit_only", [False, True])
def test_profile_hooks(fit_only):
    import torch

    from metadamage_amd import _lib, engine
    from metadamage_amd.synthetic import generate

    b = generate(200, seed=5)
    ty, tN, tm = engine.to_device_counts(b.y, b.N, b.mm)
    o = _lib.default_opts(mode=_lib.MODE_MAP)
    res = engine.alloc_outputs(200, opts=o)
    engine.fit_batch_device(ty, tN, tm, o, res)  # warm
    torch.cuda.synchronize()
    engine.profile_enable(True, fit_only=fit_only)
    try:
        for _ in range(3):
            engine.fit_batch_device(ty, tN, tm, o, res)
        call_ms, fit_ms, n = engine.profile_read()
    finally:
        engine.profile_enable(False)
    assert n == 3
    assert fit_ms > 0.0
    if fit_only:
        assert call_ms == -1.0
    else:
        assert call_ms >= fit_ms
    assert (res.status.cpu().numpy() == 0).all()
    # disabled: nothing recorded
    engine.fit_batch_device(ty, tN, tm, o, res)
    assert engine.profile_read()[2] == 0
