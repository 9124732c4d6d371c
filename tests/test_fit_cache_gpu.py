"""rs_svd_fit keeps its plan per ctx and reuses it for the same ratings (exact COO comparison):
a refit of the same TrainSet skips the CSR and tile-schedule build, a different TrainSet rebuilds.
core/svd.go:63-132 semantics are unchanged either way (checked by training error on each set)."""
import numpy as np
import pytest

import oracle as O
import rsgpu
from rsgpu import synth

pytestmark = pytest.mark.gpu


def _train_rmse(u, i, r, m):
    return float(np.sqrt(np.mean((O.svd_predict(u, i, *m) - r) ** 2)))


def test_refit_same_and_other_trainset(ctx):
    a = synth.small_like(800, 400, 40000, seed=2)
    b = synth.small_like(800, 400, 40000, seed=3)
    k = 32
    rng = np.random.default_rng(0)
    P0, Q0 = rng.normal(0, 0.1, (800, k)), rng.normal(0, 0.1, (400, k))
    errs = {}
    for name, (u, i, r, nu, ni) in (("a", a), ("a2", a), ("b", b), ("a3", a)):
        m = ctx.svd_fit(rsgpu.Ratings(u, i, r, nu, ni), P0, Q0, n_epochs=10)
        assert all(np.all(np.isfinite(x)) for x in m[:4])
        errs[name] = _train_rmse(u, i, r, m)
    # the refits of a train as well as the first fit; b (a different set) trains on its own ratings
    assert abs(errs["a2"] - errs["a"]) < 0.01 and abs(errs["a3"] - errs["a"]) < 0.01, errs
    mb = ctx.svd_fit(rsgpu.Ratings(*b), P0, Q0, n_epochs=0)
    assert errs["b"] < _train_rmse(b[0], b[1], b[2], mb) - 0.1, errs


def test_changed_rating_rebuilds(ctx):
    u, i, r, nu, ni = synth.small_like(500, 300, 20000, seed=5)
    k = 16
    rng = np.random.default_rng(1)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    ctx.svd_fit(rsgpu.Ratings(u, i, r, nu, ni), P0, Q0, n_epochs=5)
    r2 = r.copy()
    r2[:] = 5.0  # same ids, all ratings changed: a stale plan would train towards the old ratings
    m = ctx.svd_fit(rsgpu.Ratings(u, i, r2, nu, ni), P0, Q0, n_epochs=20)
    pred = O.svd_predict(u, i, *m)
    assert abs(float(np.mean(pred)) - 5.0) < 0.05
