"""GPU tests of K2's tile schedule (RS_PP_SCHED_TILE, csrc/svdpp_tile.hip): SVD++ (core/svd.go:316-427) with
K1's user tiles, one q_i atomic row per (item, tile) run and the y rows moved once per epoch by composed maps.

  * One workgroup of one wave trains the ratings in the schedule's visit order, which rs_svdpp_tile_order
    exports: the result equals the oracle's restatement of that order (or_svdpp_fit_tiles) within fp32 and
    2^-24 fixed-point rounding (TOL).
  * On the ML-100K fold and the configs[2] shape (ML-1M, k = 128) the library's launch (Hogwild over the
    waves and workgroups) reaches the held-out RMSE of the sequential restatements within 0.005 -- the bound
    test_svdpp_gpu.py / test_configs_gpu.py hold the user-major kernel to.

SVD++ parity is unpinned by the reference (core/base_test.go:38-40 is commented out): the checks are against
the oracle's fp64 restatements."""
import numpy as np
import pytest

import oracle as O
import rsgpu
from helpers import folds, rmse
from rsgpu import synth

pytestmark = pytest.mark.gpu
TOL = 2e-4


def _maxdiff(a, b):
    return max(float(np.max(np.abs(np.asarray(x) - np.asarray(y)))) for x, y in zip(a, b))


def _data(nu=200, ni=150, n=4000, seed=3):
    rng = np.random.default_rng(seed)
    pairs = np.unique(np.stack([rng.integers(0, nu, 3 * n), (rng.zipf(1.6, 3 * n) - 1) % ni]), axis=1)
    pairs = pairs[:, rng.permutation(pairs.shape[1])[:n]]
    u, i = pairs[0], pairs[1]
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    return u, i, rng.integers(1, 6, len(u)).astype(float), nu, ni


@pytest.fixture
def tile_ctx(ctx):
    yield ctx
    ctx.svdpp_set_schedule(rsgpu.PP_SCHED_AUTO, 0, 16)


@pytest.mark.parametrize("k,epochs", [(8, 1), (8, 3), (100, 2)])
def test_svdpp_tile_one_wave_equals_restatement(tile_ctx, k, epochs):
    ctx = tile_ctx
    u, i, r, nu, ni = _data()
    R = rsgpu.Ratings(u, i, r, nu, ni)
    rng = np.random.default_rng(k)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
    ctx.svdpp_set_schedule(rsgpu.PP_SCHED_TILE, 1, 1)
    got = ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=epochs)
    assert ctx.svdpp_schedule_used() == rsgpu.PP_SCHED_TILE
    pos, run_off, tile_off = ctx.svdpp_tile_order(R, k, 1, 1)
    assert len(tile_off) > 2  # several tiles: the tile-local GlobalBias and the y moves between tiles
    assert np.array_equal(np.sort(pos), np.arange(len(r)))
    rowptr, items, rr = O.csr_by(u, nu, i, r)
    ref = O.svdpp_fit_tiles(rowptr, items, rr, pos, run_off, tile_off, P0, Q0, Y0, epochs=epochs)
    d = _maxdiff(ref[:5], got[:5])
    print(f"k={k} epochs={epochs}: max |gpu - restatement| {d:.2e}, GlobalBias {abs(ref[5] - got[5]):.2e}")
    assert d <= TOL
    assert abs(ref[5] - got[5]) <= TOL
    # the user-major schedule is another visit order: the results differ beyond the rounding
    usr = O.svdpp_fit_lazy(rowptr, items, rr, P0, Q0, Y0, epochs=epochs)
    assert _maxdiff(usr[:3], got[:3]) > 10 * TOL


def test_svdpp_tile_schedule_falls_back_for_wide_rows(tile_ctx):
    """A user whose row does not fit one tile's LDS: the user-major kernel runs instead."""
    ctx = tile_ctx
    k = 8
    n = 12000
    u = np.zeros(n, np.int64)
    i = np.arange(n)
    r = np.random.default_rng(0).integers(1, 6, n).astype(float)
    R = rsgpu.Ratings(u, i, r, 1, n)
    rng = np.random.default_rng(1)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (1, n, n))
    ctx.svdpp_set_schedule(rsgpu.PP_SCHED_TILE, 0, 16)
    got = ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=1)
    assert ctx.svdpp_schedule_used() == rsgpu.PP_SCHED_USER
    assert all(np.all(np.isfinite(x)) for x in got[:5])
    with pytest.raises(rsgpu.RsError):
        ctx.svdpp_tile_order(R, k, 0, 16)


def test_svdpp_tile_rmse_near_literal(tile_ctx, ml100k):
    """ML-100K fold 1, defaults (k = 20, 20 epochs, lr 0.007, reg 0.02): the library's tile launch against the
    literal reference order (test_svdpp_gpu.py's bound for the user-major kernel)."""
    ctx = tile_ctx
    f, k = folds(*ml100k)[0], 20
    rng = np.random.default_rng(4)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (f.nu, f.ni, f.ni))
    a = O.svdpp_fit(f.iu, f.ii, f.r, f.nu, P0, Q0, Y0)
    ref = rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *a), f.te_r)
    ctx.svdpp_set_schedule(rsgpu.PP_SCHED_TILE, 0, 16)
    b = ctx.svdpp_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, Y0)
    assert ctx.svdpp_schedule_used() == rsgpu.PP_SCHED_TILE
    got = rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *b), f.te_r)
    print(f"ML-100K fold 1: tile {got:.4f}, literal {ref:.4f}")
    assert abs(got - ref) <= 0.005, (got, ref)


@pytest.mark.timeout(300)
def test_svdpp_tile_config2_k128_ml1m(tile_ctx):
    """configs[2] (ML-1M shape, k = 128, 20 epochs): held-out RMSE within 0.005 of the user-major restatement
    (test_configs_gpu.py's bound), and the epoch time of both schedules printed."""
    ctx = tile_ctx
    u, i, r, nu, ni = synth.ml1m_like()
    n = len(r)
    te = np.zeros(n, bool)
    te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
    tr = ~te
    k = 128
    rng = np.random.default_rng(3)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
    R = rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni)
    out = {}
    for name, sched in (("tile", rsgpu.PP_SCHED_TILE), ("user", rsgpu.PP_SCHED_USER)):
        ctx.svdpp_set_schedule(sched, 0, 16)
        got = ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=20)
        assert ctx.svdpp_schedule_used() == sched
        ms = ctx.last_kernel_ms() / 20
        assert all(np.all(np.isfinite(x)) for x in got[:5]) and np.isfinite(got[5])
        out[name] = rmse(O.svdpp_predict(u[tr], i[tr], nu, u[te], i[te], *got), r[te])
        print(f"config2 {name}: {ms:.3f} ms per epoch, held-out RMSE {out[name]:.4f}", flush=True)
    rowptr, items, rr = O.csr_by(u[tr], nu, i[tr], r[tr])
    ref = O.svdpp_fit_lazy(rowptr, items, rr, P0, Q0, Y0, epochs=20)
    e_ref = rmse(O.svdpp_predict(u[tr], i[tr], nu, u[te], i[te], *ref), r[te])
    print(f"config2: oracle (user-major restatement) {e_ref:.4f}", flush=True)
    assert abs(out["tile"] - e_ref) <= 0.005, (out, e_ref)
