"""FAST SVD / SVD++ on rating scales other than stars (VERDICT r4 #2 / advisor r4).

The reference keeps its biases and factors in unbounded float64 (core/svd.go:105-128, 316-427) and its
loader takes any rating (core/data.go:302-304).  The FAST kernels hold P / Q / Y as int32 fixed point
while a call runs; the scale now follows the ratings' spread (sgd_plan.hpp fx_shift_for: 2^-24 and
|v| < 128 on stars, 2^-20 and |v| < 2048 for 1-100 ratings), and so does the divergence guard's range
bound (a quarter of the range).  These tests run ML-100K (core/base_test.go's data) rescaled to 1-100
(x 20) and to -10..10 ((r - 3) x 5) against the fp64 restatement on the same scaled data:

* RMSE within 0.003 x scale (P2 in the scale's own units: the star-scale bound times the factor the
  ratings were stretched by) of a sequential restatement (see each test for which order);
* one wave exact to the scaled 1e-5 contract on 1-100 ratings (the fixed point at 2^-20);
* no divergence-guard refit and no RS_ERR_NUMERIC.

Learning rates: the reference itself diverges on 1-100 ratings at its default lr = 0.005 (NaN after
20 epochs in the restatement), so the x20 runs use lr = 0.0005 (SVD) / 1e-4 (SVD++), at which it
trains (held-out RMSE 18.6 and 19.3 on the 1-100 scale); the SVD++ -10..10 runs use 1e-3 for the same
reason (default 0.007 diverges there too).
"""
import numpy as np
import pytest

import oracle as O
import rsgpu
from helpers import folds, rmse

pytestmark = pytest.mark.gpu

SCALES = {"x20": (lambda r: 20.0 * r, 20.0), "pm10": (lambda r: (r - 3.0) * 5.0, 5.0)}
SVD_LR = {"x20": 0.0005, "pm10": 0.005}
PP_LR = {"x20": 1e-4, "pm10": 1e-3}


@pytest.fixture(scope="module")
def scaled(ml100k):
    U, I, R = ml100k
    return {name: folds(U, I, f(np.asarray(R, np.float64))) for name, (f, _) in SCALES.items()}


@pytest.mark.parametrize("scale", sorted(SCALES))
def test_svd_fast_on_rating_scale(ctx, scaled, scale):
    """5-fold, k = 100, 20 epochs: no refit, no error, and within 0.003 x scale (P2 in the scale's units) of the
    reference visit order (or_svd_fit: svd.go:92-130 over the TrainSet in data order), and within the
    base_test.go:34-36 bound in star units where the reference order itself meets it (on -10..10 at lr 0.005 it
    lands at 5.20, 1.04 in star units, on its own).

    Round 5 measured 18.741 at x20 against the reference order's 18.649 (0.0046 in star units).  The gap was the
    GlobalBias fold, not the visit order: the per-stream chains folded by the mean of their moves advance
    GlobalBias by about one stream's ~30 ratings per epoch, so at lr 0.0005 it lagged the biases; the sequential
    chain converges within 1 / lr ratings.  The single-GPU epoch now folds the chains smoothed (sgd_tile.hip
    header; the oracle's or_svd_fit_works2 compose = 2 restates it): on the CPU with 2816 streams in random
    order, x20 0.93679 -> 0.93347 star units against 0.93243 for the reference, stars 0.93687 -> 0.93650
    against 0.93675."""
    k, lr, mult = 100, SVD_LR[scale], SCALES[scale][1]
    ref_r, gpu_r, refits = [], [], []
    for f in scaled[scale]:
        rng = np.random.default_rng(7)
        P0, Q0 = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
        a = O.svd_fit(f.iu, f.ii, f.r, P0, Q0, lr=lr)
        ref_r.append(rmse(O.svd_predict(f.tu, f.ti, *a), f.te_r))
        b = ctx.svd_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, lr=lr)  # raises on RS_ERR_NUMERIC
        refits.append(ctx.fit_refits())
        assert all(np.all(np.isfinite(x)) for x in b[:4])
        gpu_r.append(rmse(rsgpu.svd_predict(f.tu, f.ti, *b), f.te_r))
    ref_m, gpu_m = float(np.mean(ref_r)), float(np.mean(gpu_r))
    print(f"{scale}: GPU {gpu_m:.4f}, reference order {ref_m:.4f} ({(gpu_m - ref_m) / mult:+.4f} star units)")
    assert refits == [0] * len(refits), refits
    assert abs(gpu_m - ref_m) <= 0.003 * mult, (gpu_m, ref_m)
    if ref_m / mult <= 0.934:
        assert gpu_m / mult <= 0.934 + 0.008, gpu_m


def test_svd_fast_one_wave_exact_on_1_100(ctx, scaled):
    """One workgroup of one wave on 1-100 ratings (fixed point 2^-20): the sequential SGD in the tile
    order, to 1e-5 x 20 (the star-scale contract in the scale's units)."""
    f = scaled["x20"][0]
    n, k = 20000, 64
    u, i, r = f.iu[:n], f.ii[:n], f.r[:n]
    rng = np.random.default_rng(3)
    P0, Q0 = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
    bu0, bi0 = rng.normal(0, 2.0, f.nu), rng.normal(0, 2.0, f.ni)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, f.nu, f.ni), k)
    plan.set_tiles(workgroups=1, waves=1, target=4000)
    plan.upload(P0, Q0, bu0, bi0, 70.0)
    plan.epochs(2, lr=0.0005)
    got = plan.download()
    rowptr, items, rr = O.csr_by(u, f.nu, i, r)
    cu = np.repeat(np.arange(f.nu, dtype=np.int32), np.diff(rowptr))
    pos, off = plan.tile_order()
    ref = O.svd_fit_works(cu[pos], np.asarray(items, np.int32)[pos], np.asarray(rr)[pos], off, P0, Q0, bu0, bi0,
                          70.0, epochs=2, lr=0.0005, compose=2)
    plan.close()
    d = max(float(np.max(np.abs(np.asarray(x) - np.asarray(y)))) for x, y in zip(ref[:4], got[:4]))
    assert d <= 2e-4 and abs(ref[4] - got[4]) <= 2e-4, d


@pytest.mark.parametrize("scale", sorted(SCALES))
def test_svdpp_fast_on_rating_scale(ctx, scaled, scale):
    """Folds 0-1, k = 20 (the SVD++ default), 20 epochs: FAST within 0.005 x scale of the user-major
    lazy restatement (the star-scale SVD++ bound of test_svdpp_gpu.py in the scale's units), no
    RS_ERR_NUMERIC."""
    k, lr, mult = 20, PP_LR[scale], SCALES[scale][1]
    for f in scaled[scale][:2]:
        rng = np.random.default_rng(4)
        P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (f.nu, f.ni, f.ni))
        rowptr, items, rr = O.csr_by(f.iu, f.nu, f.ii, f.r)
        a = O.svdpp_fit_lazy(rowptr, items, rr, P0, Q0, Y0, lr=lr)
        ref = rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *a), f.te_r)
        b = ctx.svdpp_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, Y0, lr=lr)
        assert all(np.all(np.isfinite(x)) for x in b[:5])
        got = rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *b), f.te_r)
        assert abs(got - ref) <= 0.005 * mult, (got, ref)
