"""GPU parity tests of SlopeOne (core/slope_one.go): the deviation matrix on the
int8-MFMA pair kernel (X M^T, M X^T, M M^T) and on the merge-order kernel, and SlopeOne.Predict on
the device -- all bitwise equal to the oracle's restatement (including the signs of zero:
dev[j][i] = -dev[i][j] is written as a negation, so a zero mean difference gives +0 / -0)."""
import numpy as np
import pytest

import oracle as O
import rsgpu
from helpers import folds, mae, rmse

pytestmark = pytest.mark.gpu
EPS = 0.008


def same_bits(a, b):
    return np.array_equal(np.asarray(a).view(np.uint64), np.asarray(b).view(np.uint64))


@pytest.fixture(scope="module")
def item_rows(ml100k):
    U, I, R = ml100k
    iu, ii, nu, ni = O.trainset_ids(U, I)
    rowptr, ids, rr = O.csr_by(ii, ni, iu, R)
    return rowptr, ids, rr, nu, ni


@pytest.mark.parametrize("mfma", [True, False])
def test_dev_ml100k_bitwise(ctx, item_rows, mfma, monkeypatch):
    rowptr, ids, rr, nu, ni = item_rows
    ref = O.slope_one_fit(rowptr, ids, rr)
    if not mfma:
        monkeypatch.setenv("RSGPU_KNN_NO_MFMA", "1")
    got = ctx.knn_sims(rsgpu.DEV_SLOPE_ONE, rowptr, ids, rr, nu)
    assert same_bits(ref, got)


@pytest.mark.parametrize("scale,seed", [(2, 1), (1, 2), (0, 3)])
def test_dev_random_sets_bitwise(ctx, scale, seed):
    """Half stars (MFMA, s = 2), integer stars 1..11 (s = 1), and non-representable ratings
    (merge path), ragged rows with empty ones."""
    rng = np.random.default_rng(seed)
    L, R = 300, 500
    deg = rng.integers(0, 60, L)
    deg[::17] = 0
    rows, ids = [], []
    for a in range(L):
        ids.append(np.sort(rng.choice(R, deg[a], replace=False)))
    ids = np.concatenate(ids).astype(np.int32)
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    n = len(ids)
    if scale == 2:
        r = rng.integers(1, 11, n) / 2.0
    elif scale == 1:
        r = rng.integers(1, 12, n).astype(float)
    else:
        r = rng.uniform(0.5, 5.0, n)
    perm = np.concatenate([rowptr[a] + rng.permutation(deg[a]) for a in range(L)]).astype(np.int64)
    ids, r = ids[perm], r[perm]  # data order inside rows is unsorted
    ref = O.slope_one_fit(rowptr, ids, r)
    got = ctx.knn_sims(rsgpu.DEV_SLOPE_ONE, rowptr, ids, r, R)
    assert same_bits(ref, got)


@pytest.mark.parametrize("n_parts", [2, 3])
def test_dev_parts_cover_exactly(ctx, item_rows, n_parts):
    rowptr, ids, rr, nu, ni = item_rows
    full = ctx.knn_sims(rsgpu.DEV_SLOPE_ONE, rowptr, ids, rr, nu)
    acc = np.full((ni, ni), np.nan)
    for p in range(n_parts):
        out = np.full((ni, ni), np.nan)
        ctx.knn_sims(rsgpu.DEV_SLOPE_ONE, rowptr, ids, rr, nu, part=p, n_parts=n_parts, out=out)
        m = ~np.isnan(out)
        assert not np.any(m & ~np.isnan(acc))
        acc[m] = out[m]
    assert same_bits(acc, full)


def test_predict_bitwise_and_accuracy(ctx, ml100k):
    """Device Predict bitwise equal to slope_one.go:21-45 (unknown users / items included) on every
    fold of a 5-fold ML-100K split, and the CV means within core/base_test.go:46-48's bound."""
    rs_, ms_ = [], []
    for f in folds(*ml100k):
        ip, iid, ir = O.csr_by(f.ii, f.ni, f.iu, f.r)
        up, uit, ur = O.csr_by(f.iu, f.nu, f.ii, f.r)
        gm = float(np.mean(f.r))
        dev = O.slope_one_fit(ip, iid, ir)
        tu = np.concatenate([f.tu, [-1, 0, -1]]).astype(np.int32)
        ti = np.concatenate([f.ti, [0, -1, -1]]).astype(np.int32)
        ref = O.slope_one_predict(dev, up, uit, ur, gm, tu, ti)
        plan = ctx.knn_plan(rsgpu.DEV_SLOPE_ONE, ip, iid, ir, f.nu)
        got = plan.slope_one_predict(up, uit, ur, gm, tu, ti)
        assert same_bits(plan.sims(), dev)
        plan.close()
        assert same_bits(ref, got)
        rs_.append(rmse(got[:len(f.te_r)], f.te_r))
        ms_.append(mae(got[:len(f.te_r)], f.te_r))
    assert np.mean(rs_) <= 0.946 + EPS and np.mean(ms_) <= 0.743 + EPS


def test_predict_rejects_non_slope_one_plan(ctx, item_rows):
    rowptr, ids, rr, nu, ni = item_rows
    plan = ctx.knn_plan(rsgpu.SIM_COSINE, rowptr[:51], ids[:rowptr[50]], rr[:rowptr[50]], nu)
    with pytest.raises(rsgpu.RsError):
        plan.slope_one_predict(np.array([0, 1], np.int64), np.array([0], np.int32), np.array([3.0]),
                               3.0, np.array([0], np.int32), np.array([0], np.int32))
    plan.close()
