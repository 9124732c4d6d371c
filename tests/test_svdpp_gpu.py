"""GPU parity tests of K2 (SVD++, core/svd.go:259-427) through the C-ABI.

SVD++ parity is unpinned by the reference (its test, core/base_test.go:38-40, is commented out);
the checks are against the fp64 restatement of svd.go:316-427 (oracle/)."""
import numpy as np
import pytest

import oracle as O
import rsgpu
from helpers import folds, rmse

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def fold0(ml100k):
    return folds(*ml100k)[0]


def _maxdiff(a, b):
    return max(float(np.max(np.abs(np.asarray(x) - np.asarray(y)))) for x, y in zip(a, b))


@pytest.mark.parametrize("k,epochs,n", [(20, 1, 2000), (20, 2, 2000), (128, 1, 1500)])
def test_svdpp_ordered_matches_literal_oracle(ctx, fold0, k, epochs, n):
    f = fold0
    u, i, r = f.iu[:n], f.ii[:n], f.r[:n]
    nu, ni = int(u.max()) + 1, int(i.max()) + 1
    rng = np.random.default_rng(21)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
    ref = O.svdpp_fit(u, i, r, nu, P0, Q0, Y0, epochs=epochs)
    got = ctx.svdpp_fit(rsgpu.Ratings(u, i, r, nu, ni), P0, Q0, Y0, n_epochs=epochs,
                        mode=rsgpu.SGD_ORDERED)
    assert _maxdiff(ref[:5], got[:5]) <= TOL
    assert abs(ref[5] - got[5]) <= TOL


def _disjoint(n_users=150, seed=9):
    rng = np.random.default_rng(seed)
    deg = rng.integers(1, 30, n_users)
    users = np.repeat(np.arange(n_users), deg)
    items = np.arange(len(users))
    perm = rng.permutation(len(users))
    return users[perm], items[perm], rng.integers(1, 6, len(users)).astype(float), n_users, len(users)


@pytest.mark.parametrize("k", [20, 100, 128])
def test_svdpp_fast_lazy_matches_literal_race_free(ctx, k):
    """Lazy per-user y update == literal update in user-major order (no two users share an item)."""
    u, i, r, nu, ni = _disjoint()
    rng = np.random.default_rng(k)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
    rowptr, items, rr = O.csr_by(u, nu, i, r)
    for epochs in (1, 3):
        ref = O.svdpp_fit_userwise(rowptr, items, rr, P0, Q0, Y0, epochs=epochs)
        got = ctx.svdpp_fit(rsgpu.Ratings(u, i, r, nu, ni), P0, Q0, Y0, n_epochs=epochs,
                            write_back=rsgpu.WB_ATOMIC)
        assert _maxdiff(ref[:5], got[:5]) <= TOL, (k, epochs)
        assert abs(ref[5] - got[5]) <= TOL


@pytest.mark.parametrize("heavy,k", [(16, 20), (40, 128), (1, 300)])
def test_svdpp_fast_heavy_blocks_race_free(ctx, monkeypatch, heavy, k):
    """Heavy-user blocks (pass 1/3 split over four waves, pass 2 on a producer wave whose q deltas
    go through the LDS ring to three writer waves): forced onto every user with >= `heavy` ratings
    (RSGPU_PP_HEAVY), the epoch must still equal the restatement on race-free input -- long rows
    wrap the ring many times."""
    rng = np.random.default_rng(heavy)
    deg = rng.integers(1, 300, 40)
    users = np.repeat(np.arange(40), deg)
    items = np.arange(len(users))
    perm = rng.permutation(len(users))
    u, i, nu, ni = users[perm], items[perm], 40, len(users)
    r = rng.integers(1, 6, len(users)).astype(float)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
    rowptr, it, rr = O.csr_by(u, nu, i, r)
    monkeypatch.setenv("RSGPU_PP_HEAVY", str(heavy))
    for epochs in (1, 2):
        ref = O.svdpp_fit_userwise(rowptr, it, rr, P0, Q0, Y0, epochs=epochs)
        got = ctx.svdpp_fit(rsgpu.Ratings(u, i, r, nu, ni), P0, Q0, Y0, n_epochs=epochs,
                            write_back=rsgpu.WB_ATOMIC)
        assert _maxdiff(ref[:5], got[:5]) <= TOL, (heavy, k, epochs)
        assert abs(ref[5] - got[5]) <= TOL


def test_svdpp_fast_rmse_near_literal(ctx, fold0):
    """Fast (user-major lazy kernel, Hogwild) vs the literal reference order on ML-100K fold 1,
    defaults (k=20, 20 epochs, lr 0.007, reg 0.02)."""
    f, k = fold0, 20
    rng = np.random.default_rng(4)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (f.nu, f.ni, f.ni))
    a = O.svdpp_fit(f.iu, f.ii, f.r, f.nu, P0, Q0, Y0)
    ref = rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *a), f.te_r)
    b = ctx.svdpp_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, Y0)
    got = rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *b), f.te_r)
    assert abs(got - ref) <= 0.005, (got, ref)
    assert got <= 0.92 + 0.008 + 0.01  # the reference's (disabled) bound, base_test.go:38-40
