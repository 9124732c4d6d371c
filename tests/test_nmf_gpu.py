"""GPU parity tests of K3 (NMF multiplicative epoch, core/svd.go:158-251) through the C-ABI.

Both passes read the start-of-epoch factors exactly as the reference does and accumulate each row
in data order, so the only difference from the fp64 restatement is fp32 rounding."""
import numpy as np
import pytest

import oracle as O
import rsgpu
from helpers import folds, rmse

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fold0(ml100k):
    return folds(*ml100k)[0]


@pytest.mark.parametrize("as_written", [False, True])
@pytest.mark.parametrize("k,epochs", [(15, 1), (15, 2), (100, 1), (130, 1)])
def test_nmf_matches_oracle(ctx, fold0, as_written, k, epochs):
    f = fold0
    rng = np.random.default_rng(3)
    P0, Q0 = rng.uniform(0, 1, (f.nu, k)), rng.uniform(0, 1, (f.ni, k))
    rP, rQ = O.nmf_fit(f.iu, f.ii, f.r, P0, Q0, epochs=epochs, as_written=as_written)
    gP, gQ = ctx.nmf_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, n_epochs=epochs,
                         as_written=as_written)
    np.testing.assert_allclose(gP, rP, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(gQ, rQ, rtol=2e-5, atol=1e-6)


def test_nmf_intended_rmse_parity(ctx, ml100k):
    """core/base_test.go:42-44 bound (0.963 + 0.008) with the intended update, 5 folds, defaults."""
    k = 15
    ref_r, gpu_r = [], []
    for f in folds(*ml100k):
        rng = np.random.default_rng(5)
        P0, Q0 = rng.uniform(0, 1, (f.nu, k)), rng.uniform(0, 1, (f.ni, k))
        a = O.nmf_fit(f.iu, f.ii, f.r, P0, Q0, epochs=50, as_written=False)
        ref_r.append(rmse(O.nmf_predict(f.tu, f.ti, *a), f.te_r))
        b = ctx.nmf_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, as_written=False)
        gpu_r.append(rmse(O.nmf_predict(f.tu, f.ti, *b), f.te_r))
    assert abs(np.mean(gpu_r) - np.mean(ref_r)) <= 1e-4
    assert np.mean(gpu_r) <= 0.963 + 0.008


def test_nmf_as_written_goes_nonfinite(ctx, fold0):
    """Q5: the reference as written (svd.go:246-248) diverges; so does the faithful port."""
    f = fold0
    rng = np.random.default_rng(5)
    P0, Q0 = rng.uniform(0, 1, (f.nu, 15)), rng.uniform(0, 1, (f.ni, 15))
    P, Q = ctx.nmf_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, as_written=True)
    with np.errstate(all="ignore"):
        assert not np.all(np.isfinite(O.nmf_predict(f.tu, f.ti, P, Q)))
