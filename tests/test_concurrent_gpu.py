"""Concurrent Fit on one device, as the reference's CrossValidate runs it (core/eval.go:28-35: the folds
split over nJobs goroutines by utils.go:145-157 `parallel`, each fitting its own estimator copy).

Every rs_ctx holds one HIP stream; the entry points are re-entrant across contexts.  Here
five host threads, one rs_ctx each, fit the five ML-100K folds at the same time (ctypes releases the GIL
for the duration of a library call, so the calls overlap on the host and on the device):
  * ORDERED SVD: bitwise equal to the same calls made one after the other;
  * FAST SVD: the 5-fold mean held-out RMSE within P2's 0.003 of the reference visit order;
  * KNN Sims (Cosine, MSD, Pearson, each in its own thread, twice over): bitwise equal to serial calls.
"""
import threading

import numpy as np
import pytest

import oracle as O
import rsgpu
from helpers import folds, rmse

pytestmark = pytest.mark.gpu


def _run_threads(fns):
    out, err = [None] * len(fns), [None] * len(fns)

    def one(x):
        try:
            out[x] = fns[x]()
        except BaseException as e:  # noqa: BLE001 -- reraised below
            err[x] = e

    th = [threading.Thread(target=one, args=(x,)) for x in range(len(fns))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return out


def _fit(f, P0, Q0, mode, epochs):
    with rsgpu.Context(0) as c:  # one rs_ctx per thread, as one estimator copy per goroutine
        return c.svd_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, n_epochs=epochs, mode=mode)


def test_concurrent_ordered_fits_bitwise(ml100k):
    fs = folds(*ml100k)
    k = 20
    init = []
    for x, f in enumerate(fs):
        rng = np.random.default_rng(100 + x)
        init.append((rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))))
    serial = [_fit(f, *init[x], rsgpu.SGD_ORDERED, 3) for x, f in enumerate(fs)]
    conc = _run_threads([lambda f=f, x=x: _fit(f, *init[x], rsgpu.SGD_ORDERED, 3) for x, f in enumerate(fs)])
    for a, b in zip(serial, conc):
        assert all(np.array_equal(p, q) for p, q in zip(a[:4], b[:4])) and a[4] == b[4]


def test_concurrent_fast_fits_p2(ml100k):
    fs = folds(*ml100k)
    k = 100
    init, ref = [], []
    for f in fs:
        rng = np.random.default_rng(7)
        P0, Q0 = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
        init.append((P0, Q0))
        ref.append(rmse(O.svd_predict(f.tu, f.ti, *O.svd_fit(f.iu, f.ii, f.r, P0, Q0)), f.te_r))
    got = _run_threads([lambda f=f, x=x: _fit(f, *init[x], rsgpu.SGD_FAST, 20) for x, f in enumerate(fs)])
    for g in got:
        assert all(np.all(np.isfinite(v)) for v in g[:4])
    e = float(np.mean([rmse(O.svd_predict(f.tu, f.ti, *g), f.te_r) for f, g in zip(fs, got)]))
    print(f"concurrent FAST 5-fold RMSE {e:.4f} vs reference order {np.mean(ref):.4f}")
    assert abs(e - float(np.mean(ref))) <= 0.003


def test_concurrent_knn_sims_bitwise(ml100k):
    f = folds(*ml100k)[0]
    rowptr, ids, vals = O.csr_by(f.ii, f.ni, f.iu, f.r)  # item-based: left = items, right = users
    kinds = [rsgpu.SIM_COSINE, rsgpu.SIM_MSD, rsgpu.SIM_PEARSON] * 2

    def sims(kind):
        with rsgpu.Context(0) as c:
            return c.knn_sims(kind, rowptr, ids, vals, f.nu)

    serial = [sims(kd) for kd in kinds]
    conc = _run_threads([lambda kd=kd: sims(kd) for kd in kinds])
    for a, b in zip(serial, conc):
        assert np.array_equal(a, b, equal_nan=True)
