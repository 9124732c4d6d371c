"""ctypes binding of oracle/build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference hot path (Oneaccount1/recommend-sys core/svd.go, core/sim.go,
core/knn.go, core/data.go).  See oracle.h for the file:line each function follows and how the
restatement is pinned.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product path (recommend-sys_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_dp = C.POINTER(C.c_double)

COSINE, MSD, PEARSON = 0, 1, 2
BASIC, CENTERED, ZSCORE, BASELINE = 0, 1, 2, 3


def build() -> str:
    src = os.path.join(_HERE, "oracle.c")
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        L.or_trainset_ids.argtypes = [C.c_int64, _i64p, _i64p, _i32p, _i32p,
                                      C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.or_svd_fit.argtypes = [C.c_int64, _i32p, _i32p, _f64p, C.c_int32, C.c_int32,
                                 C.c_double, C.c_double, _f64p, _f64p, _f64p, _f64p, _dp]
        L.or_svd_predict.argtypes = [C.c_int64, _i32p, _i32p, C.c_int32, _f64p, _f64p, _f64p,
                                     _f64p, C.c_double, _f64p]
        L.or_svdpp_fit.argtypes = [C.c_int64, _i32p, _i32p, _f64p, C.c_int32, C.c_int32,
                                   C.c_int32, C.c_double, C.c_double, _f64p, _f64p, _f64p,
                                   _f64p, _f64p, _dp]
        L.or_svdpp_predict.argtypes = [C.c_int64, _i32p, _i32p, C.c_int32, C.c_int64, _i32p,
                                       _i32p, C.c_int32, _f64p, _f64p, _f64p, _f64p, _f64p,
                                       C.c_double, _f64p]
        L.or_nmf_fit.argtypes = [C.c_int64, _i32p, _i32p, _f64p, C.c_int32, C.c_int32,
                                 C.c_int32, C.c_int32, C.c_double, C.c_int32, _f64p, _f64p]
        L.or_nmf_predict.argtypes = [C.c_int64, _i32p, _i32p, C.c_int32, _f64p, _f64p, _f64p]
        L.or_sim.argtypes = [C.c_int32, C.c_int64, _i32p, _f64p, C.c_int64, _i32p, _f64p]
        L.or_sim.restype = C.c_double
        L.or_knn_sims.argtypes = [C.c_int32, C.c_int32, _i64p, _i32p, _f64p, _f64p]
        for fn in (L.or_knn_predict, L.or_knn_predict_stable):
            fn.argtypes = [C.c_int32, C.c_int32, _f64p, _i64p, _i32p, _f64p, _f64p,
                           _f64p, _f64p, C.c_double, C.c_int32, C.c_int32, C.c_int64,
                           _i32p, _i32p, _f64p]
        L.or_go_sort_desc.argtypes = [C.c_int64, _f64p, _i64p]
        L.or_baseline_fit.argtypes = [C.c_int64, _i32p, _i32p, _f64p, C.c_int32, C.c_double,
                                      C.c_double, _f64p, _f64p, _dp]
        L.or_svdpp_fit_userwise.argtypes = [C.c_int32, _i64p, _i32p, _f64p, C.c_int32, C.c_int32,
                                            C.c_double, C.c_double, _f64p, _f64p, _f64p, _f64p,
                                            _f64p, _dp]
        L.or_svdpp_fit_lazy.argtypes = [C.c_int32, _i64p, _i32p, _f64p, C.c_int32, C.c_int32, C.c_double,
                                        C.c_double, _f64p, _f64p, _f64p, _f64p, _f64p, _dp]
        L.or_svd_fit_works.argtypes = [C.c_int64, _i32p, _i32p, _f64p, C.c_int64, _i64p, C.c_int32,
                                       C.c_int32, C.c_double, C.c_double, _f64p, _f64p, _f64p, _f64p, _dp]
        L.or_svd_fit_works_damped.argtypes = [C.c_int64, _i32p, _i32p, _f64p, C.c_int64, _i64p, _i32p, C.c_double,
                                              C.c_int32, C.c_int32, C.c_double, C.c_double, _f64p, _f64p, _f64p,
                                              _f64p, _dp, C.c_int32]
        L.or_svd_fit_works2.argtypes = [C.c_int64, _i32p, _i32p, _f64p, C.c_int64, _i64p, C.c_int32,
                                        C.c_int32, C.c_double, C.c_double, _f64p, _f64p, _f64p, _f64p, _dp,
                                        C.c_int32]
        L.or_svd_fit_chunked.argtypes = [C.c_int32, _i64p, _i32p, _f64p, C.c_int32, C.c_int32,
                                         C.c_int32, C.c_double, C.c_double, _f64p, _f64p, _f64p,
                                         _f64p, _dp]
        L.or_knn_sims_rows.argtypes = [C.c_int32, C.c_int32, _i64p, _i32p, _f64p, C.c_int32,
                                       C.c_int32, _f64p]
        L.or_knn_sims_rows_mt.argtypes = [C.c_int32, C.c_int32, _i64p, _i32p, _f64p, C.c_int32,
                                          C.c_int32, C.c_int32, _f64p]
        L.or_svdpp_fit_jobs.argtypes = [C.c_int64, _i32p, _i32p, _f64p, C.c_int32, C.c_int32,
                                        C.c_int32, C.c_double, C.c_double, _f64p, _f64p, _f64p,
                                        _f64p, _f64p, _dp, C.c_int32, C.c_int64]
        L.or_gb_warm_start.argtypes = [C.c_int32, _i64p, _i32p, _f64p, _f64p, _f64p]
        L.or_gb_warm_start.restype = C.c_double
        L.or_slope_one_fit.argtypes = [C.c_int32, _i64p, _i32p, _f64p, _f64p]
        L.or_slope_one_predict.argtypes = [C.c_int32, _f64p, C.c_int32, _i64p, _i32p, _f64p,
                                           C.c_double, C.c_int64, _i32p, _i32p, _f64p]
        _lib = L
    return _lib


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


# --------------------------------------------------------------------------------------------
# data.go restatements

def trainset_ids(users, items):
    """data.go:131-154: inner ids by first appearance (users, then items)."""
    users, items = _i64(users), _i64(items)
    n = users.shape[0]
    iu = np.empty(n, np.int32)
    ii = np.empty(n, np.int32)
    nu, ni = C.c_int32(0), C.c_int32(0)
    if lib().or_trainset_ids(n, users, items, iu, ii, C.byref(nu), C.byref(ni)) != 0:
        raise MemoryError("or_trainset_ids")
    return iu, ii, nu.value, ni.value


def kfold_indices(n, k, perm):
    """data.go:49-70 KFold with an injected permutation (the reference's rand.Perm is unseeded,
    Q4).  Returns [(train_index, test_index)] with train = perm[:begin] ++ perm[end:]."""
    fold = n // k
    out = []
    begin = end = 0
    for f in range(k):
        end += fold
        if f < n % k:
            end += 1
        test = perm[begin:end]
        train = np.concatenate([perm[:begin], perm[end:]])
        out.append((train, test))
        begin = end
    return out


def csr_by(key, n_rows, *cols):
    """Stable CSR grouping by `key` (data.go:185-216 adjacency lists keep data order)."""
    key = np.asarray(key)
    order = np.argsort(key, kind="stable")
    rowptr = np.zeros(n_rows + 1, np.int64)
    np.add.at(rowptr, key + 1, 1)
    rowptr = np.cumsum(rowptr).astype(np.int64)
    return (rowptr,) + tuple(np.ascontiguousarray(np.asarray(c)[order]) for c in cols)


# --------------------------------------------------------------------------------------------
# estimators

def svd_fit(u, i, r, P, Q, bu=None, bi=None, gb=0.0, epochs=20, lr=0.005, reg=0.02):
    P, Q = _f64(P).copy(), _f64(Q).copy()
    k = P.shape[1]
    bu = np.zeros(P.shape[0]) if bu is None else _f64(bu).copy()
    bi = np.zeros(Q.shape[0]) if bi is None else _f64(bi).copy()
    g = C.c_double(gb)
    lib().or_svd_fit(len(r), _i32(u), _i32(i), _f64(r), k, epochs, lr, reg, P, Q, bu, bi,
                     C.byref(g))
    return P, Q, bu, bi, g.value


def svd_fit_works(u, i, r, work_off, P, Q, bu=None, bi=None, gb=0.0, epochs=1, lr=0.005, reg=0.02, compose=False):
    """The FAST schedules' own semantics: ratings (in this order) cut into works at work_off, each
    with a work-local GlobalBias folded after the epoch (or_svd_fit_works2): compose=False the mean of the
    works' moves (the multi-GPU exchanges), True their chains composed in work order (the single-GPU tile
    schedule)."""
    P, Q = _f64(P).copy(), _f64(Q).copy()
    bu = np.zeros(P.shape[0]) if bu is None else _f64(bu).copy()
    bi = np.zeros(Q.shape[0]) if bi is None else _f64(bi).copy()
    g = C.c_double(gb)
    wo = _i64(work_off)
    lib().or_svd_fit_works2(len(r), _i32(u), _i32(i), _f64(r), len(wo) - 1, wo, P.shape[1], epochs, lr,
                            reg, P, Q, bu, bi, C.byref(g), int(compose))
    return P, Q, bu, bi, g.value


def svd_fit_works_damped(u, i, r, work_off, deg, kconc, P, Q, bu=None, bi=None, gb=0.0, epochs=1, lr=0.005,
                         reg=0.02, compose=2):
    """svd_fit_works with the tile schedule's hot-run damping (or_svd_fit_works_damped): runs of an item with
    deg[item] x kconc >= 4 runs in flight keep min(1, 1 / (R f)) of their move."""
    P, Q = _f64(P).copy(), _f64(Q).copy()
    bu = np.zeros(P.shape[0]) if bu is None else _f64(bu).copy()
    bi = np.zeros(Q.shape[0]) if bi is None else _f64(bi).copy()
    g = C.c_double(gb)
    wo = _i64(work_off)
    lib().or_svd_fit_works_damped(len(r), _i32(u), _i32(i), _f64(r), len(wo) - 1, wo, _i32(deg), float(kconc),
                                  P.shape[1], epochs, lr, reg, P, Q, bu, bi, C.byref(g), int(compose))
    return P, Q, bu, bi, g.value


def svd_predict(u, i, P, Q, bu, bi, gb):
    out = np.empty(len(u))
    lib().or_svd_predict(len(u), _i32(u), _i32(i), P.shape[1], _f64(P), _f64(Q), _f64(bu),
                         _f64(bi), gb, out)
    return out


def gb_warm_start(rowptr, items, r, bu, bi):
    return lib().or_gb_warm_start(len(rowptr) - 1, _i64(rowptr), _i32(items), _f64(r), _f64(bu),
                                  _f64(bi))


def svd_fit_chunked(rowptr, items, r, P, Q, chunk, bu=None, bi=None, gb=0.0, epochs=20,
                    lr=0.005, reg=0.02, warm=True):
    """Restatement of the GPU FAST SVD schedule (with its GlobalBias warm start when warm)."""
    P, Q = _f64(P).copy(), _f64(Q).copy()
    bu = np.zeros(P.shape[0]) if bu is None else _f64(bu).copy()
    bi = np.zeros(Q.shape[0]) if bi is None else _f64(bi).copy()
    if warm and epochs > 0:
        gb = gb_warm_start(rowptr, items, r, bu, bi)
    g = C.c_double(gb)
    lib().or_svd_fit_chunked(P.shape[0], _i64(rowptr), _i32(items), _f64(r), chunk, P.shape[1],
                             epochs, lr, reg, P, Q, bu, bi, C.byref(g))
    return P, Q, bu, bi, g.value


def svdpp_fit(u, i, r, n_users, P, Q, Y, epochs=20, lr=0.007, reg=0.02):
    P, Q, Y = _f64(P).copy(), _f64(Q).copy(), _f64(Y).copy()
    bu, bi = np.zeros(P.shape[0]), np.zeros(Q.shape[0])
    g = C.c_double(0.0)
    lib().or_svdpp_fit(len(r), _i32(u), _i32(i), _f64(r), n_users, P.shape[1], epochs, lr, reg,
                       P, Q, Y, bu, bi, C.byref(g))
    return P, Q, Y, bu, bi, g.value


def svdpp_fit_userwise(rowptr, items, r, P, Q, Y, epochs=20, lr=0.007, reg=0.02, warm=True):
    """Restatement of the GPU FAST SVD++ schedule (with its GlobalBias warm start when warm)."""
    P, Q, Y = _f64(P).copy(), _f64(Q).copy(), _f64(Y).copy()
    bu, bi = np.zeros(P.shape[0]), np.zeros(Q.shape[0])
    g = C.c_double(gb_warm_start(rowptr, items, r, bu, bi) if warm and epochs > 0 else 0.0)
    lib().or_svdpp_fit_userwise(P.shape[0], _i64(rowptr), _i32(items), _f64(r), P.shape[1], epochs,
                                lr, reg, P, Q, Y, bu, bi, C.byref(g))
    return P, Q, Y, bu, bi, g.value


def svdpp_fit_lazy(rowptr, items, r, P, Q, Y, epochs=20, lr=0.007, reg=0.02, warm=True):
    """svdpp_fit_userwise's schedule in the lazy O(nnz k) form (or_svdpp_fit_lazy)."""
    P, Q, Y = _f64(P).copy(), _f64(Q).copy(), _f64(Y).copy()
    bu, bi = np.zeros(P.shape[0]), np.zeros(Q.shape[0])
    g = C.c_double(gb_warm_start(rowptr, items, r, bu, bi) if warm and epochs > 0 else 0.0)
    lib().or_svdpp_fit_lazy(P.shape[0], _i64(rowptr), _i32(items), _f64(r), P.shape[1], epochs, lr, reg,
                            P, Q, Y, bu, bi, C.byref(g))
    return P, Q, Y, bu, bi, g.value


def svdpp_predict(tu, ti, n_users, u, i, P, Q, Y, bu, bi, gb):
    out = np.empty(len(u))
    lib().or_svdpp_predict(len(tu), _i32(tu), _i32(ti), n_users, len(u), _i32(u), _i32(i),
                           P.shape[1], _f64(P), _f64(Q), _f64(Y), _f64(bu), _f64(bi), gb, out)
    return out


def nmf_fit(u, i, r, P, Q, epochs=50, reg=0.06, as_written=True):
    P, Q = _f64(P).copy(), _f64(Q).copy()
    lib().or_nmf_fit(len(r), _i32(u), _i32(i), _f64(r), P.shape[0], Q.shape[0], P.shape[1],
                     epochs, reg, int(as_written), P, Q)
    return P, Q


def nmf_predict(u, i, P, Q):
    out = np.empty(len(u))
    lib().or_nmf_predict(len(u), _i32(u), _i32(i), P.shape[1], _f64(P), _f64(Q), out)
    return out


def sim(kind, a_ids, a_r, b_ids, b_r):
    return lib().or_sim(kind, len(a_ids), _i32(a_ids), _f64(a_r), len(b_ids), _i32(b_ids),
                        _f64(b_r))


def knn_sims(kind, rowptr, ids, ratings):
    L = len(rowptr) - 1
    out = np.empty((L, L))
    lib().or_knn_sims(kind, L, _i64(rowptr), _i32(ids), _f64(ratings), out)
    return out


def knn_sims_rows_mt(kind, rowptr, sorted_ids, sorted_r, row_begin, row_end, n_jobs):
    """knn_sims_rows on n_jobs threads, rows split as knn.go:192-216 splits them (CPU baseline)."""
    L = len(rowptr) - 1
    out = np.empty((row_end - row_begin, L))
    lib().or_knn_sims_rows_mt(kind, L, _i64(rowptr), _i32(sorted_ids), _f64(sorted_r), row_begin,
                              row_end, n_jobs, out)
    return out


def svdpp_fit_jobs(u, i, r, n_users, P, Q, Y, epochs=1, lr=0.007, reg=0.02, n_jobs=1):
    """svdpp_fit with svd.go:399-422's per-rating nJobs split of the y-update (CPU baseline)."""
    P, Q, Y = _f64(P).copy(), _f64(Q).copy(), _f64(Y).copy()
    bu, bi = np.zeros(P.shape[0]), np.zeros(Q.shape[0])
    g = C.c_double(0.0)
    lib().or_svdpp_fit_jobs(len(r), _i32(u), _i32(i), _f64(r), n_users, P.shape[1], epochs, lr, reg,
                            P, Q, Y, bu, bi, C.byref(g), n_jobs, len(r))
    return P, Q, Y, bu, bi, g.value


def svdpp_fit_sample(u, i, r, n_users, P, Q, Y, n_visit, lr=0.007, reg=0.02, n_jobs=1):
    """The first n_visit ratings of one svdpp_fit_jobs epoch, N(u) over all ratings (a timed slice)."""
    P, Q, Y = _f64(P).copy(), _f64(Q).copy(), _f64(Y).copy()
    bu, bi = np.zeros(P.shape[0]), np.zeros(Q.shape[0])
    g = C.c_double(0.0)
    lib().or_svdpp_fit_jobs(len(r), _i32(u), _i32(i), _f64(r), n_users, P.shape[1], 1, lr, reg,
                            P, Q, Y, bu, bi, C.byref(g), n_jobs, n_visit)


def knn_sims_rows(kind, rowptr, sorted_ids, sorted_r, row_begin, row_end):
    """Rows of the pair loop (rows must already be ID-sorted, data.go:236-243)."""
    L = len(rowptr) - 1
    out = np.empty((row_end - row_begin, L))
    lib().or_knn_sims_rows(kind, L, _i64(rowptr), _i32(sorted_ids), _f64(sorted_r), row_begin,
                           row_end, out)
    return out


def go_sort_desc(keys):
    """Go 1.24 sort.Sort's permutation under Less(i, j) = keys[i] > keys[j] (knn.go:43-45, 107-108)."""
    keys = np.ascontiguousarray(keys, dtype=np.float64)
    perm = np.empty(len(keys), np.int64)
    lib().or_go_sort_desc(len(keys), _f64(keys), _i64(perm))
    return perm


def knn_predict(type_, sims, right_rowptr, right_ids, right_r, means, stddevs, bias,
                global_mean, k, min_k, left, right, stable=False):
    """knn.go:75-141; ties in Go sort.Sort's order (stable=True: candidate order)."""
    L = sims.shape[0]
    z = np.zeros(max(L, 1))
    out = np.empty(len(left))
    fn = lib().or_knn_predict_stable if stable else lib().or_knn_predict
    fn(type_, L, _f64(sims), _i64(right_rowptr), _i32(right_ids),
                         _f64(right_r), _f64(z if means is None else means),
                         _f64(z if stddevs is None else stddevs), _f64(z if bias is None else bias),
                         global_mean, k, min_k, len(left), _i32(left), _i32(right), out)
    return out


def slope_one_fit(rowptr, ids, ratings):
    """slope_one.go:47-93: dev matrix from the item CSR (user ids, data order)."""
    L = len(rowptr) - 1
    out = np.empty((L, L))
    lib().or_slope_one_fit(L, _i64(rowptr), _i32(ids), _f64(ratings), out)
    return out


def slope_one_predict(dev, user_rowptr, user_items, user_ratings, global_mean, users, items):
    """slope_one.go:21-45 for inner-id pairs (-1 = unknown)."""
    out = np.empty(len(users))
    lib().or_slope_one_predict(dev.shape[0], _f64(dev), len(user_rowptr) - 1, _i64(user_rowptr),
                               _i32(user_items), _f64(user_ratings), global_mean, len(users),
                               _i32(users), _i32(items), out)
    return out


def baseline_fit(u, i, r, n_users, n_items, epochs=20, lr=0.005, reg=0.02):
    bu, bi = np.zeros(n_users), np.zeros(n_items)
    g = C.c_double(0.0)
    lib().or_baseline_fit(len(r), _i32(u), _i32(i), _f64(r), epochs, lr, reg, bu, bi,
                          C.byref(g))
    return bu, bi, g.value
