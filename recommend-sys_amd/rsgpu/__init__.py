"""ctypes binding of librsgpu.so (include/rsgpu.h) -- the host side used by tests and bench.py.

This module is plumbing over the C-ABI: every compute call goes to the HIP library and fails
loudly (RsError) when the library or a gfx950 device is missing.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
import weakref

import numpy as np

from . import _build

LIB_PATH = _build.LIB
_lib = None

RS_OK = 0
RS_ERR_INVALID, RS_ERR_HIP, RS_ERR_NOMEM, RS_ERR_UNSUPPORTED, RS_ERR_NO_DEVICE, RS_ERR_NUMERIC = -1, -2, -3, -4, -5, -6
SGD_FAST, SGD_ORDERED = 0, 1
WB_TILE, WB_STORE, WB_ATOMIC_DIRECT, WB_ATOMIC = 0, 1, 2, 3  # WB_TILE: the default schedule
SIM_COSINE, SIM_MSD, SIM_PEARSON = 0, 1, 2
TIE_GO_SORT, TIE_STABLE = 0, 1  # KNN.Predict tie order (rs_knn_plan_set_tie_order)
DEV_SLOPE_ONE = 3  # rs_knn_sims kind: SlopeOne deviation matrix (slope_one.go:64-92)
EXCHANGE_ROTATE, EXCHANGE_AVERAGE, EXCHANGE_ROTATE_Q, EXCHANGE_QDELTA = 0, 1, 2, 3  # multi-GPU exchange (rsgpu.h)
GB_FOLD_MEAN, GB_FOLD_SMOOTH = 0, 1  # rs_svd_plan_set_gb_fold
FAULT_DIVERGE = -2  # rs_svd_plan_inject_fault: perturb a replica before the consistency check (rsgpu.h)
TILE_RULE_LPT, TILE_RULE_FILL, TILE_RULE_FILL_DEVICE = 0, 1, 2  # how users are cut into tiles (rsgpu.h)

HEADER_SYMBOLS = (
    "rs_version", "rs_device_count", "rs_open", "rs_close", "rs_last_error", "rs_synchronize",
    "rs_last_kernel_ms",
    "rs_svd_fit", "rs_svd_predict", "rs_svdpp_fit", "rs_nmf_fit", "rs_baseline_fit",
    "rs_knn_sims", "rs_knn_sims_part", "rs_knn_part_blocks", "rs_sim_pair", "rs_svd_plan_create", "rs_svd_plan_destroy",
    "rs_svd_plan_upload", "rs_svd_plan_download", "rs_svd_plan_epochs",
    "rs_svd_plan_device_ptrs", "rs_svd_plan_set_mode", "rs_svd_plan_set_split", "rs_svd_plan_set_schedule", "rs_svd_plan_trace",
    "rs_svd_plan_set_item_split", "rs_svd_plan_set_timing", "rs_svd_plan_set_user_weights",
    "rs_svd_plan_epoch_delta", "rs_svd_plan_apply_delta", "rs_svd_plan_last_kernel_ms",
    "rs_svd_plan_predict", "rs_svd_plan_evaluate",
    "rs_knn_plan_create", "rs_knn_plan_destroy", "rs_knn_plan_sims", "rs_knn_plan_predict",
    "rs_svd_plan_create_csr", "rs_svd_plan_init_normal", "rs_slope_one_predict",
    "rs_trainset_ids", "rs_csr_build", "rs_global_mean",
    "rs_synth_create", "rs_synth_csr", "rs_synth_destroy",
    "rs_svd_plan_set_item_weights", "rs_svd_plan_epoch_qdelta", "rs_svd_plan_apply_qdelta",
    "rs_svd_plan_set_hot_replicas", "rs_svd_plan_set_fixed_q", "rs_svd_plan_set_tiles",
    "rs_svd_plan_set_tile_claim", "rs_svd_plan_tile_order", "rs_svd_plan_tile_clocks",
    "rs_svd_plan_set_tile_rule", "rs_svd_plan_tile_rule", "rs_svd_plan_set_guard", "rs_svd_plan_refits", "rs_svd_plan_fixed_point", "rs_svd_plan_schedule_digest", "rs_fit_schedule_digest",
    "rs_comm_unique_id", "rs_svd_plan_join", "rs_svd_plan_epochs_sharded", "rs_svd_plan_leave",
    "rs_svd_plan_set_user_blocks", "rs_svd_group_create", "rs_svd_group_epochs", "rs_svd_group_destroy",
    "rs_item_shards", "rs_svd_fit_multi", "rs_tile_schedule_host", "rs_svd_plan_set_exchange", "rs_svd_plan_set_qdelta_wire", "rs_svd_plan_set_qdelta_split",
    "rs_svd_plan_set_qdelta_curvature", "rs_svd_plan_set_damp_concurrency", "rs_svd_plan_set_cold_store", "rs_svd_plan_set_gb_fold",
    "rs_comm_info", "rs_rotation_step", "rs_svd_plan_shard_info", "rs_svd_plan_qdelta_info", "rs_svd_plan_inject_fault",
    "rs_svd_plan_time_blocks", "rs_knn_plan_set_tie_order", "rs_fit_refits", "rs_open_r",
    "rs_svd_plan_set_hot_split",
)
COMM_ID_BYTES = 128


class RsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"librsgpu error {code}: {msg}")
        self.code = code


class _Ratings(C.Structure):
    _fields_ = [("nnz", C.c_int64), ("n_users", C.c_int32), ("n_items", C.c_int32),
                ("users", C.c_void_p), ("items", C.c_void_p), ("ratings", C.c_void_p)]


class _Report(C.Structure):  # rs_report
    _fields_ = [("refits", C.c_int32), ("error", C.c_char * 508)]


class _SgdParams(C.Structure):
    _fields_ = [("n_factors", C.c_int32), ("n_epochs", C.c_int32), ("lr", C.c_double),
                ("reg", C.c_double), ("mode", C.c_int32), ("write_back", C.c_int32)]


_vp = C.c_void_p
_i32, _i64, _dbl, _flt = C.c_int32, C.c_int64, C.c_double, C.c_float


def _torch_stream(t):
    """torch's current HIP stream on tensor t's device (a hipStream_t as int)."""
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream


def lib():
    """Loads librsgpu.so (building it first when the sources are newer)."""
    global _lib
    if _lib is None:
        if os.path.exists(os.path.join(_build.CSRC, "sgd.hip")):
            _build.build()
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"librsgpu.so missing at {LIB_PATH}; run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        sig = {
            "rs_version": (_i32, []),
            "rs_device_count": (C.c_int, [C.POINTER(_i32)]),
            "rs_open": (C.c_int, [_i32, C.POINTER(_vp)]),
            "rs_close": (None, [_vp]),
            "rs_last_error": (C.c_char_p, [_vp]),
            "rs_synchronize": (C.c_int, [_vp]),
            "rs_last_kernel_ms": (C.c_int, [_vp, C.POINTER(_dbl)]),
            "rs_svd_fit": (C.c_int, [_vp, C.POINTER(_Ratings), C.POINTER(_SgdParams), _vp, _vp,
                                     _vp, _vp, _vp]),
            "rs_svd_predict": (C.c_int, [_vp, _i64, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp,
                                         _vp, _dbl, _vp]),
            "rs_svdpp_fit": (C.c_int, [_vp, C.POINTER(_Ratings), C.POINTER(_SgdParams), _vp, _vp,
                                       _vp, _vp, _vp, _vp]),
            "rs_nmf_fit": (C.c_int, [_vp, C.POINTER(_Ratings), _i32, _i32, _dbl, _i32, _vp, _vp]),
            "rs_baseline_fit": (C.c_int, [_vp, C.POINTER(_Ratings), _i32, _dbl, _dbl, _vp, _vp,
                                          _vp]),
            "rs_knn_sims": (C.c_int, [_vp, _i32, _i32, _i32, _vp, _vp, _vp, _vp]),
            "rs_knn_sims_part": (C.c_int, [_vp, _i32, _i32, _i32, _vp, _vp, _vp, _i32, _i32, _vp]),
            "rs_knn_part_blocks": (C.c_int, [_i32, _i32, _i32, _vp]),
            "rs_sim_pair": (C.c_int, [_vp, _i32, _i64, _vp, _vp, _i64, _vp, _vp, _vp]),
            "rs_svd_plan_create": (C.c_int, [_vp, C.POINTER(_Ratings), _i32, C.POINTER(_vp)]),
            "rs_svd_plan_destroy": (None, [_vp]),
            "rs_svd_plan_upload": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
            "rs_svd_plan_download": (C.c_int, [_vp, _vp, _vp, _vp, _vp, _vp]),
            "rs_svd_plan_epochs": (C.c_int, [_vp, _i32, _flt, _flt, _vp]),
            "rs_svd_plan_device_ptrs": (C.c_int, [_vp, C.POINTER(_vp), C.POINTER(_vp),
                                                  C.POINTER(_vp), C.POINTER(_i32)]),
            "rs_svd_plan_set_mode": (C.c_int, [_vp, _i32, _i32]),
            "rs_svd_plan_set_split": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_set_schedule": (C.c_int, [_vp, _i32, _i32]),
            "rs_svd_plan_trace": (C.c_int, [_vp, _vp, _vp]),
            "rs_svd_plan_set_item_split": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_set_user_weights": (C.c_int, [_vp, _vp]),
            "rs_svd_plan_epoch_delta": (C.c_int, [_vp, _flt, _flt, _vp, _vp, _vp]),
            "rs_svd_plan_apply_delta": (C.c_int, [_vp, _vp, _vp, _dbl, _vp]),
            "rs_svd_plan_set_timing": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_last_kernel_ms": (C.c_int, [_vp, C.POINTER(_dbl), C.POINTER(_i32)]),
            "rs_svd_plan_predict": (C.c_int, [_vp, _i64, _vp, _vp, _vp]),
            "rs_knn_plan_create": (C.c_int, [_vp, _i32, _i32, _i32, _vp, _vp, _vp, C.POINTER(_vp)]),
            "rs_knn_plan_destroy": (None, [_vp]),
            "rs_knn_plan_sims": (C.c_int, [_vp, _vp]),
            "rs_knn_plan_predict": (C.c_int, [_vp, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _dbl,
                                              _i32, _i32, _i64, _vp, _vp, _vp]),
            "rs_svd_plan_evaluate": (C.c_int, [_vp, _i64, _vp, _vp, _vp, C.POINTER(_dbl), C.POINTER(_dbl)]),
            "rs_slope_one_predict": (C.c_int, [_vp, _i32, _vp, _vp, _vp, _dbl, _i64, _vp, _vp, _vp]),
            "rs_svd_plan_create_csr": (C.c_int, [_vp, _i32, _i32, _vp, _vp, _vp, _i32, C.POINTER(_vp)]),
            "rs_svd_plan_init_normal": (C.c_int, [_vp, _dbl, _dbl, C.c_uint64]),
            "rs_trainset_ids": (C.c_int, [_i64, _vp, _i32, _vp, _vp, C.POINTER(_i32)]),
            "rs_csr_build": (C.c_int, [_i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp]),
            "rs_global_mean": (C.c_int, [_i64, _vp, _i32, C.POINTER(_dbl)]),
            "rs_synth_create": (C.c_int, [_i32, _i32, _dbl, _dbl, _i32, _i32, _dbl, C.c_uint64, _i32,
                                          _i32, _i32, _i32, _i32, C.POINTER(_vp)]),
            "rs_svd_plan_set_item_weights": (C.c_int, [_vp, _vp]),
            "rs_svd_plan_set_hot_replicas": (C.c_int, [_vp, _i32, _i32]),
            "rs_svd_plan_set_fixed_q": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_set_tiles": (C.c_int, [_vp, _i32, _i32, _i32, _i32, _i32]),
            "rs_svd_plan_set_tile_claim": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_set_tile_rule": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_set_guard": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_refits": (C.c_int, [_vp, C.POINTER(_i32)]),
            "rs_svd_plan_fixed_point": (C.c_int, [_vp, C.POINTER(_i32)]),
            "rs_svd_plan_tile_rule": (C.c_int, [_vp, C.POINTER(_i32)]),
            "rs_svd_plan_schedule_digest": (C.c_int, [_vp, C.POINTER(C.c_uint64)]),
            "rs_fit_schedule_digest": (C.c_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(_i32)]),
            "rs_svd_plan_tile_order": (C.c_int, [_vp, _vp, _vp, C.POINTER(_i32)]),
            "rs_svd_plan_tile_clocks": (C.c_int, [_vp, _vp, _i64]),
            "rs_svd_plan_epoch_qdelta": (C.c_int, [_vp, _flt, _flt, _vp, _vp, _vp]),
            "rs_svd_plan_apply_qdelta": (C.c_int, [_vp, _vp, _vp, _dbl, _vp]),
            "rs_synth_csr": (C.c_int, [_vp, C.POINTER(_i64), C.POINTER(_vp), C.POINTER(_vp),
                                       C.POINTER(_vp)]),
            "rs_synth_destroy": (None, [_vp]),
            "rs_comm_unique_id": (C.c_int, [_vp]),
            "rs_svd_plan_join": (C.c_int, [_vp, _vp, _i32, _i32, _i32]),
            "rs_svd_plan_epochs_sharded": (C.c_int, [_vp, _i32, _flt, _flt, _vp]),
            "rs_svd_plan_leave": (C.c_int, [_vp]),
            "rs_svd_plan_set_user_blocks": (C.c_int, [_vp, _i32, _vp]),
            "rs_svd_group_create": (C.c_int, [_vp, _i32, _i32, C.POINTER(_vp)]),
            "rs_svd_group_epochs": (C.c_int, [_vp, _i32, _flt, _flt]),
            "rs_svd_group_destroy": (None, [_vp]),
            "rs_item_shards": (C.c_int, [_i64, _vp, _i32, _i32, _vp]),
            "rs_tile_schedule_host": (C.c_int, [_i32, _i32, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _i32, _vp,
                                                _vp, _vp, C.POINTER(_i32), C.POINTER(_dbl)]),
            "rs_svd_fit_multi": (C.c_int, [_vp, _i32, C.POINTER(_Ratings), C.POINTER(_SgdParams), _i32,
                                           _vp, _vp, _vp, _vp, _vp, C.POINTER(_Report)]),
            "rs_svd_plan_set_exchange": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_set_qdelta_wire": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_set_qdelta_split": (C.c_int, [_vp, C.c_double, _i32]),
            "rs_svd_plan_set_qdelta_curvature": (C.c_int, [_vp, C.c_double]),
            "rs_svd_plan_set_damp_concurrency": (C.c_int, [_vp, C.c_float]),
            "rs_svd_plan_set_cold_store": (C.c_int, [_vp, C.c_double]),
            "rs_svd_plan_set_gb_fold": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_inject_fault": (C.c_int, [_vp, _i32]),
            "rs_svd_plan_time_blocks": (C.c_int, [_vp, _flt, _flt, _vp, _i32]),
            "rs_knn_plan_set_tie_order": (C.c_int, [_vp, _i32]),
            "rs_fit_refits": (C.c_int, [_vp, C.POINTER(_i32)]),
            "rs_open_r": (C.c_int, [_i32, C.POINTER(_vp), C.POINTER(_Report)]),
            "rs_svd_plan_set_hot_split": (C.c_int, [_vp, _dbl, _i64, _i32]),
            "rs_comm_info": (C.c_int, [C.POINTER(_i32), _vp, _i32]),
            "rs_rotation_step": (C.c_int, [_i32, _i32, _i32, _vp]),
            "rs_svd_plan_shard_info": (C.c_int, [_vp, C.POINTER(_i32), C.POINTER(_i32), C.POINTER(_i32),
                                                 C.POINTER(_i32)]),
            "rs_svd_plan_qdelta_info": (C.c_int, [_vp, C.POINTER(_i32), C.POINTER(_i32)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _check(code, ctx=None):
    if code != RS_OK:
        msg = lib().rs_last_error(ctx)
        raise RsError(code, msg.decode() if msg else "")


def device_count() -> int:
    n = _i32(0)
    code = lib().rs_device_count(C.byref(n))
    return n.value if code == RS_OK else 0


# ---- TrainSet construction (host C++, no GPU; core/data.go:131-216) ------------------------------

def trainset_ids(outer, n_threads=0):
    """data.go:137-151: inner ids by first appearance.  Returns (inner int32, outer_of_inner int64)."""
    o = np.ascontiguousarray(outer, dtype=np.int64)
    inner = np.empty(len(o), np.int32)
    inv = np.empty(len(o), np.int64)
    n = _i32(0)
    _check(lib().rs_trainset_ids(len(o), _ptr(o), n_threads, _ptr(inner), _ptr(inv), C.byref(n)))
    return inner, inv[:n.value].copy()


def csr_build(rows, cols, vals, n_rows, n_threads=0):
    """data.go:185-216: stable CSR (data order in a row).  Returns (rowptr int64, cols int32, vals f32)."""
    r = np.ascontiguousarray(rows, dtype=np.int32)
    c = np.ascontiguousarray(cols, dtype=np.int32)
    v = np.ascontiguousarray(vals, dtype=np.float64)
    rowptr = np.empty(n_rows + 1, np.int64)
    co, vo = np.empty(len(r), np.int32), np.empty(len(r), np.float32)
    _check(lib().rs_csr_build(len(r), n_rows, _ptr(r), _ptr(c), _ptr(v), n_threads, _ptr(rowptr),
                              _ptr(co), _ptr(vo)))
    return rowptr, co, vo


def global_mean(ratings, n_threads=0):
    """data.go:134 stat.Mean (fixed-order chunked sum)."""
    r = np.ascontiguousarray(ratings, dtype=np.float64)
    m = _dbl(0)
    _check(lib().rs_global_mean(len(r), _ptr(r), n_threads, C.byref(m)))
    return m.value


class Synth:
    """Synthetic inner-id user-CSR (rs_synth_*; BASELINE configs[4] generator).  The arrays are
    numpy views of library memory, valid until close()."""

    def __init__(self, n_users, n_items, mean_deg=100.0, sigma=1.0, min_deg=1, max_deg=None,
                 zipf_s=0.9, seed=20250826, item_lo=0, item_hi=None, user_lo=0, user_hi=None,
                 n_threads=0):
        """Rows are users [user_lo, user_hi) (row x = user user_lo + x); items [item_lo, item_hi)."""
        h = C.c_void_p()
        max_deg = n_items // 2 if max_deg is None else max_deg
        item_hi = n_items if item_hi is None else item_hi
        user_hi = n_users if user_hi is None else user_hi
        _check(lib().rs_synth_create(n_users, n_items, mean_deg, sigma, min_deg, max_deg, zipf_s,
                                     seed, item_lo, item_hi, user_lo, user_hi, n_threads, C.byref(h)))
        n_users = user_hi - user_lo
        self.h, self.n_users, self.n_items = h, n_users, n_items
        nnz, rp, co, va = _i64(0), C.c_void_p(), C.c_void_p(), C.c_void_p()
        _check(lib().rs_synth_csr(h, C.byref(nnz), C.byref(rp), C.byref(co), C.byref(va)))
        self.nnz = nnz.value
        mk = lambda p, t, n: np.ctypeslib.as_array(C.cast(p, C.POINTER(t)), shape=(n,)) if n else np.empty(0)
        self.rowptr = mk(rp, C.c_int64, n_users + 1)
        self.cols = mk(co, C.c_int32, self.nnz)
        self.vals = mk(va, C.c_float, self.nnz)

    def close(self):
        if self.h:
            self.rowptr = self.cols = self.vals = None
            lib().rs_synth_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Ratings:
    """COO TrainSet ratings in train-set order with inner ids (core/data.go:109-127)."""

    def __init__(self, users, items, ratings, n_users=None, n_items=None):
        self.users = np.ascontiguousarray(users, dtype=np.int32)
        self.items = np.ascontiguousarray(items, dtype=np.int32)
        self.ratings = np.ascontiguousarray(ratings, dtype=np.float64)
        self.n_users = int(self.users.max() + 1 if n_users is None and len(self.users) else (n_users or 0))
        self.n_items = int(self.items.max() + 1 if n_items is None and len(self.items) else (n_items or 0))

    def c(self):
        return _Ratings(len(self.ratings), self.n_users, self.n_items, _ptr(self.users),
                        _ptr(self.items), _ptr(self.ratings))


class Context:
    """One HIP stream on one gfx950 device (rs_open / rs_close)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        code = lib().rs_open(device, C.byref(h))
        if code != RS_OK:
            raise RsError(code, lib().rs_last_error(None).decode())
        self.h = h
        self.device = device
        self._plans = weakref.WeakSet()

    def close(self):
        if self.h:
            for pl in list(self._plans):
                pl.close()
            lib().rs_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, code):
        _check(code, self.h)

    def last_kernel_ms(self) -> float:
        """Device time of the kernels of the last estimator call on this context."""
        ms = _dbl(0)
        self.check(lib().rs_last_kernel_ms(self.h, C.byref(ms)))
        return ms.value

    # ---- estimators --------------------------------------------------------------------------

    def fit_refits(self):
        """Divergence refits (a quarter of the workgroups each) the last svd_fit made (rs_fit_refits)."""
        n = _i32(0)
        self.check(lib().rs_fit_refits(self.h, C.byref(n)))
        return n.value

    def fit_schedule_digest(self):
        """(digest, tile rule) of the tile schedule the last FAST svd_fit built (rs_fit_schedule_digest)."""
        d, rule = C.c_uint64(0), _i32(0)
        self.check(lib().rs_fit_schedule_digest(self.h, C.byref(d), C.byref(rule)))
        return d.value, rule.value

    def svd_fit(self, r: Ratings, P, Q, bu=None, bi=None, gb=0.0, n_epochs=20, lr=0.005,
                reg=0.02, mode=SGD_FAST, write_back=WB_TILE, inplace=False):
        """core/svd.go:63-132 through rs_svd_fit.  inplace=True: P, Q, bu, bi (float64, C order) are trained in
        place, as the Go binding's slices are (no copies); otherwise copies are trained and returned."""
        if inplace:
            for a in (P, Q, bu, bi):
                assert isinstance(a, np.ndarray) and a.dtype == np.float64 and a.flags.c_contiguous and a.flags.writeable
        else:
            P = np.array(P, dtype=np.float64, order="C")
            Q = np.array(Q, dtype=np.float64, order="C")
            bu = np.zeros(r.n_users) if bu is None else np.array(bu, dtype=np.float64)
            bi = np.zeros(r.n_items) if bi is None else np.array(bi, dtype=np.float64)
        g = np.array([gb], dtype=np.float64)
        assert P.shape == (r.n_users, P.shape[1]) and Q.shape == (r.n_items, P.shape[1])
        prm = _SgdParams(P.shape[1], n_epochs, lr, reg, mode, write_back)
        rc = r.c()
        self.check(lib().rs_svd_fit(self.h, C.byref(rc), C.byref(prm), _ptr(P), _ptr(Q),
                                    _ptr(bu), _ptr(bi), _ptr(g)))
        return P, Q, bu, bi, float(g[0])

    def svdpp_fit(self, r: Ratings, P, Q, Y, bu=None, bi=None, gb=0.0, n_epochs=20, lr=0.007,
                  reg=0.02, mode=SGD_FAST, write_back=WB_TILE):
        """core/svd.go:316-427 (ORDERED: literal per-rating y updates; FAST: the user-major lazy-y
        kernel)."""
        P = np.array(P, dtype=np.float64, order="C")
        Q = np.array(Q, dtype=np.float64, order="C")
        Y = np.array(Y, dtype=np.float64, order="C")
        bu = np.zeros(r.n_users) if bu is None else np.array(bu, dtype=np.float64)
        bi = np.zeros(r.n_items) if bi is None else np.array(bi, dtype=np.float64)
        g = np.array([gb], dtype=np.float64)
        prm = _SgdParams(P.shape[1], n_epochs, lr, reg, mode, write_back)
        rc = r.c()
        self.check(lib().rs_svdpp_fit(self.h, C.byref(rc), C.byref(prm), _ptr(P), _ptr(Q), _ptr(Y),
                                      _ptr(bu), _ptr(bi), _ptr(g)))
        return P, Q, Y, bu, bi, float(g[0])

    def nmf_fit(self, r: Ratings, P, Q, n_epochs=50, reg=0.06, as_written=True):
        """core/svd.go:158-251 (as_written reproduces svd.go:243-249, Q5)."""
        P = np.array(P, dtype=np.float64, order="C")
        Q = np.array(Q, dtype=np.float64, order="C")
        rc = r.c()
        self.check(lib().rs_nmf_fit(self.h, C.byref(rc), P.shape[1], n_epochs, reg,
                                    int(as_written), _ptr(P), _ptr(Q)))
        return P, Q

    def baseline_fit(self, r: Ratings, n_epochs=20, lr=0.005, reg=0.02):
        """core/base.go:135-163 BaseLine.Fit (exact reference order, float64)."""
        bu, bi, g = np.zeros(r.n_users), np.zeros(r.n_items), np.zeros(1)
        rc = r.c()
        self.check(lib().rs_baseline_fit(self.h, C.byref(rc), n_epochs, lr, reg, _ptr(bu),
                                         _ptr(bi), _ptr(g)))
        return bu, bi, float(g[0])

    def knn_sims(self, kind, rowptr, ids, ratings, n_right, part=0, n_parts=1, out=None):
        """core/knn.go:143-217 pair loop -> dense L x L float64 Sims (NaN = no co-rating).
        With n_parts > 1 only this part's entries of `out` (L x L, e.g. a shared memmap) are written
        (rs_knn_sims_part): the union over parts is the full matrix."""
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        ratings = np.ascontiguousarray(ratings, dtype=np.float64)
        L = len(rowptr) - 1
        if out is None:
            out = np.empty((L, L))
        if out.shape != (L, L) or out.dtype != np.float64 or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous L x L float64 array")
        self.check(lib().rs_knn_sims_part(self.h, kind, L, n_right, _ptr(rowptr), _ptr(ids),
                                          _ptr(ratings), part, n_parts, _ptr(out)))
        return out

    def sim_pair(self, kind, a_ids, a_r, b_ids, b_r):
        """core/sim.go Cosine / MSD / Pearson of two ID-ascending lists, on the device."""
        a_ids = np.ascontiguousarray(a_ids, dtype=np.int32)
        b_ids = np.ascontiguousarray(b_ids, dtype=np.int32)
        a_r = np.ascontiguousarray(a_r, dtype=np.float64)
        b_r = np.ascontiguousarray(b_r, dtype=np.float64)
        out = np.empty(1)
        self.check(lib().rs_sim_pair(self.h, kind, len(a_ids), _ptr(a_ids), _ptr(a_r),
                                     len(b_ids), _ptr(b_ids), _ptr(b_r), _ptr(out)))
        return float(out[0])

    def svd_plan(self, r: Ratings, n_factors: int) -> "SvdPlan":
        return SvdPlan(self, r, n_factors)

    def svd_plan_csr(self, n_users, n_items, rowptr, cols, vals, n_factors: int) -> "SvdPlan":
        return SvdPlan(self, None, n_factors, csr=(n_users, n_items, rowptr, cols, vals))

    def knn_plan(self, kind, rowptr, ids, ratings, n_right) -> "KnnPlan":
        return KnnPlan(self, kind, rowptr, ids, ratings, n_right)


class SvdPlan:
    """Device-resident user-CSR + factors (rs_svd_plan_*)."""

    def __init__(self, ctx: Context, r, n_factors: int, csr=None):
        """r: Ratings (COO), or None with csr = (n_users, n_items, rowptr, cols, vals float32)."""
        self.ctx = ctx
        h = C.c_void_p()
        self.h = None
        if csr is None:
            self.n_users, self.n_items, self.k = r.n_users, r.n_items, n_factors
            self.nnz = len(r.ratings)
            rc = r.c()
            ctx.check(lib().rs_svd_plan_create(ctx.h, C.byref(rc), n_factors, C.byref(h)))
        else:
            nu, ni, rowptr, cols, vals = csr
            rowptr = np.ascontiguousarray(rowptr, np.int64)
            cols = np.ascontiguousarray(cols, np.int32)
            vals = np.ascontiguousarray(vals, np.float32)
            self.n_users, self.n_items, self.k, self.nnz = nu, ni, n_factors, int(rowptr[nu])
            ctx.check(lib().rs_svd_plan_create_csr(ctx.h, nu, ni, _ptr(rowptr), _ptr(cols), _ptr(vals),
                                                   n_factors, C.byref(h)))
        self.h = h
        self._groups = weakref.WeakSet()  # SvdGroups over this plan: destroyed before it
        ctx._plans.add(self)

    def init_normal(self, mean=0.0, std=0.1, seed=1):
        """Device-side factor init (svd.go:77-85 distribution); GlobalBias = FAST warm start."""
        self.ctx.check(lib().rs_svd_plan_init_normal(self.h, mean, std, seed))

    def upload(self, P=None, Q=None, bu=None, bi=None, gb=None):
        arrs = [None if a is None else np.ascontiguousarray(a, dtype=np.float64)
                for a in (P, Q, bu, bi)]
        g = None if gb is None else np.array([gb], dtype=np.float64)
        self.ctx.check(lib().rs_svd_plan_upload(self.h, *[_ptr(a) for a in arrs], _ptr(g)))

    def download(self):
        P = np.empty((self.n_users, self.k))
        Q = np.empty((self.n_items, self.k))
        bu, bi, g = np.empty(self.n_users), np.empty(self.n_items), np.empty(1)
        self.ctx.check(lib().rs_svd_plan_download(self.h, _ptr(P), _ptr(Q), _ptr(bu), _ptr(bi),
                                                  _ptr(g)))
        return P, Q, bu, bi, float(g[0])

    def epochs(self, n, lr=0.005, reg=0.02, stream=None):
        self.ctx.check(lib().rs_svd_plan_epochs(self.h, n, lr, reg, stream))

    def set_mode(self, write_back=WB_TILE, ring_depth=16):
        self.ctx.check(lib().rs_svd_plan_set_mode(self.h, write_back, ring_depth))

    def set_user_blocks(self, n_blocks, bounds=None):
        """Tile schedule in n_blocks consecutive user blocks (rs_svd_plan_set_user_blocks); bounds:
        n_blocks + 1 user ids (None: from this plan's ratings)."""
        b = None if bounds is None else np.ascontiguousarray(bounds, np.int32)
        self.ctx.check(lib().rs_svd_plan_set_user_blocks(self.h, n_blocks, _ptr(b)))

    def set_exchange(self, mode=EXCHANGE_ROTATE):
        """Multi-GPU exchange a later join / group sets up (rs_svd_plan_set_exchange)."""
        self.ctx.check(lib().rs_svd_plan_set_exchange(self.h, mode))

    def set_qdelta_split(self, hot_ratings, cold_every):
        """RS_EXCHANGE_QDELTA's hot / cold split (rs_svd_plan_set_qdelta_split)."""
        self.ctx.check(lib().rs_svd_plan_set_qdelta_split(self.h, float(hot_ratings), int(cold_every)))

    def set_gb_fold(self, mode):
        """GB_FOLD_SMOOTH (default) or GB_FOLD_MEAN for single-GPU tile epochs (rs_svd_plan_set_gb_fold)."""
        self.ctx.check(lib().rs_svd_plan_set_gb_fold(self.h, int(mode)))

    def set_cold_store(self, runs_in_flight):
        """Cold runs end in write-through stores (rs_svd_plan_set_cold_store; 0 turns it off)."""
        self.ctx.check(lib().rs_svd_plan_set_cold_store(self.h, float(runs_in_flight)))

    def set_damp_concurrency(self, kconc):
        """Test hook: the hot-run damping with runs in flight R = deg x kconc (kconc > 0 forces the damped kernel;
        0 restores the library's rule; rs_svd_plan_set_damp_concurrency)."""
        self.ctx.check(lib().rs_svd_plan_set_damp_concurrency(self.h, float(kconc)))

    def set_qdelta_curvature(self, gamma):
        """RS_EXCHANGE_QDELTA's merge-weight curvature (rs_svd_plan_set_qdelta_curvature: a = 1 - lr x gamma)."""
        self.ctx.check(lib().rs_svd_plan_set_qdelta_curvature(self.h, float(gamma)))

    def set_qdelta_wire(self, bits):
        """RS_EXCHANGE_QDELTA's moves on the wire: 16 (fp16, default) or 32 (int32 fixed point; exact sums)."""
        self.ctx.check(lib().rs_svd_plan_set_qdelta_wire(self.h, bits))

    def time_blocks(self, n_blocks, lr=0.005, reg=0.02):
        """One epoch with every user block / stratum launched alone and timed: ms per block
        (rs_svd_plan_time_blocks; trains the model like an epoch)."""
        ms = np.zeros(n_blocks)
        self.ctx.check(lib().rs_svd_plan_time_blocks(self.h, lr, reg, _ptr(ms), n_blocks))
        return ms

    def set_hot_split(self, share=0.02, min_stratum=1 << 17, merge=0):
        """ROTATE_Q hot items split into per-block copies (rs_svd_plan_set_hot_split; merge 0 scaled, 1 average,
        2 sum of moves); before the join."""
        self.ctx.check(lib().rs_svd_plan_set_hot_split(self.h, share, min_stratum, merge))

    def inject_fault(self, sub_epoch):
        """Test hook: the next sharded call throws at that sub-epoch, once (rs_svd_plan_inject_fault)."""
        self.ctx.check(lib().rs_svd_plan_inject_fault(self.h, sub_epoch))

    def join(self, comm_id: bytes, rank: int, n_ranks: int, n_blocks: int = 0):
        """Item-sharded multi-GPU (rs_svd_plan_join; collective over the ranks): comm_id from
        comm_unique_id() on rank 0, sent to every rank."""
        assert len(comm_id) == COMM_ID_BYTES
        buf = C.create_string_buffer(bytes(comm_id), COMM_ID_BYTES)
        self.ctx.check(lib().rs_svd_plan_join(self.h, buf, rank, n_ranks, n_blocks))

    def shard_info(self):
        """(rank, n_ranks, exchange, user blocks) of a joined plan; ranks from the RCCL communicator."""
        v = [_i32(0) for _ in range(4)]
        self.ctx.check(lib().rs_svd_plan_shard_info(self.h, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def qdelta_info(self):
        """(hot items, blocks between full merges) of a plan joined with EXCHANGE_QDELTA."""
        v = [_i32(0) for _ in range(2)]
        self.ctx.check(lib().rs_svd_plan_qdelta_info(self.h, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def epochs_sharded(self, n, lr=0.005, reg=0.02, stream=None):
        self.ctx.check(lib().rs_svd_plan_epochs_sharded(self.h, n, lr, reg, stream))

    def leave(self):
        self.ctx.check(lib().rs_svd_plan_leave(self.h))

    def set_tiles(self, workgroups=0, waves=16, target=0, run_cap=0, ring=0):
        """WB_TILE schedule parameters (rs_svd_plan_set_tiles); rebuilds the tiles."""
        self.ctx.check(lib().rs_svd_plan_set_tiles(self.h, workgroups, waves, target, run_cap, ring))

    def set_tile_rule(self, rule):
        """TILE_RULE_LPT / _SNAKE / _SNAKE_DEVICE (rs_svd_plan_set_tile_rule); rebuilds the tiles."""
        self.ctx.check(lib().rs_svd_plan_set_tile_rule(self.h, rule))

    def set_guard(self, on=True):
        """Divergence guard of the tile schedule (rs_svd_plan_set_guard; default on)."""
        self.ctx.check(lib().rs_svd_plan_set_guard(self.h, int(bool(on))))

    def refits(self):
        v = _i32(0)
        self.ctx.check(lib().rs_svd_plan_refits(self.h, C.byref(v)))
        return v.value

    def fixed_point(self):
        """The fixed-point shift S of the FAST kernels (rs_svd_plan_fixed_point)."""
        v = _i32(0)
        self.ctx.check(lib().rs_svd_plan_fixed_point(self.h, C.byref(v)))
        return v.value

    def tile_rule(self):
        v = _i32(0)
        self.ctx.check(lib().rs_svd_plan_tile_rule(self.h, C.byref(v)))
        return v.value

    def schedule_digest(self):
        """64-bit digest of the tile schedule in HBM (rs_svd_plan_schedule_digest)."""
        v = C.c_uint64(0)
        self.ctx.check(lib().rs_svd_plan_schedule_digest(self.h, C.byref(v)))
        return v.value

    def set_tile_claim(self, runs_per_claim=4):
        """Runs per claim from a tile's run queue (4, 8), or 0: runs dealt on the host
        (rs_svd_plan_set_tile_claim); rebuilds the tiles."""
        self.ctx.check(lib().rs_svd_plan_set_tile_claim(self.h, runs_per_claim))

    def tile_order(self):
        """(pos, work_off): user-CSR positions in the tile schedule's visit order and the boundaries
        of its (tile, wave) GlobalBias work items (rs_svd_plan_tile_order)."""
        nw = _i32(0)
        self.ctx.check(lib().rs_svd_plan_tile_order(self.h, None, None, C.byref(nw)))
        pos = np.empty(self.nnz, np.int64)
        off = np.empty(nw.value + 1, np.int64)
        self.ctx.check(lib().rs_svd_plan_tile_order(self.h, pos.ctypes.data, off.ctypes.data, C.byref(nw)))
        return pos, off

    def set_schedule(self, heavy_min=1024, light_blocks=-1):
        """WB_ATOMIC schedule: items with >= heavy_min ratings get a producer wave + 3 writer waves;
        light items stride over light_blocks blocks (-1: 1.5 per CU, 0: one wave per item)."""
        self.ctx.check(lib().rs_svd_plan_set_schedule(self.h, heavy_min, light_blocks))

    def trace(self, n_work=None):
        """Diagnostic timeline: trace() enables it; trace(n_work) returns (ticks[n_work, 3], users)
        of the last epoch (n_work = the plan's work items: its non-empty users when not split)."""
        if n_work is None:
            self.ctx.check(lib().rs_svd_plan_trace(self.h, None, None))
            return None
        n = n_work
        t = np.zeros((n, 3), np.int64)
        u = np.zeros(n, np.int32)
        self.ctx.check(lib().rs_svd_plan_trace(self.h, t.ctypes.data, u.ctypes.data))
        return t, u

    def set_split(self, split_cap):
        self.ctx.check(lib().rs_svd_plan_set_split(self.h, split_cap))

    def set_fixed_q(self, on=True):
        """Hybrid FAST epochs keep Q as int32 fixed point (2^-24) with integer atomics."""
        self.ctx.check(lib().rs_svd_plan_set_fixed_q(self.h, 1 if on else 0))

    def set_hot_replicas(self, n_hot, copies=4):
        """Live-merged row copies for the n_hot most-rated items (0 = none)."""
        self.ctx.check(lib().rs_svd_plan_set_hot_replicas(self.h, n_hot, copies))

    def set_item_split(self, item_cap):
        self.ctx.check(lib().rs_svd_plan_set_item_split(self.h, item_cap))

    def device_ptrs(self):
        ps = [C.c_void_p() for _ in range(3)]
        ld = _i32(0)
        self.ctx.check(lib().rs_svd_plan_device_ptrs(self.h, *[C.byref(p) for p in ps],
                                                     C.byref(ld)))
        return [p.value for p in ps], ld.value

    def set_user_weights(self, w):
        self._w = None if w is None else np.ascontiguousarray(w, dtype=np.float32)
        self.ctx.check(lib().rs_svd_plan_set_user_weights(self.h, _ptr(self._w)))

    def epoch_delta(self, dP_ptr, gbsum_ptr, lr=0.005, reg=0.02, stream=None):
        """Device pointers (ints): dP n_users x ld float32, gbsum one float64."""
        self.ctx.check(lib().rs_svd_plan_epoch_delta(self.h, lr, reg, dP_ptr, gbsum_ptr, stream))

    def apply_delta(self, dP_ptr, gbsum_ptr, inv_total_nnz, stream=None):
        self.ctx.check(lib().rs_svd_plan_apply_delta(self.h, dP_ptr, gbsum_ptr, inv_total_nnz,
                                                     stream))

    def set_item_weights(self, w):
        self._iw = None if w is None else np.ascontiguousarray(w, dtype=np.float32)
        self.ctx.check(lib().rs_svd_plan_set_item_weights(self.h, _ptr(self._iw)))

    def epoch_qdelta_t(self, dQ, gbsum, lr, reg, stream=None):
        """User-sharded mode: dQ (torch, n_items x ld fp32), gbsum (torch, 1 float64).  stream None:
        torch's current stream on dQ's device, so the kernels are ordered with the collectives
        torch enqueues there (the library's own ctx stream is not)."""
        stream = _torch_stream(dQ) if stream is None else stream
        self.ctx.check(lib().rs_svd_plan_epoch_qdelta(self.h, lr, reg, dQ.data_ptr(), gbsum.data_ptr(),
                                                      stream))

    def apply_qdelta_t(self, dQ, gbsum, inv_total_nnz, stream=None):
        stream = _torch_stream(dQ) if stream is None else stream
        self.ctx.check(lib().rs_svd_plan_apply_qdelta(self.h, dQ.data_ptr(), gbsum.data_ptr(),
                                                      inv_total_nnz, stream))

    # torch-tensor forms used by rsgpu.multi.ItemShardedStep
    def epoch_delta_t(self, dP, gbsum, lr, reg, stream=None):
        stream = _torch_stream(dP) if stream is None else stream  # ordered with torch's collectives
        self.epoch_delta(dP.data_ptr(), gbsum.data_ptr(), lr, reg, stream)

    def apply_delta_t(self, dP, gbsum, inv_total_nnz, stream=None):
        stream = _torch_stream(dP) if stream is None else stream
        self.apply_delta(dP.data_ptr(), gbsum.data_ptr(), inv_total_nnz, stream)

    @property
    def ld(self):
        return self.device_ptrs()[1]

    def set_timing(self, on: bool):
        self.ctx.check(lib().rs_svd_plan_set_timing(self.h, int(on)))

    def last_kernel_ms(self):
        ms, n = _dbl(0), _i32(0)
        self.ctx.check(lib().rs_svd_plan_last_kernel_ms(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def predict(self, users, items):
        """svd.go:32-51 on the device factors for inner-id pairs (-1 = unknown)."""
        u, i = np.ascontiguousarray(users, np.int32), np.ascontiguousarray(items, np.int32)
        out = np.empty(len(u))
        self.ctx.check(lib().rs_svd_plan_predict(self.h, len(u), _ptr(u), _ptr(i), _ptr(out)))
        return out

    def evaluate(self, users, items, ratings):
        """(RMSE, MAE) over a test set (utils.go:162-180) on the device."""
        u, i = np.ascontiguousarray(users, np.int32), np.ascontiguousarray(items, np.int32)
        r = np.ascontiguousarray(ratings, np.float64)
        a, b = _dbl(0), _dbl(0)
        self.ctx.check(lib().rs_svd_plan_evaluate(self.h, len(u), _ptr(u), _ptr(i), _ptr(r),
                                                  C.byref(a), C.byref(b)))
        return a.value, b.value

    def close(self):
        if self.h:
            for g in list(self._groups):  # a group holds the plan's shard state: it goes first
                g.close()
            lib().rs_svd_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id() -> bytes:
    """RS_COMM_ID_BYTES bytes naming a new RCCL communicator (rank 0 sends them to every rank)."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(lib().rs_comm_unique_id(buf))
    return buf.raw


def rotation_step(rank, n_ranks, sub_epoch):
    """(rank-block trained, send-to rank, rank-block received, recv-from rank) of the ROTATE exchange's
    sub-epoch (rs_rotation_step; host only)."""
    out = np.zeros(4, np.int32)
    _check(lib().rs_rotation_step(rank, n_ranks, sub_epoch, _ptr(out)))
    return tuple(int(x) for x in out)


def comm_info():
    """(RCCL version code, path of the librccl this process runs against) (rs_comm_info)."""
    v = _i32(0)
    buf = C.create_string_buffer(4096)
    _check(lib().rs_comm_info(C.byref(v), buf, 4096))
    return v.value, buf.value.decode()


def tile_schedule_host(n_users, n_items, rowptr, cols, vals, n_factors, workgroups=256, waves=16,
                       n_blocks=1, want_pos=False):
    """Host-only tile schedule build (rs_tile_schedule_host): (ms, n_tiles, pos or None)."""
    rowptr = np.ascontiguousarray(rowptr, np.int64)
    cols = np.ascontiguousarray(cols, np.int32)
    vals = np.ascontiguousarray(vals, np.float32)
    nnz = int(rowptr[-1])
    pos = np.empty(nnz, np.int64) if want_pos else None
    nt, ms = _i32(0), _dbl(0)
    _check(lib().rs_tile_schedule_host(n_users, n_items, _ptr(rowptr), _ptr(cols), _ptr(vals), n_factors,
                                       workgroups, waves, n_blocks, 0, _ptr(pos), None, None,
                                       C.byref(nt), C.byref(ms)))
    return ms.value, nt.value, pos


def item_shards(items, n_items, n_shards):
    """Item ranges of near-equal ratings (rs_item_shards): bounds, n_shards + 1 entries."""
    items = np.ascontiguousarray(items, np.int32)
    b = np.empty(n_shards + 1, np.int32)
    _check(lib().rs_item_shards(len(items), _ptr(items), n_items, n_shards, _ptr(b)))
    return b


class SvdGroup:
    """Several shard plans driven by one process (rs_svd_group_*): RCCL when each plan has its own
    device, else the in-process exchange."""

    def __init__(self, plans, n_blocks=0):
        self.plans = list(plans)
        arr = (C.c_void_p * len(self.plans))(*[p.h for p in self.plans])
        h = C.c_void_p()
        self.h = None
        _check(lib().rs_svd_group_create(arr, len(self.plans), n_blocks, C.byref(h)))
        self.h = h
        for p in self.plans:
            p._groups.add(self)

    def epochs(self, n, lr=0.005, reg=0.02):
        _check(lib().rs_svd_group_epochs(self.h, n, lr, reg))

    def close(self):
        if self.h is not None:
            lib().rs_svd_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def svd_fit_multi(devices, r: "Ratings", P, Q, bu=None, bi=None, gb=0.0, n_epochs=20, lr=0.005,
                  reg=0.02, n_blocks=0):
    """rs_svd_fit_multi: core/svd.go:63-132 over item shards on `devices` (one host thread each)."""
    P = np.array(P, dtype=np.float64, order="C")
    Q = np.array(Q, dtype=np.float64, order="C")
    bu = np.zeros(r.n_users) if bu is None else np.array(bu, dtype=np.float64)
    bi = np.zeros(r.n_items) if bi is None else np.array(bi, dtype=np.float64)
    g = np.array([gb], dtype=np.float64)
    dev = np.ascontiguousarray(devices, np.int32)
    prm = _SgdParams(P.shape[1], n_epochs, lr, reg, SGD_FAST, WB_TILE)
    rc = r.c()
    rep = _Report()
    code = lib().rs_svd_fit_multi(_ptr(dev), len(dev), C.byref(rc), C.byref(prm), n_blocks, _ptr(P), _ptr(Q),
                                  _ptr(bu), _ptr(bi), _ptr(g), C.byref(rep))
    _last_multi.refits = rep.refits
    if code != RS_OK:
        raise RsError(code, rep.error.decode(errors="replace"))
    return P, Q, bu, bi, float(g[0])


_last_multi = threading.local()


def fit_multi_refits():
    """Refits of this thread's last svd_fit_multi (its rs_report's refits)."""
    return getattr(_last_multi, "refits", 0)


def svd_predict(users, items, P, Q, bu, bi, gb):
    u = np.ascontiguousarray(users, dtype=np.int32)
    i = np.ascontiguousarray(items, dtype=np.int32)
    P, Q = np.ascontiguousarray(P, np.float64), np.ascontiguousarray(Q, np.float64)
    bu, bi = np.ascontiguousarray(bu, np.float64), np.ascontiguousarray(bi, np.float64)
    out = np.empty(len(u))
    _check(lib().rs_svd_predict(None, len(u), _ptr(u), _ptr(i), P.shape[0], Q.shape[0],
                                P.shape[1], _ptr(P), _ptr(Q), _ptr(bu), _ptr(bi), gb, _ptr(out)))
    return out


class KnnPlan:
    """Device-resident KNN similarities with Predict on the device (rs_knn_plan_*)."""

    TYPES = {"basic": 0, "centered": 1, "zscore": 2, "baseline": 3}

    def __init__(self, ctx: Context, kind, rowptr, ids, ratings, n_right):
        self.ctx = ctx
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        ratings = np.ascontiguousarray(ratings, dtype=np.float64)
        self.L = len(rowptr) - 1
        h = C.c_void_p()
        self.h = None
        ctx.check(lib().rs_knn_plan_create(ctx.h, kind, self.L, n_right, _ptr(rowptr), _ptr(ids),
                                           _ptr(ratings), C.byref(h)))
        self.h = h
        ctx._plans.add(self)

    def sims(self):
        out = np.empty((self.L, self.L))
        self.ctx.check(lib().rs_knn_plan_sims(self.h, _ptr(out)))
        return out

    def set_tie_order(self, tie=0):
        """TIE_GO_SORT (default: knn.go:107-108's sort.Sort order) or TIE_STABLE (rs_knn_plan_set_tie_order)."""
        self.ctx.check(lib().rs_knn_plan_set_tie_order(self.h, tie))

    def predict(self, knn_type, right_rowptr, right_ids, right_r, left, right, global_mean,
                means=None, stddevs=None, bias=None, k=40, min_k=1):
        """core/knn.go:75-141 for (left, right) inner-id pairs on the device."""
        t = self.TYPES[knn_type] if isinstance(knn_type, str) else int(knn_type)
        rp = np.ascontiguousarray(right_rowptr, dtype=np.int64)
        ri = np.ascontiguousarray(right_ids, dtype=np.int32)
        rr = np.ascontiguousarray(right_r, dtype=np.float64)
        lq = np.ascontiguousarray(left, dtype=np.int32)
        rq = np.ascontiguousarray(right, dtype=np.int32)
        arrs = [None if a is None else np.ascontiguousarray(a, dtype=np.float64)
                for a in (means, stddevs, bias)]
        out = np.empty(len(lq))
        self.ctx.check(lib().rs_knn_plan_predict(self.h, t, len(rp) - 1, _ptr(rp), _ptr(ri), _ptr(rr),
                                                 *[_ptr(a) for a in arrs], float(global_mean), k, min_k,
                                                 len(lq), _ptr(lq), _ptr(rq), _ptr(out)))
        return out

    def slope_one_predict(self, user_rowptr, user_items, user_ratings, global_mean, users, items):
        """slope_one.go:21-45 on the device dev matrix (plan kind DEV_SLOPE_ONE); user CSR in data order."""
        rp = np.ascontiguousarray(user_rowptr, np.int64)
        it = np.ascontiguousarray(user_items, np.int32)
        rr = np.ascontiguousarray(user_ratings, np.float64)
        u, i = np.ascontiguousarray(users, np.int32), np.ascontiguousarray(items, np.int32)
        out = np.empty(len(u))
        self.ctx.check(lib().rs_slope_one_predict(self.h, len(rp) - 1, _ptr(rp), _ptr(it), _ptr(rr),
                                                  global_mean, len(u), _ptr(u), _ptr(i), _ptr(out)))
        return out

    def close(self):
        if self.h:
            lib().rs_knn_plan_destroy(self.h)
            self.h = None
