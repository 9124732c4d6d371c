"""Experiment: fast-mode RMSE on 5-fold ML-100K and ML-1M-shape epoch time per write-back mode."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import rsgpu
from rsgpu import synth
from helpers import folds, rmse
d = np.load(os.path.join(REPO, "tests/golden/ml100k.npz"))
U, I, R = d["users"].astype(np.int64), d["items"].astype(np.int64), d["ratings"].astype(np.float64)
fs = folds(U, I, R)
ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
rings = [int(x) for x in os.environ.get("RINGS", "4,8,16").split(",")]
wbs = [int(x) for x in os.environ.get("WBS", "0,1").split(",")]
for wb in wbs:
    res = []
    for f in fs:
        rng = np.random.default_rng(7)
        P0, Q0 = rng.normal(0, 0.1, (f.nu, 100)), rng.normal(0, 0.1, (f.ni, 100))
        b = ctx.svd_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, write_back=wb)
        res.append(rmse(rsgpu.svd_predict(f.tu, f.ti, *b), f.te_r))
    for ring in rings:
        plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
        plan.set_mode(wb, ring)
        rng = np.random.default_rng(1)
        plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
        plan.set_timing(True)
        plan.epochs(20)
        ms, n = plan.last_kernel_ms()
        P, Q, bu, bi, gb = plan.download()
        tr = rmse(rsgpu.svd_predict(u, i, P, Q, bu, bi, gb), r)
        plan.close()
        print(f"wb={wb} ring={ring} ml100k_cv_rmse={np.mean(res):.4f} ml1m_epoch_us={ms/n*1e3:.1f} upd/s={len(r)/(ms/n/1e3):.3e} train_rmse20={tr:.4f}", flush=True)
