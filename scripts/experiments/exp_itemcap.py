"""Experiment: ML-1M-shaped set, k=100 -- epoch time and held-out RMSE (90/10 split, 20 epochs)
per (user split_cap, item_cap)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu
from rsgpu import synth
ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
n = len(r)
te = np.zeros(n, bool)
te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
tr = ~te
rng = np.random.default_rng(5)
P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
for ucap, icap in [(256, 0), (0, 0), (256, 2048), (256, 1024), (256, 512), (256, 384), (256, 256)]:
    plan = ctx.svd_plan(rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni), 100)
    plan.set_split(ucap)
    plan.set_item_split(icap)
    plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), float(np.mean(r[tr])))
    plan.epochs(1)
    plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), float(np.mean(r[tr])))
    plan.set_timing(True)
    plan.epochs(20)
    ms, k = plan.last_kernel_ms()
    P, Q, bu, bi, gb = plan.download()
    plan.close()
    e = np.sqrt(np.mean((rsgpu.svd_predict(u[te], i[te], P, Q, bu, bi, gb) - r[te]) ** 2))
    print(f"user_cap={ucap:4d} item_cap={icap:4d} sgd_kernel_us={ms / k * 1e3:7.1f} holdout_rmse={e:.4f}", flush=True)
