"""Experiment: RMSE cost of splitting heavy users into pseudo-users whose rows are merged (count-
weighted average of p and b_u) after every epoch, on 5-fold ML-100K (k=100, 20 epochs), FAST kernel."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tests"), os.path.join(REPO, "scripts")]
import oracle as O  # noqa: E402
import rsgpu  # noqa: E402
from helpers import folds, rmse  # noqa: E402
from exp_split import split_users  # noqa: E402

ctx = rsgpu.Context(0)
d = np.load(os.path.join(REPO, "tests/golden/ml100k.npz"))
U, I, R = d["users"].astype(np.int64), d["ratings"].astype(np.float64), None
U, I, R = d["users"].astype(np.int64), d["items"].astype(np.int64), d["ratings"].astype(np.float64)
k = 100
for cap in (0, 400, 200, 100, 50):
    res = []
    for f in folds(U, I, R):
        rng = np.random.default_rng(7)
        P0, Q0 = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
        if cap:
            pu, npu = split_users(f.iu, cap)
            owner = np.zeros(npu, np.int64)
            owner[pu] = f.iu
            cnt = np.bincount(pu, minlength=npu).astype(float)
        else:
            pu, npu, owner, cnt = f.iu, f.nu, np.arange(f.nu), np.bincount(f.iu, minlength=f.nu).astype(float)
        rowptr, items, rr = O.csr_by(f.iu, f.nu, f.ii, f.r)
        gb = O.gb_warm_start(rowptr, items, rr, np.zeros(f.nu), np.zeros(f.ni))
        plan = ctx.svd_plan(rsgpu.Ratings(pu, f.ii, f.r, npu, f.ni), k)
        P, bu = P0, np.zeros(f.nu)
        Q, bi = Q0, np.zeros(f.ni)
        for ep in range(20):
            plan.upload(P[owner], Q, bu[owner], bi, gb)
            plan.epochs(1)
            Pp, Q, bup, bi, gb = plan.download()
            tot = np.bincount(owner, weights=cnt, minlength=f.nu)
            P = np.zeros((f.nu, k))
            np.add.at(P, owner, Pp * cnt[:, None])
            P /= np.maximum(tot, 1)[:, None]
            bu = np.bincount(owner, weights=bup * cnt, minlength=f.nu) / np.maximum(tot, 1)
        plan.close()
        res.append(rmse(rsgpu.svd_predict(f.tu, f.ti, P, Q, bu, bi, gb), f.te_r))
    print(f"cap={cap:4d} cv_rmse={np.mean(res):.4f} folds={np.round(res, 4).tolist()}", flush=True)
