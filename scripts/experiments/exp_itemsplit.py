"""Experiment: RMSE cost of splitting hot ITEMS into pseudo-items (ratings dealt by position in the
user-CSR order) whose rows are merged by count-weighted average after every epoch, on 5-fold
ML-100K (k=100, 20 epochs, FAST kernel, default user split).  Also prints the ML-1M-shaped item
degree profile (how many items a cap would split)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"),
                os.path.join(REPO, "tests")]
import oracle as O  # noqa: E402
import rsgpu  # noqa: E402
from helpers import folds, rmse  # noqa: E402
from rsgpu import synth  # noqa: E402


def split_items(u, i, n_items, cap):
    """Pseudo-item id per rating and owner / count arrays (piece c of item x gets ratings
    c*d/R .. (c+1)*d/R in user-CSR order)."""
    order = np.lexsort((np.arange(len(u)), u))  # user-CSR order, stable
    d = np.bincount(i, minlength=n_items)
    R = np.maximum(1, -(-d // cap)) if cap else np.ones(n_items, np.int64)
    seen = np.zeros(n_items, np.int64)
    piece = np.zeros(len(u), np.int64)
    for t in order:
        x = i[t]
        piece[t] = seen[x] * R[x] // d[x]
        seen[x] += 1
    first = np.concatenate([[0], np.cumsum(R)[:-1]])
    pid = first[i] + piece
    owner = np.repeat(np.arange(n_items), R)
    cnt = np.bincount(pid, minlength=int(R.sum())).astype(float)
    return pid.astype(np.int32), int(R.sum()), owner, cnt


if __name__ == "__main__":
    _, i1, _, _, ni1 = synth.ml1m_like()
    d1 = np.sort(np.bincount(i1, minlength=ni1))[::-1]
    for cap in (256, 512, 1024):
        m = d1 > cap
        print(f"ml1m items with deg > {cap}: {m.sum()} holding {d1[m].sum() / d1.sum():.2f} of ratings")
    ctx = rsgpu.Context(0)
    d = np.load(os.path.join(REPO, "tests/golden/ml100k.npz"))
    U, I, R = d["users"].astype(np.int64), d["items"].astype(np.int64), d["ratings"].astype(np.float64)
    k = 100
    for cap in (0, 512, 256, 128, 64):
        res = []
        for f in folds(U, I, R):
            rng = np.random.default_rng(7)
            P, Q = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
            pid, npi, owner, cnt = split_items(f.iu, f.ii, f.ni, cap)
            rowptr, items, rr = O.csr_by(f.iu, f.nu, f.ii, f.r)
            gb = O.gb_warm_start(rowptr, items, rr, np.zeros(f.nu), np.zeros(f.ni))
            plan = ctx.svd_plan(rsgpu.Ratings(f.iu, pid, f.r, f.nu, npi), k)
            bu, bi = np.zeros(f.nu), np.zeros(f.ni)
            for ep in range(20):
                plan.upload(P, Q[owner], bu, bi[owner], gb)
                plan.epochs(1)
                P, Qp, bu, bip, gb = plan.download()
                tot = np.bincount(owner, weights=cnt, minlength=f.ni)
                Q = np.zeros((f.ni, k))
                np.add.at(Q, owner, Qp * cnt[:, None])
                Q /= np.maximum(tot, 1)[:, None]
                bi = np.bincount(owner, weights=bip * cnt, minlength=f.ni) / np.maximum(tot, 1)
            plan.close()
            res.append(rmse(rsgpu.svd_predict(f.tu, f.ti, P, Q, bu, bi, gb), f.te_r))
        print(f"item cap={cap:4d} pieces={npi - f.ni:4d} cv_rmse={np.mean(res):.4f}", flush=True)
