"""Experiment: what bounds the FAST atomic SGD epoch on the ML-1M-shaped set?
  full      the bench set as is (Zipf items, heaviest user 2314 ratings)
  split200  same ratings, every user cut into pseudo-users of <= 200 ratings (no long chains)
  uniform   split200 with items redrawn uniformly (no hot rows)"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu
from rsgpu import synth



def split_users(u, cap):
    order = np.argsort(u, kind="stable")
    su = u[order]
    starts = np.r_[0, np.flatnonzero(np.diff(su)) + 1]
    rank = np.arange(len(su)) - np.repeat(starts, np.diff(np.r_[starts, len(su)]))
    pseudo = np.zeros(len(u), np.int64)
    key = su.astype(np.int64) * 100000 + rank // cap
    _, inv = np.unique(key, return_inverse=True)
    pseudo[order] = inv
    return pseudo.astype(np.int32), int(inv.max()) + 1


def run(name, uu, ii, n_u, wb=0):
    plan = ctx.svd_plan(rsgpu.Ratings(uu, ii, r, n_u, ni), 100)
    plan.set_mode(wb, 8)
    plan.upload(rng.normal(0, 0.1, (n_u, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(n_u), np.zeros(ni), 3.58)
    plan.set_timing(True)
    plan.epochs(5)
    ms, n = plan.last_kernel_ms()
    plan.close()
    print(f"{name:24s} wb={wb} users={n_u} epoch_us={ms / n * 1e3:8.1f}", flush=True)

if __name__ == "__main__":
    ctx = rsgpu.Context(0)
    u, i, r, nu, ni = synth.ml1m_like()
    rng = np.random.default_rng(5)
    run("full", u, i, nu)
    for cap in (400, 200, 100, 50):
        pu, npu = split_users(u, cap)
        run(f"split{cap}", pu, i, npu)
    pu, npu = split_users(u, 200)
    iu = rng.integers(0, ni, len(u)).astype(np.int32)
    run("split200-uniform", pu, iu, npu)
    run("full-uniform", u, iu, nu)
    run("split200 store", pu, i, npu, wb=1)
    run("split200-uniform store", pu, iu, npu, wb=1)
