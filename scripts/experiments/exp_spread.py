"""Experiment: is the Zipf penalty of the FAST atomic epoch hot-row serialization?  The ML-1M-shaped
set with each of the top-H items' ratings spread over R distinct item ids (round-robin by user),
which is what R replicas of a hot row would do to the atomic traffic (without their read cost)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu
from rsgpu import synth
ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
rng = np.random.default_rng(5)
deg_i = np.bincount(i, minlength=ni)
order = np.argsort(-deg_i, kind="stable")


def run(name, ii, n_i):
    plan = ctx.svd_plan(rsgpu.Ratings(u, ii, r, nu, n_i), 100)
    plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (n_i, 100)), np.zeros(nu), np.zeros(n_i), 3.58)
    plan.epochs(1)
    plan.set_timing(True)
    plan.epochs(5)
    ms, n = plan.last_kernel_ms()
    plan.close()
    print(f"{name:28s} items={n_i} epoch_us={ms / n * 1e3:8.1f}", flush=True)


run("zipf", i, ni)
for H in (16, 64, 256):
    for R in (2, 4, 8):
        hot = order[:H]
        slot = np.full(ni, -1)
        slot[hot] = np.arange(H)
        ii = i.copy().astype(np.int64)
        m = slot[i] >= 0
        ii[m] = ni + slot[i[m]] * R + (u[m] % R)   # replicas appended after the original ids
        run(f"spread top{H} x{R}", ii.astype(np.int32), ni + H * R)
