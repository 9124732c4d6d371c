"""Experiment: per-work-item timeline of one FAST epoch (ML-1M shape) under RS_SGD_WB_ATOMIC,
for a few heavy thresholds: when do the heavy users finish, how long are light users' chains."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
deg = np.bincount(u, minlength=nu)
nw = int((deg > 0).sum())
warm = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)  # first plan of a process runs slow
warm.upload(np.zeros((nu, 100)), np.zeros((ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
warm.epochs(5)
warm.download()
warm.close()
for heavy in [int(x) for x in os.environ.get("HEAVY", "0,512").split(",")]:
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
    plan.set_mode(int(os.environ.get("WB", "0")), 8)
    plan.set_schedule(heavy, int(os.environ.get('RSGPU_LIGHT_BLOCKS', '-1')))
    rng = np.random.default_rng(1)
    plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
    plan.trace()
    plan.epochs(5)
    t, wu = plan.trace(nw)
    plan.close()
    t = (t - t[:, 0].min()) / 100.0  # us
    d = deg[wu]
    end = t[:, 2]
    print(f"heavy={heavy}: epoch span {end.max():.0f} us; start max {t[:, 0].max():.0f} us")
    for q in (0.5, 0.9, 0.99, 1.0):
        print(f"   end quantile {q}: {np.quantile(end, q):.0f} us")
    top = np.argsort(-d)[:8]
    for w in top:
        print(f"   deg {d[w]:5d}: start {t[w, 0]:6.0f} chain end {t[w, 1]:6.0f} drained {t[w, 2]:6.0f} "
              f"-> {1e3 * (t[w, 1] - t[w, 0]) / d[w]:.0f} ns/rating")
    # chain rate of light users by degree band
    rate = (t[:, 1] - t[:, 0]) / np.maximum(d, 1) * 1e3
    for lo, hi in ((20, 50), (50, 150), (150, 400), (400, 1000)):
        m = (d >= lo) & (d < hi)
        if m.any():
            print(f"   deg [{lo},{hi}): n={m.sum()} median {np.median(rate[m]):.0f} ns/rating, "
                  f"median start {np.median(t[m, 0]):.0f} us, median end {np.median(end[m]):.0f} us")
    sys.stdout.flush()
