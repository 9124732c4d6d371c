"""Experiment: fixed-point item rows (rs_svd_plan_set_fixed_q) on the ML-1M shape, k=100 -- epoch
time (timing mode: conversions included) and 20-epoch held-out RMSE (90/10 split, same init) with
fp32 and with int32 Q, hot replicas at their default; plus the bench's ML-1M-shaped full set."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
n = len(r)
te = np.zeros(n, bool)
te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
tr = ~te
rng = np.random.default_rng(5)
P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
R_tr = rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni)
R_all = rsgpu.Ratings(u, i, r, nu, ni)
gb0 = float(np.mean(r[tr]))
for rep in range(2):
    for fx in (0, 1):
        plan = ctx.svd_plan(R_all, 100)
        plan.set_fixed_q(fx)
        plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), float(np.mean(r)))
        plan.epochs(3)
        best = 1e9
        for _ in range(3):
            plan.set_timing(True)
            plan.epochs(5)
            ms, k = plan.last_kernel_ms()
            best = min(best, ms / k * 1e3)
        plan.close()
        t0 = time.time()
        plan = ctx.svd_plan(R_tr, 100)
        plan.set_fixed_q(fx)
        plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), gb0)
        plan.epochs(20)
        e = plan.evaluate(u[te], i[te], r[te])[0]
        Pd, Qd, bu, bi, gb = plan.download()
        plan.close()
        print(f"fixed_q={fx} epoch_us={best:8.1f} held-out RMSE {e:.4f} max|Q|={np.abs(Qd).max():.3f} "
              f"max|P|={np.abs(Pd).max():.3f} ({time.time() - t0:.1f} s)", flush=True)
