"""Experiment: user splitting (rs_svd_plan_set_split) together with the heavy threshold
(rs_svd_plan_set_schedule) and fixed-point Q, on the ML-1M shape, k=100, hot replicas at their
default: epoch time (timing mode) and 20-epoch held-out RMSE (90/10 split, same init).
CFGS = "split:heavy:fx[:ring_depth],..."."""
import os
import sys

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
cfgs = [tuple(int(v) for v in c.split(":")) for c in
        os.environ.get("CFGS", "0:1024:0,0:1024:1,1200:1000:1,800:700:1,600:500:1,400:350:1").split(",")]


def setup(plan, split, heavy, fx, depth=8):
    plan.set_mode(rsgpu.WB_ATOMIC, depth)
    plan.set_split(split)
    plan.set_schedule(heavy, -1)
    plan.set_fixed_q(fx)


for cfg in cfgs:
    split, heavy, fx = cfg[:3]
    depth = cfg[3] if len(cfg) > 3 else 8
    plan = ctx.svd_plan(R_all, 100)
    setup(plan, split, heavy, fx, depth)
    plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), float(np.mean(r)))
    plan.epochs(3)
    best = 1e9
    for _ in range(3):
        plan.set_timing(True)
        plan.epochs(5)
        ms, k = plan.last_kernel_ms()
        best = min(best, ms / k * 1e3)
    plan.close()
    plan = ctx.svd_plan(R_tr, 100)
    setup(plan, split, heavy, fx, depth)
    plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), gb0)
    plan.epochs(20)
    e = plan.evaluate(u[te], i[te], r[te])[0]
    plan.close()
    print(f"split={split:5d} heavy={heavy:5d} fx={fx} depth={depth} epoch_us={best:8.1f} held-out RMSE {e:.4f}", flush=True)
