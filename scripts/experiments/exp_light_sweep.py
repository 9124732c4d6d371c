"""Experiment: light-path knobs on the end-of-round-1 default schedule (ML-1M shape, k=100): ring
depth (rs_svd_plan_set_mode) x light blocks (rs_svd_plan_set_schedule), epoch time in timing mode.
CFGS = "depth:light_blocks,..." (light_blocks -1 = 1.5 per CU)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
rng = np.random.default_rng(5)
P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
R_all = rsgpu.Ratings(u, i, r, nu, ni)
cfgs = [tuple(int(v) for v in c.split(":")) for c in
        os.environ.get("CFGS", "8:-1,16:-1,4:-1,8:256,8:512,16:512,8:768,16:768").split(",")]
for depth, lb in cfgs:
    plan = ctx.svd_plan(R_all, 100)
    plan.set_mode(rsgpu.WB_ATOMIC, depth)
    plan.set_schedule(1000, lb)
    plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), float(np.mean(r)))
    plan.epochs(3)
    best = 1e9
    for _ in range(3):
        plan.set_timing(True)
        plan.epochs(5)
        ms, k = plan.last_kernel_ms()
        best = min(best, ms / k * 1e3)
    P = plan.download()[0]
    plan.close()
    print(f"depth={depth:3d} light_blocks={lb:5d} epoch_us={best:8.1f} finite={np.isfinite(P).all()}", flush=True)
