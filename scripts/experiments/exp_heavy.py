"""Experiment: FAST epoch time on the ML-1M shape vs the hybrid write-back's heavy threshold
(rs_svd_plan_set_heavy), plus the direct-atomic and diagnostic modes for reference."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402
from helpers import rmse  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
deg = np.bincount(u, minlength=nu)
print("users with >= 2048/1024/512/256 ratings:", [(int((deg >= t).sum())) for t in (2048, 1024, 512, 256)])
cases = [(rsgpu.WB_ATOMIC_DIRECT, 0), (100, 0)] + [(rsgpu.WB_ATOMIC, h) for h in
                                                   (int(x) for x in os.environ.get("HEAVY", "0,2048,1024,512,256,128").split(","))]
for wb, heavy in cases:
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
    plan.set_mode(wb, int(os.environ.get("RING", "8")))
    plan.set_schedule(heavy, int(os.environ.get('RSGPU_LIGHT_BLOCKS', '-1')))
    rng = np.random.default_rng(1)
    plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
    plan.set_timing(True)
    plan.epochs(20)
    ms, n = plan.last_kernel_ms()
    P, Q, bu, bi, gb = plan.download()
    tr = rmse(rsgpu.svd_predict(u, i, P, Q, bu, bi, gb), r)
    plan.close()
    print(f"wb={wb} heavy={heavy} epoch_us={ms / n * 1e3:.1f} upd/s={len(r) / (ms / n / 1e3):.3e} train_rmse20={tr:.4f}",
          flush=True)
