"""(experiment) ML-1M-shaped K1 epoch (bench.py's workload) under the round-6 switches: cold-run stores and the
GlobalBias fold; kernel time by HIP events (rs_svd_plan_last_kernel_ms), median of 5 calls of 20 epochs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommend-sys_amd"))
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like(seed=20250824)
for cold, fold in [(None, None), (0.0, None), (None, 0), (0.0, 0), (None, None)]:
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
    if cold is not None:
        plan.set_cold_store(cold)
    if fold is not None:
        plan.set_gb_fold(fold)
    plan.init_normal(0.0, 0.1, seed=1)
    plan.upload(gb=float(np.mean(r)))
    plan.set_timing(True)
    plan.epochs(3)
    ms = []
    for _ in range(5):
        plan.epochs(20)
        m, n = plan.last_kernel_ms()
        ms.append(m / max(1, n) * 1000.0)
    print(f"cold {cold} fold {fold}: kernel {np.median(ms):.1f} us per epoch ({', '.join(f'{x:.1f}' for x in ms)})", flush=True)
    plan.close()
ctx.close()
