"""(experiment) ML-1M-shaped K1 kernel time of the library under a given tree: python exp_k1_lib_ab.py <repo root>"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(sys.argv[1], "recommend-sys_amd"))
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like(seed=20250824)
plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
plan.init_normal(0.0, 0.1, seed=1)
plan.upload(gb=float(np.mean(r)))
plan.set_timing(True)
plan.epochs(3)
ms = []
for _ in range(7):
    plan.epochs(20)
    m, n = plan.last_kernel_ms()
    ms.append(m / max(1, n) * 1000.0)
print(f"{sys.argv[1]}: kernel {np.median(ms):.1f} us per epoch ({', '.join(f'{x:.1f}' for x in ms)})", flush=True)
plan.close()
ctx.close()
