"""Experiment: default FAST epoch time (ML-1M shape) of the library under ROOT (argv[1]); run for two
checkouts in one GPU session to compare code versions on the same box."""
import os
import sys

ROOT = os.path.abspath(sys.argv[1])
sys.path[:0] = [os.path.join(ROOT, "recommend-sys_amd")]
import numpy as np  # noqa: E402
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
modes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")]
for wb in modes:
    out = []
    for rep in range(3):
        plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
        plan.set_mode(wb, 8)
        rng = np.random.default_rng(1)
        plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
        plan.set_timing(True)
        plan.epochs(20)
        ms, n = plan.last_kernel_ms()
        plan.close()
        out.append(ms / n * 1e3)
    print(f"{os.path.basename(ROOT)} wb={wb} epoch_us={' '.join(f'{x:.0f}' for x in out)}", flush=True)
