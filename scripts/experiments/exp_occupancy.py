"""Experiment: FAST epoch time (ML-1M shape, RS_SGD_WB_ATOMIC) vs the number of light blocks (waves
striding over the light users) and the heavy threshold: fewer atomics in flight, shorter queues."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) == 1:  # driver: one child per setting (the env var is read by set_heavy)
    for lb in os.environ.get("LBS", "0,2048,1024,512,256").split(","):
        for heavy in os.environ.get("HEAVY", "0,1024,512").split(","):
            env = dict(os.environ, RSGPU_LIGHT_BLOCKS=lb)
            r = subprocess.run([sys.executable, __file__, lb, heavy], env=env, capture_output=True, text=True)
            print(r.stdout.strip() or r.stderr[-2000:], flush=True)
    sys.exit(0)
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402
from helpers import rmse  # noqa: E402
lb, heavy = int(sys.argv[1]), int(sys.argv[2])
ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
warm = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)  # first plan of a process runs slow
warm.upload(np.zeros((nu, 100)), np.zeros((ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
warm.epochs(5)
warm.download()
warm.close()
plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
plan.set_mode(int(os.environ.get("WB", "0")), int(os.environ.get("RING", "8")))
plan.set_schedule(heavy, int(os.environ.get('RSGPU_LIGHT_BLOCKS', '-1')))
rng = np.random.default_rng(1)
plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
plan.set_timing(True)
plan.epochs(20)
ms, n = plan.last_kernel_ms()
P, Q, bu, bi, gb = plan.download()
tr = rmse(rsgpu.svd_predict(u, i, P, Q, bu, bi, gb), r)
plan.close()
print(f"wb={os.environ.get('WB', '0')} ring={os.environ.get('RING', '8')} light_blocks={lb} heavy={heavy} epoch_us={ms / n * 1e3:.1f} upd/s={len(r) / (ms / n / 1e3):.3e} train_rmse20={tr:.4f}")
