"""(experiment) What a ROTATE rank's epoch costs in kernels at N ranks: bench.py's ML-1M-shaped shard cut into N x 2 user
blocks (the rotation's rank-blocks x pieces), every block launched alone and timed (rs_svd_plan_time_blocks)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "recommend-sys_amd"))
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like(seed=20250824)
for nb in (1, 2, 4, 8, 16):
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
    if nb > 1:
        plan.set_user_blocks(nb)
    plan.init_normal(0.0, 0.1, seed=1)
    plan.upload(gb=float(np.mean(r)))
    plan.time_blocks(nb)
    ms = np.median([plan.time_blocks(nb) for _ in range(5)], axis=0)
    print(f"{nb:2d} user blocks: sum {ms.sum() * 1000:.1f} us per epoch, per block {ms.mean() * 1000:.1f} us "
          f"(min {ms.min() * 1000:.1f}, max {ms.max() * 1000:.1f})", flush=True)
    plan.close()
ctx.close()
