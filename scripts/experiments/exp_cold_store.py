"""Experiment (round 6): cold-run write-through stores (rs_svd_plan_set_cold_store) on the ML-1M shape -- SGD kernel
time (HIP events) and the 90/10 held-out RMSE after 20 epochs against the threshold (runs in flight).

    python scripts/experiments/exp_cold_store.py [thr ...]
"""
import sys
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402


def main(thrs):
    u, i, r, nu, ni = synth.ml1m_like()
    perm = np.random.default_rng(0).permutation(len(r))
    te, tr = perm[: len(r) // 10], perm[len(r) // 10:]
    ctx = rsgpu.Context(0)
    for thr in thrs:
        plan = ctx.svd_plan(rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni), 100)
        plan.set_cold_store(thr)
        plan.init_normal(0.0, 0.1, seed=1)
        plan.upload(gb=float(np.mean(r[tr])))
        plan.set_timing(True)
        ms = []
        for e in range(20):
            plan.epochs(1)
            ms.append(plan.last_kernel_ms()[0])
        rm = plan.evaluate(u[te], i[te], r[te])[0]
        plan.close()
        print(f"cold {thr:g}: epoch {np.median(ms[3:]) * 1e3:.1f} us (min {min(ms[3:]) * 1e3:.1f}), "
              f"held-out RMSE {rm:.4f}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main([float(x) for x in sys.argv[1:]] or [0.0, 0.02, 0.05, 0.1, 0.2, 1.0])
