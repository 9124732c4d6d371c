"""Experiment: stability of the tile schedule on a Zipf-headed synthetic set (the configs[4] generator
at small scale, test_csr_plan_gpu's shape): held-out RMSE after 10 epochs for tile parameters.

    python scripts/experiments/exp_tile_stability.py wg,waves,target,run_cap,ring ...
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402


def main():
    cfgs = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]
    nu, ni, k = 20000, 4000, 64
    s = rsgpu.Synth(nu, ni, mean_deg=60.0, seed=20250826, n_threads=8)
    deg = np.diff(s.rowptr)
    users = np.repeat(np.arange(nu, dtype=np.int32), deg)
    hold = np.random.default_rng(0).random(s.nnz) < 0.05
    keep = ~hold
    tr_rowptr = np.concatenate([[0], np.cumsum(np.bincount(users[keep], minlength=nu))]).astype(np.int64)
    print("nnz", s.nnz, "max item degree", int(np.bincount(s.cols, minlength=ni).max()), flush=True)
    ctx = rsgpu.Context(0)
    for c in cfgs:
        plan = ctx.svd_plan_csr(nu, ni, tr_rowptr, s.cols[keep], s.vals[keep], k)
        plan.set_tiles(*c)
        plan.init_normal(0.0, 0.1, seed=1)
        e0 = plan.evaluate(users[hold], s.cols[hold], s.vals[hold])[0]
        plan.set_timing(True)
        plan.epochs(10, 0.005, 0.02)
        ms, nl = plan.last_kernel_ms()
        e = plan.evaluate(users[hold], s.cols[hold], s.vals[hold])[0]
        print(f"{str(c):24s} epoch {1000 * ms / nl:7.1f} us  held-out RMSE {e0:.4f} -> {e:.4f}", flush=True)
        plan.close()
    ctx.close()
    s.close()


if __name__ == "__main__":
    main()
