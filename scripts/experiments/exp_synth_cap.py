"""test_synth_plan_trains_and_holds_out's set (20000 users x 4000 items, mean degree 60, Zipf head:
hottest item 16271 of 1.13M ratings, k = 64) trained 10 epochs at several tile run caps (0 = the
automatic cap): held-out RMSE, to separate the run-cap floor's staleness from run-to-run Hogwild noise."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "recommend-sys_amd"))
import rsgpu  # noqa: E402

nu, ni, k = 20000, 4000, 64
with rsgpu.Context(0) as ctx:
    s = rsgpu.Synth(nu, ni, mean_deg=60.0, seed=20250826, n_threads=8)
    deg = np.diff(s.rowptr)
    users = np.repeat(np.arange(nu, dtype=np.int32), deg)
    hold = np.zeros(s.nnz, bool)
    hold[np.random.default_rng(0).random(s.nnz) < 0.05] = True
    keep = ~hold
    tr_rowptr = np.concatenate([[0], np.cumsum(np.bincount(users[keep], minlength=nu))]).astype(np.int64)
    caps = [int(x) for x in (sys.argv[1:] or ["0", "3", "4", "0", "3", "4"])]
    for cap in caps:
        plan = ctx.svd_plan_csr(nu, ni, tr_rowptr, s.cols[keep], s.vals[keep], k)
        if cap:
            plan.set_tiles(run_cap=cap)
        plan.init_normal(0.0, 0.1, seed=1)
        rmse0, _ = plan.evaluate(users[hold], s.cols[hold], s.vals[hold])
        out = []
        for e in range(10):
            plan.epochs(1, 0.005, 0.02)
            out.append(plan.evaluate(users[hold], s.cols[hold], s.vals[hold])[0])
        plan.close()
        print(f"cap {cap}: rmse0 {rmse0:.4f} per epoch " + " ".join(f"{x:.4f}" for x in out), flush=True)
    s.close()
