"""(experiment) 1m_k100_r32's refits on a given library tree: python exp_r32_bisect.py <repo root> [mode]
mode: eval (held-out after every epoch, as tests/stability_sets.run), noeval (10 one-epoch calls), one (one 10-epoch call)"""
import os
import sys

import numpy as np

root = sys.argv[1]
mode = sys.argv[2] if len(sys.argv) > 2 else "eval"
sys.path.insert(0, os.path.join(root, "recommend-sys_amd"))
import rsgpu  # noqa: E402

U, I, deg, zs, k, ep = 20000, 2000, 50.0, 0.65, 100, 10
ctx = rsgpu.Context(0)
s = rsgpu.Synth(U, I, mean_deg=deg, zipf_s=zs, seed=20250901, n_threads=16)
users = np.repeat(np.arange(U, dtype=np.int32), np.diff(s.rowptr))
hold = np.random.default_rng(0).random(s.nnz) < 0.05
keep = ~hold
rp = np.concatenate([[0], np.cumsum(np.bincount(users[keep], minlength=U))]).astype(np.int64)
cols, vals = s.cols[keep].copy(), s.vals[keep].copy()
hu, hi, hr = users[hold], s.cols[hold].copy(), s.vals[hold].astype(np.float64)
s.close()
for rep in range(4):
    plan = ctx.svd_plan_csr(U, I, rp, cols, vals, k)
    plan.set_tile_claim(4)
    plan.init_normal(0.0, 0.1, seed=1)
    plan.upload(gb=float(np.mean(vals, dtype=np.float64)))
    curve = []
    if mode == "one":
        plan.epochs(ep)
    else:
        for _ in range(ep):
            plan.epochs(1)
            if mode == "eval":
                curve.append(plan.evaluate(hu, hi, hr)[0])
    curve.append(plan.evaluate(hu, hi, hr)[0])
    print(f"{os.path.basename(root.rstrip('/'))} {mode}: refits {plan.refits()} held-out " + " ".join(f"{x:.4f}" for x in curve), flush=True)
    plan.close()
ctx.close()
