"""Experiment: hot replicas (rs_svd_plan_set_hot_replicas) on the ML-1M shape, k=100 -- epoch time
and 20-epoch held-out RMSE (90/10 split, same init) against the reference visit order's (oracle C
restatement of svd.go), for several (n_hot, copies)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle")]
import oracle as O  # noqa: E402
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
n = len(r)
te = np.zeros(n, bool)
te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
tr = ~te
rng = np.random.default_rng(5)
P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
t0 = time.time()
ref = O.svd_fit(u[tr], i[tr], r[tr], P0, Q0, epochs=20)
e_ref = float(np.sqrt(np.mean((O.svd_predict(u[te], i[te], *ref) - r[te]) ** 2)))
print(f"reference order held-out RMSE {e_ref:.4f} ({time.time() - t0:.1f} s)", flush=True)
R_tr = rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni)
R_all = rsgpu.Ratings(u, i, r, nu, ni)
gb0 = float(np.mean(r[tr]))
cfgs = [tuple(int(v) for v in c.split("x")) for c in
        os.environ.get("CFGS", "0x4,128x8,192x8,256x8,320x8,384x8,256x6,192x6").split(",")]
for n_hot, copies in cfgs:
    plan = ctx.svd_plan(R_all, 100)
    plan.set_hot_replicas(n_hot, copies)
    plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), float(np.mean(r)))
    plan.epochs(3)
    best = 1e9
    for _ in range(3):
        plan.set_timing(True)
        plan.epochs(5)
        ms, k = plan.last_kernel_ms()
        best = min(best, ms / k * 1e3)
    plan.close()
    plan = ctx.svd_plan(R_tr, 100)
    plan.set_hot_replicas(n_hot, copies)
    plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), gb0)
    plan.epochs(20)
    e = plan.evaluate(u[te], i[te], r[te])[0]
    plan.close()
    print(f"hot={n_hot:5d} x{copies} epoch_us={best:8.1f} held-out RMSE {e:.4f} (ref {e_ref:.4f}, "
          f"d={e - e_ref:+.4f})", flush=True)
