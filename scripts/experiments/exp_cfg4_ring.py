"""Experiment: configs[4]'s per-GPU shard (SVD k=256, the 1/8 item shard of the 10M x 1M x 1e9 set) under
tile parameters -- the q-ring depth (runs ahead per wave), waves per workgroup, run cap.  In this sparse
regime a run is about one rating, so every rating pays a q_i row load and an atomic row; the ring depth
is how many of them a wave keeps in flight.  Epoch time (HIP events) and the held-out RMSE after five
epochs (the test_config4 bound: < 0.95).

    python scripts/experiments/exp_cfg4_ring.py [waves,ring,run_cap ...]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402

cfgs = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(16, 2, 0), (16, 4, 0), (16, 6, 0)]
n_users, n_items, k = 10_000_000, 1_000_000, 256
ctx = rsgpu.Context(0)
s = rsgpu.Synth(n_users, n_items, mean_deg=100.0, seed=20250826, item_lo=0, item_hi=n_items // 8, n_threads=16)
deg = np.diff(s.rowptr)
users = np.repeat(np.arange(n_users, dtype=np.int32), deg)
hold = np.random.default_rng(0).random(s.nnz) < 0.001
keep = ~hold
tr_rowptr = np.concatenate([[0], np.cumsum(np.bincount(users[keep], minlength=n_users))]).astype(np.int64)
nnz = int(keep.sum())
t0 = time.perf_counter()
plan = ctx.svd_plan_csr(n_users, n_items, tr_rowptr, s.cols[keep], s.vals[keep], k)
print(f"plan built in {time.perf_counter() - t0:.1f} s, {nnz} ratings", flush=True)
ab = nnz * (16 + 8 * k) + n_users * (16 + 8 * k)
for waves, ring, cap in cfgs:
    t0 = time.perf_counter()
    plan.set_tiles(0, waves, 0, cap, ring)
    tb = time.perf_counter() - t0
    plan.init_normal(0.0, 0.1, seed=1)
    plan.set_timing(True)
    plan.epochs(5)
    ms, nl = plan.last_kernel_ms()
    plan.set_timing(False)
    e5 = plan.evaluate(users[hold], s.cols[hold], s.vals[hold])[0]
    t_ep = ms / nl
    print(f"waves {waves:>2} ring {ring} run_cap {cap}: epoch {t_ep:.1f} ms, frac {ab / (t_ep / 1e3) / 8e12:.3f}, "
          f"held-out RMSE after 5 epochs {e5:.4f} (tiles rebuilt in {tb:.1f} s)", flush=True)
plan.close()
s.close()
