"""Experiment: where the default FAST epoch (hybrid schedule, ML-1M shape, k=100) spends its time.
Same kernel, inputs / write-back changed one factor at a time:
  base         the bench workload
  drop         writers drop the q_i atomics (DIAG 101): the schedule without memory-side atomics
  spread64x4   the top-64 items' ratings dealt over 4 distinct rows each (atomic serialisation of
               hot rows / 4, without the read cost a real replica scheme would pay)
  uniform      items uniform (same user degrees): no hot rows at all
  cap256       users cut into <= 256-rating pieces (rs_svd_plan_set_split): no long user chains
  uniform+cap  both
Plus the heavy-user timeline of base (chain ns/rating of the longest users)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
rng = np.random.default_rng(5)
deg_i = np.bincount(i, minlength=ni)
order = np.argsort(-deg_i, kind="stable")


def run(name, uu, ii, n_i, wb=0, split=0, reps=3):
    plan = ctx.svd_plan(rsgpu.Ratings(uu, ii, r, nu, n_i), 100)
    if wb:
        plan.set_mode(wb, 8)
    if split:
        plan.set_split(split)
    plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (n_i, 100)), np.zeros(nu),
                np.zeros(n_i), 3.58)
    plan.epochs(3)
    best = 1e9
    for _ in range(reps):
        plan.set_timing(True)
        plan.epochs(5)
        ms, n = plan.last_kernel_ms()
        best = min(best, ms / n * 1e3)
    plan.close()
    print(f"{name:14s} epoch_us={best:8.1f}", flush=True)
    return best


run("warmup", u, i, ni, reps=1)
run("base", u, i, ni)
run("drop", u, i, ni, wb=101)
H, R = 64, 4
slot = np.full(ni, -1)
slot[order[:H]] = np.arange(H)
ii = i.astype(np.int64).copy()
m = slot[i] >= 0
ii[m] = ni + slot[i[m]] * R + (u[m] % R)
run("spread64x4", u, ii.astype(np.int32), ni + H * R)
H, R = 256, 4
slot = np.full(ni, -1)
slot[order[:H]] = np.arange(H)
ii = i.astype(np.int64).copy()
m = slot[i] >= 0
ii[m] = ni + slot[i[m]] * R + (u[m] % R)
run("spread256x4", u, ii.astype(np.int32), ni + H * R)
# uniform items with the same (user, degree) structure, no repeats within a user
iu = np.empty_like(i)
for x in range(nu):
    sel = np.nonzero(u == x)[0]
    iu[sel] = rng.choice(ni, len(sel), replace=False)
run("uniform", u, iu, ni)
run("cap256", u, i, ni, split=256)
run("uniform+cap", u, iu, ni, split=256)
