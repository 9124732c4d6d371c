"""Experiment: with hot replicas on (the default), what do the heavy users' chains still cost?
Timing only (split_cap uses the averaging merge; only its schedule matters here)."""
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


def run(name, split=0, heavy=1024, lb=-1, wb=0, reps=3):
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
    plan.set_mode(wb, 8)
    plan.set_schedule(heavy, lb)
    if split:
        plan.set_split(split)
    plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(nu),
                np.zeros(ni), 3.58)
    plan.epochs(3)
    best = 1e9
    for _ in range(reps):
        plan.set_timing(True)
        plan.epochs(5)
        ms, n = plan.last_kernel_ms()
        best = min(best, ms / n * 1e3)
    plan.close()
    print(f"{name:28s} epoch_us={best:8.1f}", flush=True)


run("warmup", reps=1)
run("replicas (default)")
for cap in (1024, 512, 256, 128):
    run(f"replicas + split {cap}", split=cap)
for lb in (256, 512, 768):
    run(f"replicas + split 256 lb={lb}", split=256, lb=lb)
run("replicas drop", wb=101)
run("replicas drop split 256", wb=101, split=256)
