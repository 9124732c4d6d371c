"""Experiment (follow-up of exp_decompose.py): floors of the hybrid FAST epoch without atomics, and
its sensitivity to the light-wave count, on the ML-1M shape (k=100)."""
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
iu = np.empty_like(i)
for x in range(nu):
    sel = np.nonzero(u == x)[0]
    iu[sel] = rng.choice(ni, len(sel), replace=False)


def run(name, ii, wb=0, split=0, heavy=1024, lb=-1, reps=3):
    plan = ctx.svd_plan(rsgpu.Ratings(u, ii, r, nu, ni), 100)
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
    print(f"{name:34s} epoch_us={best:8.1f}", flush=True)


run("warmup", i, reps=1)
run("base", i)
run("drop", i, wb=101)
run("drop cap256", i, wb=101, split=256)
run("drop uniform cap256", iu, wb=101, split=256)
run("nowb(direct) cap256", i, wb=100, split=256)
run("nowb(direct) uniform cap256", iu, wb=100, split=256)
for lb in (128, 256, 768, 1536):
    run(f"base lb={lb}", i, lb=lb)
for lb in (256, 768, 1536):
    run(f"drop cap256 lb={lb}", i, wb=101, split=256, lb=lb)
for lb in (768, 1536):
    run(f"uniform cap256 lb={lb}", iu, split=256, lb=lb)
