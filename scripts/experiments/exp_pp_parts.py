"""Experiment: what bounds the SVD++ FAST epoch (K2, k=128, ML-1M shape)?  Epoch time of the full set,
of the light users only (< 1024 ratings), and of the heavy users only (their serial chains without
the light users' atomic traffic)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

u, i, r, nu, ni = synth.ml1m_like()
deg = np.bincount(u, minlength=nu)
heavy = deg[u] >= 1024
ctx = rsgpu.Context(0)
k = 128
rng = np.random.default_rng(3)
P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
for name, sel in (("full", np.ones(len(r), bool)), ("light", ~heavy), ("heavy", heavy)):
    R = rsgpu.Ratings(u[sel], i[sel], r[sel], nu, ni)
    ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=1)
    best = 1e9
    for _ in range(3):
        ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=5)
        best = min(best, ctx.last_kernel_ms() / 5)
    print(f"{name:>5}: {int(sel.sum())} ratings, {int((np.bincount(u[sel], minlength=nu) > 0).sum())} users, "
          f"epoch {best:.3f} ms, max degree {int(np.bincount(u[sel], minlength=nu).max())}", flush=True)
