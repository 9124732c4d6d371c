"""Experiment: SVD++ FAST epoch (k=128, ML-1M shape) vs the number of striding blocks."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import os, sys, numpy as np
sys.path[:0] = [os.path.join(%r, "recommend-sys_amd")]
import rsgpu
from rsgpu import synth
ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
k = 128
rng = np.random.default_rng(3)
P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
R = rsgpu.Ratings(u, i, r, nu, ni)
ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=1)
best = 1e9
for _ in range(3):
    ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=5)
    best = min(best, ctx.last_kernel_ms() / 5)
print(os.environ.get("RSGPU_PP_BLOCKS", "default"), f"epoch_ms={best:.3f}", flush=True)
''' % REPO
for nb in os.environ.get("NB", "default,128,256,384,512,768,1510").split(","):
    env = dict(os.environ)
    if nb != "default":
        env["RSGPU_PP_BLOCKS"] = nb
    subprocess.run([sys.executable, "-c", code], env=env, check=True)
