"""Experiment: KNN MFMA kernel time on the ML-20M-shaped set per tile order (env RSGPU_KNN_ORDER)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu
from rsgpu import synth
u, i, r, nu, ni = synth.ml20m_like()
order = np.argsort(i, kind="stable")
rowptr = np.zeros(ni + 1, np.int64)
np.add.at(rowptr, i.astype(np.int64) + 1, 1)
rowptr = np.cumsum(rowptr)
ids, rr = u[order], r[order]
ctx = rsgpu.Context(0)
for mode in ["0", "1", "2", "1", "2"]:
    os.environ["RSGPU_KNN_ORDER"] = mode
    S = ctx.knn_sims(rsgpu.SIM_COSINE, rowptr, ids, rr, nu)
    print(f"order={mode} kernel_ms={ctx.last_kernel_ms():.1f}", flush=True)
    del S
