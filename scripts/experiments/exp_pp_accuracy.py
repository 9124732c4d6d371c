"""Experiment: SVD++ FAST (K2) held-out RMSE spread vs the sequential lazy restatement on the ML-1M
shape (k=128, 20 epochs; the test_config2 setup) for several launch shapes, with the epoch time.
Each configuration runs REPS fits; the oracle runs once.  Env CFGS = "blocks:heavy[:heavy_blocks],..."
(RSGPU_PP_BLOCKS, RSGPU_PP_HEAVY, RSGPU_PP_HBLOCKS (removed); "d" keeps the library default)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle as O  # noqa: E402
import rsgpu  # noqa: E402
from helpers import rmse  # noqa: E402
from rsgpu import synth  # noqa: E402

u, i, r, nu, ni = synth.ml1m_like()
n = len(r)
te = np.zeros(n, bool)
te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
tr = ~te
k = 128
rng = np.random.default_rng(3)
P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
R = rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni)
t0 = time.time()
rowptr, items, rr = O.csr_by(u[tr], nu, i[tr], r[tr])
ref = O.svdpp_fit_lazy(rowptr, items, rr, P0, Q0, Y0, epochs=20)
e_ref = rmse(O.svdpp_predict(u[tr], i[tr], nu, u[te], i[te], *ref), r[te])
print(f"oracle held-out {e_ref:.4f} ({time.time() - t0:.1f} s)", flush=True)
# the same lazy schedule with the users visited heaviest first (the GPU's LPT work order)
deg = np.diff(rowptr)
lpt = np.argsort(-deg, kind="stable")
new_id = np.empty(nu, np.int64)
new_id[lpt] = np.arange(nu)
rp2, it2, rr2 = O.csr_by(new_id[u[tr]], nu, i[tr], r[tr])
P2, Q2, Y2, bu2, bi2, g2 = O.svdpp_fit_lazy(rp2, it2, rr2, P0[lpt], Q0, Y0, epochs=20)
P3, bu3 = np.empty_like(P2), np.empty_like(bu2)
P3[lpt], bu3[lpt] = P2, bu2
e_lpt = rmse(O.svdpp_predict(u[tr], i[tr], nu, u[te], i[te], P3, Q2, Y2, bu3, bi2, g2), r[te])
print(f"oracle, LPT user order: held-out {e_lpt:.4f}", flush=True)
ctx = rsgpu.Context(0)
reps = int(os.environ.get("REPS", "3"))
for cfg in os.environ.get("CFGS", "d:d,256:d,128:d,64:d,d:0").split(","):
    nb, hv, hb = (cfg.split(":") + ["d"])[:3]
    for key, v in (("RSGPU_PP_BLOCKS", nb), ("RSGPU_PP_HEAVY", hv), ("RSGPU_PP_HBLOCKS", hb)):
        if v == "d":
            os.environ.pop(key, None)
        else:
            os.environ[key] = v
    errs = []
    for _ in range(reps):
        got = ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=20)
        ms = ctx.last_kernel_ms() / 20
        errs.append(rmse(O.svdpp_predict(u[tr], i[tr], nu, u[te], i[te], *got), r[te]))
    gap = max(abs(e - e_ref) for e in errs)
    gap2 = max(abs(e - e_lpt) for e in errs)
    print(f"blocks {nb:>4} heavy {hv:>5} heavy blocks {hb:>4}: held-out {' '.join(f'{e:.4f}' for e in errs)} "
          f"max gap {gap:.4f} (LPT order {gap2:.4f}); epoch {ms:.3f} ms", flush=True)
