"""Experiment (round 4): rs_svd_fit_multi held-out RMSE on the ML-1M holdout at 2/4/8 shards (test_multi_gpu's
case), repeated; run with and without RSGPU_X_OLDKEY (round 3's run key) to find what moved the 8-shard fit."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

u, i, r, nu, ni = synth.ml1m_like()
te = np.zeros(len(r), bool)  # test_multi_gpu._ml1m_holdout's split and init
te[np.random.default_rng(9).permutation(len(r))[: len(r) // 10]] = True
tr = ~te
rng = np.random.default_rng(5)
P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
for n in [int(x) for x in sys.argv[1:]] or [2, 4, 8]:
    for rep in range(2):
        try:
            got = rsgpu.svd_fit_multi([0] * n, rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni), P0, Q0)
            e = float(np.sqrt(np.mean((rsgpu.svd_predict(u[te], i[te], *got) - r[te]) ** 2)))
            print(f"n={n} rep={rep}: held-out {e:.4f}", flush=True)
        except rsgpu.RsError as x:
            print(f"n={n} rep={rep}: RS_ERR {x.code}", flush=True)
