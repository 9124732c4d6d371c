"""Experiment: SVD++ tile schedule (K2) waves per tile / workgroups vs accuracy and epoch time.
ML-100K fold 1 held-out RMSE (k=20, 20 epochs; literal reference order 0.9202) and the ML-1M shape
epoch (k=128, kernel time).  RSGPU_PP_TILE_WAVES / RSGPU_PP_TILE_WG select the variant."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle as O  # noqa: E402
import rsgpu  # noqa: E402
from helpers import folds, rmse  # noqa: E402
from rsgpu import synth  # noqa: E402

d = np.load(os.path.join(REPO, "tests", "golden", "ml100k.npz"))
f = folds(d["users"].astype(np.int64), d["items"].astype(np.int64), d["ratings"].astype(np.float64))[0]
u1, i1, r1, nu1, ni1 = synth.ml1m_like()
ctx = rsgpu.Context(0)
for cfg in sys.argv[1:]:
    wv, wg = cfg.split(",")
    os.environ["RSGPU_PP_TILE"] = "1"
    os.environ["RSGPU_PP_TILE_WAVES"] = wv
    os.environ["RSGPU_PP_TILE_WG"] = wg
    errs = []
    for seed in (4, 5):
        rng = np.random.default_rng(seed)
        P0, Q0, Y0 = (rng.normal(0, 0.1, (m, 20)) for m in (f.nu, f.ni, f.ni))
        b = ctx.svdpp_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, Y0)
        errs.append(rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *b), f.te_r))
    rng = np.random.default_rng(3)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, 128)) for m in (nu1, ni1, ni1))
    R = rsgpu.Ratings(u1, i1, r1, nu1, ni1)
    ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=1)
    ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=5)
    ms = ctx.last_kernel_ms() / 5
    print(f"waves {wv:>2} wg {wg:>4}: ML-100K RMSE {np.mean(errs):.4f} ({errs[0]:.4f}, {errs[1]:.4f}); "
          f"ML-1M k=128 epoch {ms:.3f} ms", flush=True)
