#!/usr/bin/env python3
"""Round 5: FAST SVD++ on the -10..10 rescaled ML-100K (tests/test_rating_scales_gpu.py) -- is the gap to the
sequential restatements numeric (fixed point at 2^-22) or Hogwild (users in flight)?  Runs fold 0 with the
default, fp32 Q/Y (RSGPU_PP_FX=0 in a child) and fewer light blocks (RSGPU_PP_BLOCKS)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]


def one(scale, lr):
    import numpy as np
    import oracle as O
    import rsgpu
    from helpers import folds, rmse
    d = np.load(os.path.join(REPO, "tests", "golden", "ml100k.npz"))
    U, I, R = d["users"].astype(np.int64), d["items"].astype(np.int64), d["ratings"].astype(np.float64)
    R = {"pm10": (R - 3) * 5, "x20": 20 * R, "x1": R}[scale]
    k = 20
    out = []
    with rsgpu.Context(0) as ctx:
        for f in folds(U, I, R)[:2]:
            rng = np.random.default_rng(4)
            P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (f.nu, f.ni, f.ni))
            b = ctx.svdpp_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, Y0, lr=lr)
            out.append(rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *b), f.te_r))
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1:
        print(sys.argv[1], sys.argv[2], os.environ.get("RSGPU_PP_FX"), os.environ.get("RSGPU_PP_BLOCKS"),
              one(sys.argv[1], float(sys.argv[2])), flush=True)
        sys.exit(0)
    for scale, lr in (("pm10", 1e-3), ("x1", 0.007), ("x20", 1e-4)):
        for env in ({}, {"RSGPU_PP_FX": "0"}, {"RSGPU_PP_BLOCKS": "32"}, {"RSGPU_PP_BLOCKS": "8"}):
            e = dict(os.environ, **env)
            subprocess.run([sys.executable, __file__, scale, str(lr)], env=e, check=True, timeout=300)
