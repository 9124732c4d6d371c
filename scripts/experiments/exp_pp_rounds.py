"""SVD++ FAST, the ROUNDS schedule (svdpp_round_kernel, RSGPU_PP_ROUNDS) against the one-launch user-major kernel:
epoch time and held-out RMSE on the configs[2] shape (ML-1M synthetic, k = 128, 20 epochs) and on the ML-100K fold
(k = 20) against the literal order."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
for d in ("oracle", "tests", "recommend-sys_amd"):
    sys.path.insert(0, os.path.join(HERE, "..", "..", d))
import oracle as O  # noqa: E402
import rsgpu  # noqa: E402
from helpers import folds, rmse  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
rounds = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 4, 8, 16]
u, i, r, nu, ni = synth.ml1m_like()
n = len(r)
te = np.zeros(n, bool)
te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
tr = ~te
k = 128
rng = np.random.default_rng(3)
P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
R = rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni)
for b in rounds:
    os.environ["RSGPU_PP_ROUNDS"] = str(b)
    got = ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=20)
    ms = ctx.last_kernel_ms() / 20
    e = rmse(O.svdpp_predict(u[tr], i[tr], nu, u[te], i[te], *got), r[te])
    print(f"configs[2] rounds {b}: {ms:.3f} ms/epoch, held-out {e:.4f}", flush=True)
d = np.load(os.path.join(HERE, "..", "..", "tests", "golden", "ml100k.npz"))
f = folds(d["users"].astype(np.int64), d["items"].astype(np.int64), d["ratings"].astype(np.float64))[0]
rng = np.random.default_rng(4)
P0, Q0, Y0 = (rng.normal(0, 0.1, (m, 20)) for m in (f.nu, f.ni, f.ni))
for b in rounds:
    os.environ["RSGPU_PP_ROUNDS"] = str(b)
    res = ctx.svdpp_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0, Y0)
    print(f"ML-100K rounds {b}: {rmse(O.svdpp_predict(f.iu, f.ii, f.nu, f.tu, f.ti, *res), f.te_r):.4f} "
          f"({ctx.last_kernel_ms() / 20:.3f} ms/epoch; literal order 0.9202)", flush=True)
