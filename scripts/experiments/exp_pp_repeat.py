"""Run-to-run spread of the SVD++ FAST fit on the configs[2] shape (ML-1M synthetic, k = 128, 20 epochs):
the same fit repeated (Hogwild timing differs between runs) and with other initial factors."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
for d in ("oracle", "tests", "recommend-sys_amd"):
    sys.path.insert(0, os.path.join(HERE, "..", "..", d))
import oracle as O  # noqa: E402
import rsgpu  # noqa: E402
from helpers import rmse  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
n = len(r)
te = np.zeros(n, bool)
te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
tr = ~te
k = 128
R = rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni)
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
for seed in range(runs):
    rng = np.random.default_rng(3 if seed < runs // 2 else 100 + seed)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
    try:
        got = ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=20)
        e = rmse(O.svdpp_predict(u[tr], i[tr], nu, u[te], i[te], *got), r[te])
        print(f"run {seed} (init {'3' if seed < runs // 2 else 100 + seed}): {ctx.last_kernel_ms() / 20:.3f} ms/epoch, "
              f"held-out {e:.4f}", flush=True)
    except rsgpu.RsError as ex:
        print(f"run {seed}: {ex}", flush=True)
