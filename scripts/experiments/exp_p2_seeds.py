"""P2 across initial factors: the library's one-shot FAST fit (tile schedule, defaults) against the reference
visit order's fp64 restatement (oracle or_svd_fit) on the ML-1M-shaped 90/10 holdout, k = 100, 20 epochs,
several initial-factor seeds."""
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
R = rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni)
diffs = []
for seed in [int(x) for x in sys.argv[1].split(",")]:
    rng = np.random.default_rng(seed)
    P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
    ref = O.svd_fit(u[tr], i[tr], r[tr], P0, Q0, epochs=20)
    got = ctx.svd_fit(R, P0, Q0, n_epochs=20)
    e_ref = rmse(O.svd_predict(u[te], i[te], *ref), r[te])
    e_got = rmse(rsgpu.svd_predict(u[te], i[te], *got), r[te])
    diffs.append(e_got - e_ref)
    print(f"seed {seed}: GPU {e_got:.4f}, reference order {e_ref:.4f}, diff {e_got - e_ref:+.4f}, "
          f"refits {ctx.fit_refits()}", flush=True)
print(f"max |diff| {max(abs(d) for d in diffs):.4f} over {len(diffs)} seeds (P2 bound 0.003)", flush=True)
