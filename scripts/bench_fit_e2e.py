"""End-to-end Fit through the C-ABI host boundary (the Go `Fit` call): host COO + f64
factors in, f64 factors out, 20 epochs on the ML-1M shape -- wall time of the rs_svd_fit call (plan /
schedule build, H2D/D2H, f64<->f32 packing) beside the device kernel span of the same call.  SVD k=100
(FAST) and SVD++ k=128 (FAST).  One JSON line per estimator and call.

SVD: the factors are trained in place (svd_fit(inplace=True)), as the Go binding passes the Fit's own
slices; the binding's numpy copies of P0 / Q0 are made before the clock starts.  `fit_wall_with_copies_s`
is the same call with the copies inside the clock (the previous rounds' figure)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
R = rsgpu.Ratings(u, i, r, nu, ni)
u2, i2, r2, nu2, ni2 = synth.ml1m_like(seed=7)  # a second TrainSet: alternating fits never hit the cache
R2 = rsgpu.Ratings(u2, i2, r2, nu2, ni2)
nnz, epochs = len(r), 20
rng = np.random.default_rng(3)
for name, k in (("svd", 100), ("svdpp", 128)):
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
    P2, Q2, Y2 = (rng.normal(0, 0.1, (m, k)) for m in (nu2, ni2, ni2))

    def fit(other=False, copies=True):
        if name == "svd":
            if other:
                return ctx.svd_fit(R2, P2, Q2, n_epochs=epochs)
            if copies:
                return ctx.svd_fit(R, P0, Q0, n_epochs=epochs)
            P, Q, bu, bi = P0.copy(), Q0.copy(), np.zeros(nu), np.zeros(ni)  # the caller's slices
            t0 = time.perf_counter()
            ctx.svd_fit(R, P, Q, bu, bi, n_epochs=epochs, inplace=True)
            return time.perf_counter() - t0
        return ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=epochs)

    def best_of(n, alternate):
        best, best_c = None, None
        for _ in range(n):
            if alternate:
                fit(other=True)  # evicts the cached plan
            if name == "svd":
                wall = fit(copies=False)
                kern = ctx.last_kernel_ms() / 1e3
                if alternate:
                    fit(other=True)
                t0 = time.perf_counter()
                fit()
                wall_c = time.perf_counter() - t0
            else:
                t0 = time.perf_counter()
                fit()
                wall = wall_c = time.perf_counter() - t0
                kern = ctx.last_kernel_ms() / 1e3
            if best is None or wall < best[0]:
                best = (wall, kern)
            best_c = wall_c if best_c is None else min(best_c, wall_c)
        return best + (best_c,)

    fit()  # warm-up (first plan / code object load)
    rows = [("new TrainSet (plan built)", best_of(5, True))]
    if name == "svd":
        rows.append(("same TrainSet again (plan reused)", best_of(5, False)))
    for what, (wall, kern, wall_c) in rows:
        print(json.dumps({"estimator": name, "k": k, "epochs": epochs, "nnz": nnz, "call": what,
                          "fit_wall_s": wall, "kernel_span_s": kern, "fit_wall_with_copies_s": wall_c,
                          "updates_per_s_end_to_end": nnz * epochs / wall,
                          "updates_per_s_kernels": nnz * epochs / kern,
                          "host_share": 1 - kern / wall}), flush=True)
