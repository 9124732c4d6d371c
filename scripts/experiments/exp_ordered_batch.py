"""ORDERED mode on the ML-1M shape: the batched kernel (default, RSGPU_ORDERED_NW = 16 or 8) against the
one-wave ring kernel (RSGPU_ORDERED_WAVE=1); kernel-only time of one and of three epochs, and the max
|difference| of the factors between the variants (all are the sequential epoch)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "recommend-sys_amd"))
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

u, i, r, nu, ni = synth.ml1m_like()
K = int(os.environ.get("K", "100"))
rng = np.random.default_rng(1)
P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
R = rsgpu.Ratings(u, i, r, nu, ni)
res = {}
with rsgpu.Context(0) as ctx:
    for name, env in [("batch16", {"RSGPU_ORDERED_NW": "16"}), ("batch8", {"RSGPU_ORDERED_NW": "8"}),
                      ("wave", {"RSGPU_ORDERED_WAVE": "1"})]:
        for k_, v_ in env.items():
            os.environ[k_] = v_
        for ep in (1, 3):
            t0 = time.time()
            out = ctx.svd_fit(R, P0, Q0, n_epochs=ep, mode=rsgpu.SGD_ORDERED)
            wall = time.time() - t0
            ms = ctx.last_kernel_ms()
            res[(name, ep)] = out
            print(f"{name} epochs={ep}: kernel {ms:.2f} ms = {ms / ep:.2f} ms/epoch, "
                  f"{len(r) * ep / (ms / 1e3):.3e} upd/s, wall {wall:.3f} s", flush=True)
        for k_ in env:
            del os.environ[k_]
for ep in (1, 3):
    a, b = res[("batch16", ep)], res[("wave", ep)]
    d = max(float(np.max(np.abs(np.asarray(x) - np.asarray(y)))) for x, y in zip(a[:4], b[:4]))
    print(f"epochs={ep}: max|batch16 - wave| = {d:.3e}, gb {a[4]:.9f} vs {b[4]:.9f}")
