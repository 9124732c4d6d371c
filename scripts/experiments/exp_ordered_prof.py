"""ORDERED batched kernel on the ML-1M shape: one epoch per configuration given as NAME=ENV[,ENV..]
arguments (e.g. nw16=RSGPU_ORDERED_NW:16,RSGPU_ORDERED_PROF:1); prints the kernel time (the per-phase
cycle lines of RSGPU_ORDERED_PROF go to stderr)."""
import os
import sys

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
with rsgpu.Context(0) as ctx:
    ref = None
    for arg in sys.argv[1:]:
        name, envs = arg.split("=", 1)
        env = dict(e.split(":") for e in envs.split(",") if e)
        os.environ.update(env)
        out = ctx.svd_fit(R, P0, Q0, n_epochs=1, mode=rsgpu.SGD_ORDERED)
        ms = ctx.last_kernel_ms()
        for k_ in env:
            del os.environ[k_]
        d = 0.0 if ref is None else max(float(np.max(np.abs(np.asarray(a) - np.asarray(b)))) for a, b in zip(out[:4], ref[:4]))
        ref = out if ref is None else ref
        print(f"{name}: {ms:.2f} ms/epoch, {len(r) / (ms / 1e3):.3e} upd/s, max|d| vs first {d:.2e}", flush=True)
        sys.stderr.flush()
