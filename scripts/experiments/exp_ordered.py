"""ORDERED SVD throughput (one epoch over the ML-1M shape, kernel time); with a file argument the
fitted model is saved for bitwise comparisons between kernel variants.  Round 2 tried a variant with
the next 8 ratings' rows in flight (stale rows re-read on a user/item conflict): bitwise equal, but
702 ms per epoch against 517 ms -- the chain is not the rows' load latency -- so it was dropped."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

u, i, r, nu, ni = synth.ml1m_like()
ctx = rsgpu.Context(0)
rng = np.random.default_rng(1)
P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
R = rsgpu.Ratings(u, i, r, nu, ni)
ctx.svd_fit(R, P0, Q0, n_epochs=1, mode=rsgpu.SGD_ORDERED)
m = ctx.svd_fit(R, P0, Q0, n_epochs=1, mode=rsgpu.SGD_ORDERED)
ms = ctx.last_kernel_ms()
out = sys.argv[1] if len(sys.argv) > 1 else None
if out:
    np.savez(out, *m[:4], gb=m[4])
print(f"ORDERED epoch {ms:.1f} ms, {len(r) / ms * 1e3:.3e} upd/s, gb {m[4]!r}", flush=True)
