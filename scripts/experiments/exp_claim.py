"""Experiment (round 4): claimed runs inside a tile (rs_svd_plan_set_tile_claim) against the host deal
on the ML-1M shape (BASELINE configs[1], k = 100): SGD kernel time per epoch (HIP events) and the
20-epoch held-out RMSE next to the reference visit order (oracle).

    python scripts/experiments/exp_claim.py [claim[,ring] ...]      (default: 0 4 8 0 4 8)
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

K, EP = 100, 20


def main():
    cfgs = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [(0,), (4,), (8,), (0,), (4,), (8,)]
    u, i, r, nu, ni = synth.ml1m_like()
    n = len(r)
    te = np.zeros(n, bool)
    te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
    tr = ~te
    rng = np.random.default_rng(5)
    P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    gb0 = float(np.mean(r[tr]))
    if os.environ.get("REF", "1") == "1":
        import oracle as O
        t = time.time()
        ref = O.svd_fit(u[tr], i[tr], r[tr], P0, Q0, epochs=EP)
        e_ref = float(np.sqrt(np.mean((O.svd_predict(u[te], i[te], *ref) - r[te]) ** 2)))
        print(f"reference order: held-out RMSE {e_ref:.4f} ({time.time() - t:.1f} s CPU)", flush=True)
    ctx = rsgpu.Context(0)
    full = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), K)  # the bench's set (all ratings)
    for c in cfgs:
        claim, ring = c[0], (c[1] if len(c) > 1 else 0)
        plan = ctx.svd_plan(rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni), K)
        plan.set_tiles(0, 16, 0, 0, ring)
        plan.set_tile_claim(claim)
        plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), gb0)
        plan.set_timing(True)
        plan.epochs(2)  # warm-up
        plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), gb0)
        plan.epochs(EP)
        ms, nl = plan.last_kernel_ms()
        e = plan.evaluate(u[te], i[te], r[te])[0]
        plan.close()
        full.set_tiles(0, 16, 0, 0, ring)
        full.set_tile_claim(claim)
        full.init_normal(0.0, 0.1, seed=1)
        full.set_timing(True)
        full.epochs(3)
        full.epochs(20)
        fms, fnl = full.last_kernel_ms()
        print(f"claim {claim} ring {ring}: 90% set epoch {1000 * ms / nl:7.1f} us, held-out RMSE {e:.4f};"
              f"  full set epoch {1000 * fms / fnl:7.1f} us ({n * fnl / (fms / 1e3):.3e} upd/s)", flush=True)
    full.close()
    ctx.close()


if __name__ == "__main__":
    main()
