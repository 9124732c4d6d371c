"""Experiment (round 5): K1 on the ML-1M shape (BASELINE configs[1], k = 100) at several workgroup counts --
fewer tiles mean fewer (item, tile) runs and so fewer memory-side row atomics (the kernel's bound, DESIGN.md
K1 round 5), on fewer CUs.  SGD kernel time per epoch (HIP events) and the 20-epoch held-out RMSE.

    python scripts/experiments/exp_tile_wg.py [wg ...]      (default: 256 240 224 208 192 256)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

K, EP = 100, 20


def main():
    cfgs = [int(a) for a in sys.argv[1:]] or [256, 240, 224, 208, 192, 256]
    u, i, r, nu, ni = synth.ml1m_like()
    n = len(r)
    te = np.zeros(n, bool)
    te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
    tr = ~te
    rng = np.random.default_rng(5)
    P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    gb0 = float(np.mean(r[tr]))
    ctx = rsgpu.Context(0)
    full = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), K)
    for wg in cfgs:
        plan = ctx.svd_plan(rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni), K)
        plan.set_tiles(workgroups=wg)
        plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), gb0)
        plan.epochs(EP)
        e = plan.evaluate(u[te], i[te], r[te])[0]
        plan.close()
        full.set_tiles(workgroups=wg)
        full.init_normal(0.0, 0.1, seed=1)
        full.upload(gb=float(np.mean(r)))
        full.set_timing(True)
        full.epochs(3)
        full.epochs(20)
        fms, fnl = full.last_kernel_ms()
        print(f"workgroups {wg}: full set epoch {1000 * fms / fnl:7.1f} us ({n * fnl / (fms / 1e3):.3e} upd/s), "
              f"90% set held-out RMSE {e:.4f}, refits {full.refits()}", flush=True)
    full.close()
    ctx.close()


if __name__ == "__main__":
    main()
