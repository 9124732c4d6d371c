"""Experiment: the tile schedule (RS_SGD_WB_TILE) on the ML-1M shape (BASELINE configs[1], k = 100):
epoch time (HIP events around each SGD kernel) and 20-epoch held-out RMSE for tile parameters, next
to the hybrid schedule and the reference visit order (oracle, C restatement).

    python scripts/experiments/exp_tile_sweep.py [wg,waves,target,run_cap,ring ...]
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
    cfgs = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]] or [
        (0, 16, 0, 0, 4), (0, 16, 0, 0, 8), (0, 16, 0, 0, 12), (0, 8, 0, 0, 12), (128, 16, 0, 0, 12),
        (128, 16, 0, 8, 12), (0, 16, 0, 8, 12), ("hybrid",)]
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
    for c in cfgs:
        plan = ctx.svd_plan(rsgpu.Ratings(u[tr], i[tr], r[tr], nu, ni), K)
        if c[0] == "hybrid":
            plan.set_mode(rsgpu.WB_ATOMIC)
        else:
            plan.set_tiles(*c)
        plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), gb0)
        plan.set_timing(True)
        plan.epochs(2)  # warm-up
        plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), gb0)
        plan.epochs(EP)
        ms, nl = plan.last_kernel_ms()
        e = plan.evaluate(u[te], i[te], r[te])[0]
        print(f"{str(c):24s} epoch {1000 * ms / nl:8.1f} us  ({tr.sum() * nl / (ms / 1e3):.3e} upd/s)  "
              f"held-out RMSE {e:.4f}", flush=True)
        plan.close()
    ctx.close()


if __name__ == "__main__":
    main()
