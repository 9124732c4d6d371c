"""Debug: where does the ROTATE_Q group fit of config4_sharded.py go non-finite (small scale)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "tests")]
import rsgpu  # noqa: E402
import config4_fit as C  # noqa: E402  (tests/config4_fit.py)

U, I, k, n = 200000, 20000, 64, 8
ctx = rsgpu.Context(0)
parts = C.generate(U, I, n, 20250826)
nnz = int(sum(int(p["rowptr"][-1]) for p in parts))
gb0 = float(sum(float(np.sum(p["vals"], dtype=np.float64)) for p in parts) / nnz)


def report(tag, plans):
    for x, pl in enumerate(plans[:2]):
        P, Q, bu, bi, g = pl.download() if True else None
        badp = np.where(~np.isfinite(P).all(1))[0]
        badq = np.where(~np.isfinite(Q).all(1))[0]
        print(f"{tag} shard {x}: gb {g:.5f} bad P rows {len(badp)} (first {badp[:5]}) bad Q rows {len(badq)} "
              f"(first {badq[:5]}) bad bu {int((~np.isfinite(bu)).sum())} bad bi {int((~np.isfinite(bi)).sum())} "
              f"max|P| {np.nanmax(np.abs(P)):.3g} max|Q| {np.nanmax(np.abs(Q)):.3g}", flush=True)


for waves, wg, blocks in ((1, 0, 8), (16, 0, 8), (16, 0, 16)):
    plans = []
    for p in parts:
        pl = ctx.svd_plan_csr(U, I, C.padded_rowptr(p, U), p["cols"], p["vals"], k)
        pl.set_exchange(rsgpu.EXCHANGE_ROTATE_Q)
        pl.set_tiles(workgroups=wg, waves=waves)
        pl.init_normal(0.0, 0.1, seed=1)
        pl.upload(gb=gb0)
        plans.append(pl)
    report(f"w{waves} b{blocks} init", plans)
    g = rsgpu.SvdGroup(plans, n_blocks=blocks)
    print("shard info", plans[0].shard_info(), flush=True)
    try:
        g.epochs(1)
    except rsgpu.RsError as e:
        print("epochs error", e, flush=True)
    try:
        report(f"w{waves} b{blocks} after 1", plans)
    except rsgpu.RsError as e:
        print("download error", e, flush=True)
    g.close()
    for pl in plans:
        pl.close()
# the same data through rs_svd_fit_multi (COO) for comparison
u = np.concatenate([np.repeat(np.arange(p["lo"], p["hi"], dtype=np.int32), np.diff(p["rowptr"])) for p in parts])
i = np.concatenate([p["cols"] for p in parts]).astype(np.int32)
r = np.concatenate([p["vals"] for p in parts]).astype(np.float64)
rng = np.random.default_rng(1)
P0, Q0 = rng.normal(0, 0.1, (U, k)), rng.normal(0, 0.1, (I, k))
got = rsgpu.svd_fit_multi([0] * n, rsgpu.Ratings(u, i, r, U, I), P0, Q0, n_epochs=1)
print("fit_multi finite:", [bool(np.all(np.isfinite(x))) for x in got[:4]], got[4], flush=True)
ctx.close()
