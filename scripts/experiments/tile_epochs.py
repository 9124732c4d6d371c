"""Minimal driver for profilers: builds the ML-1M-shaped plan (default tile schedule unless
WB=<mode>) and runs a few epochs; no torch import."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

t0 = time.time()
u, i, r, nu, ni = synth.ml1m_like()
ctx = rsgpu.Context(0)
plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
if "WB" in os.environ:
    plan.set_mode(int(os.environ["WB"]))
if "TILES" in os.environ:
    plan.set_tiles(*[int(x) for x in os.environ["TILES"].split(",")])
plan.init_normal(0.0, 0.1, seed=1)
print(f"plan ready {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
plan.epochs(int(os.environ.get("EPOCHS", "4")))
ctx.check(rsgpu.lib().rs_synchronize(ctx.h))
print(f"done {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
if os.environ.get("RSGPU_TILE_DIAG") == "16":  # per-wave phase clocks of the last epoch
    n = 256 * 16 * 4
    buf = np.zeros(n, np.int64)
    ctx.check(rsgpu.lib().rs_svd_plan_tile_clocks(plan.h, buf.ctypes.data, n))
    d = buf.reshape(-1, 4).astype(float)
    tot = d.sum(1)
    print("per-wave clocks (stage, ring wait, rating loops, tail): mean",
          np.round(d.mean(0)).tolist(), "max total", tot.max(), "min total", tot.min())
    busy = d[:, :3].sum(1).reshape(256, 16)  # without the tail (barrier wait + write-back)
    wg = busy.max(1)
    print("per-WG busy max over waves: mean", round(wg.mean()), "max", wg.max(), "min", wg.min())
    print("within-WG spread (max/mean over waves), mean over WGs:", round(float((busy.max(1) / busy.mean(1)).mean()), 3))
    pos, off = plan.tile_order()
    rp = np.concatenate([[0], np.cumsum(np.bincount(u, minlength=nu))])
    order = np.argsort(u, kind="stable")
    cu, ci = u[order][pos], i[order][pos]
    nt = (len(off) - 1) // 16
    st = []
    for t in range(nt):
        a, b = off[16 * t], off[16 * (t + 1)]
        uu, cnt = np.unique(cu[a:b], return_counts=True)
        st.append((b - a, len(np.unique(ci[a:b])), len(uu), cnt.max()))
    st = np.array(st, float)
    if nt == 256:
        for name, col in zip(("ratings", "runs", "users", "max user"), st.T):
            print(f"corr(WG time, {name}) = {np.corrcoef(wg, col)[0, 1]:+.2f}   range {col.min():.0f}..{col.max():.0f}")
    # per-wave ratings and runs of the schedule beside the clocks (cost-model fit)
    wr, wn = [], []
    for w in range(len(off) - 1):
        a, b = off[w], off[w + 1]
        wr.append(b - a)
        wn.append(int(np.count_nonzero(np.diff(ci[a:b]) != 0)) + (1 if b > a else 0))
    out = os.environ.get("CLOCKS_NPZ")
    if out:
        np.savez(out, clocks=buf.reshape(-1, 4), ratings=np.array(wr), runs=np.array(wn))
    for b in np.argsort(-wg)[:4]:
        print("slow WG", b, "waves busy:", busy[b].astype(int).tolist())
        print("   ring:", d.reshape(256, 16, 4)[b, :, 1].astype(int).tolist())
plan.close()
ctx.close()
