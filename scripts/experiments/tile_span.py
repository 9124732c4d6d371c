"""Per-workgroup start / end clocks of the claimed-run tile kernel (RSGPU_TILE_DIAG=32: no extra waits)
on the ML-1M shape, with each tile's schedule statistics and the XCD each workgroup ran on: what makes the
slowest workgroups slow.  Writes gpurun_out/tile_span.npz and prints a summary."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
os.environ["RSGPU_TILE_DIAG"] = "32"
import rsgpu  # noqa: E402
from rsgpu import synth  # noqa: E402

u, i, r, nu, ni = synth.ml1m_like()
ctx = rsgpu.Context(0)
plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 100)
plan.init_normal(0.0, 0.1, seed=1)
plan.epochs(3)
ctx.check(rsgpu.lib().rs_synchronize(ctx.h))
n = 256 * 16 * 4
buf = np.zeros(n, np.int64)
ctx.check(rsgpu.lib().rs_svd_plan_tile_clocks(plan.h, buf.ctypes.data, n))
d = buf.reshape(256, 16, 4)
cyc = d[:, :, 1] - d[:, :, 0]           # shader-clock cycles per wave (s_memtime, per XCD)
rt0 = d[:, :, 2]                         # s_memrealtime (100 MHz) at the wave's start
rtl = d[:, :, 3] & ((1 << 48) - 1)       # ... and its length
xcd = (d[:, 0, 3] >> 48) & 15
t0 = rt0.min()
start, end = rt0 - t0, rt0 - t0 + rtl
cu = xcd * 0
wg_end = end.max(1)
wg_len = wg_end - start.min(1)
print("real time (100 MHz ticks): kernel", int(end.max()), " WG start max", int(start.min(1).max()))
ghz = cyc.max(1) / np.maximum(1, rtl.max(1)) / 10.0
for x in range(8):
    m = xcd == x
    print(f"XCD {x}: clock {ghz[m].mean():.2f} GHz, WG real length mean {wg_len[m].mean():.0f} max {wg_len[m].max():.0f} "
          f"end max {wg_end[m].max():.0f}")
pos, off = plan.tile_order()
order = np.argsort(u, kind="stable")
ci, cu_ = i[order][pos], u[order][pos]
deg = np.bincount(i, minlength=ni)
hot = deg >= np.sort(deg)[-64]
st = []
for t in range(256):
    a, b = off[16 * t], off[16 * (t + 1)]
    items = ci[a:b]
    st.append((b - a, len(np.unique(items)), int(hot[items].sum()), len(np.unique(cu_[a:b]))))
st = np.array(st, float)
np.savez(os.path.join(REPO, "gpurun_out", "tile_span.npz"), start=start, end=end, xcd=xcd, cu=cu, stats=st)
print("kernel span (cycles):", int(end.max()), " WG length mean", int(wg_len.mean()), "max", int(wg_len.max()),
      "min", int(wg_len.min()))
print("WG start spread: max", int(start.min(1).max()))
for x in range(8):
    m = xcd == x
    print(f"XCD {x}: WGs {m.sum():3d} mean length {wg_len[m].mean():9.0f} max {wg_len[m].max():9.0f}")
for name, col in zip(("ratings", "runs", "hot-item ratings", "users"), st.T):
    print(f"corr(WG length, {name}) = {np.corrcoef(wg_len, col)[0, 1]:+.2f}")
print("within-WG end spread (max - min over waves), mean:", int((end.max(1) - end.min(1)).mean()))
plan.close()
ctx.close()
