"""Experiment: is the coherent (sc1 / atomic) SGD epoch bound by hot-row contention?
Compares the ML-1M-shaped set (Zipf items) against the same user degrees with uniform items."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu
from rsgpu import synth
ctx = rsgpu.Context(0)
u, i, r, nu, ni = synth.ml1m_like()
rng = np.random.default_rng(5)
deg = np.bincount(u, minlength=nu)
ui = np.concatenate([rng.choice(ni, d, replace=False) for d in deg])
uu = np.repeat(np.arange(nu), deg)
perm = rng.permutation(len(uu))
sets = {"zipf": (u, i), "uniform": (uu[perm].astype(np.int32), ui[perm].astype(np.int32))}
capped = deg.copy(); capped = np.minimum(capped, 200)
for name, (su, si) in sets.items():
    for wb, aux in [(1, 16), (0, 16), (0, 0)]:
        os.environ["RSGPU_SGD_WB"] = str(wb); os.environ["RSGPU_SGD_AUX"] = str(aux); os.environ["RSGPU_SGD_RING"] = "8"
        plan = ctx.svd_plan(rsgpu.Ratings(su, si, r, nu, ni), 100)
        plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
        plan.set_timing(True); plan.epochs(5)
        ms, n = plan.last_kernel_ms(); plan.close()
        print(f"{name} wb={wb} aux={aux} epoch_us={ms/n*1e3:.1f}", flush=True)
# heavy-user chain check: cap every user at 200 ratings (uniform items)
keep = np.zeros(len(uu), bool); seen = np.zeros(nu, int)
su, si = sets["uniform"]
for t in range(len(su)):
    if seen[su[t]] < 200: keep[t] = True; seen[su[t]] += 1
for wb, aux in [(1, 16), (0, 0)]:
    os.environ["RSGPU_SGD_WB"] = str(wb); os.environ["RSGPU_SGD_AUX"] = str(aux)
    plan = ctx.svd_plan(rsgpu.Ratings(su[keep], si[keep], r[keep], nu, ni), 100)
    plan.upload(rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100)), np.zeros(nu), np.zeros(ni), 0.0)
    plan.set_timing(True); plan.epochs(5)
    ms, n = plan.last_kernel_ms(); plan.close()
    print(f"uniform-cap200 nnz={keep.sum()} wb={wb} aux={aux} epoch_us={ms/n*1e3:.1f}", flush=True)
