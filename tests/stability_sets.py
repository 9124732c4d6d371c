"""FAST tile schedule stability at library defaults across set sizes, hot-item shares and k (test
infrastructure of tests/test_stability_gpu.py; round 4, VERDICT r3 "make the FAST default stable by rule").  rs_synth sets (lognormal user degrees, Zipf
items), 5 % held out, device init N(0, 0.1), GlobalBias = training mean; held-out RMSE after every epoch,
the run cap the library chose, and -- where the oracle is affordable -- the sequential reference
(core/svd.go:92-130 in a shuffled TrainSet order, same init) beside it.

    python tests/stability_sets.py [case ...] [--claim 0|4|8] [--cap C]
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle")]
import rsgpu  # noqa: E402

# name: (users, items, mean degree, zipf s, k, epochs, oracle)
CASES = {
    "1m_k64": (20000, 4000, 60.0, 0.9, 64, 10, True),
    "1m_k64_hot": (20000, 4000, 60.0, 1.1, 64, 10, True),
    "1m_k100_hot": (20000, 2000, 50.0, 1.2, 100, 10, True),
    "1m_k100_flat": (20000, 8000, 50.0, 0.6, 100, 10, True),
    "1m_k64_3pct": (20000, 2000, 50.0, 1.4, 64, 10, True),
    # round 6: hottest item just under the damping rule's 40 runs in flight (R = share x 176 x 16 on the library's grid):
    # 1.03 % (R ~ 29) and 1.13 % (R ~ 32) -- the plain kernel's upper range
    "1m_k64_r29": (20000, 4000, 60.0, 0.7, 64, 10, True),
    "1m_k100_r32": (20000, 2000, 50.0, 0.65, 100, 10, True),
    "8m_k100": (100000, 20000, 80.0, 0.9, 100, 8, False),
    "8m_k256_hot": (200000, 10000, 40.0, 1.1, 256, 5, False),
    "32m_k100": (400000, 50000, 80.0, 1.0, 100, 5, False),
    "128m_k256": (1250000, 125000, 100.0, 0.9, 256, 4, False),
}


def run(ctx, name, claim, cap, log, wg=0, damp=0.0, gb_fold=None, cold=None, ring=0):
    U, I, deg, zs, k, ep, with_oracle = CASES[name]
    t0 = time.time()
    s = rsgpu.Synth(U, I, mean_deg=deg, zipf_s=zs, seed=20250901, n_threads=16)
    d = np.diff(s.rowptr)
    users = np.repeat(np.arange(U, dtype=np.int32), d)
    hold = np.random.default_rng(0).random(s.nnz) < 0.05
    keep = ~hold
    rp = np.concatenate([[0], np.cumsum(np.bincount(users[keep], minlength=U))]).astype(np.int64)
    cols, vals = s.cols[keep].copy(), s.vals[keep].copy()
    hu, hi, hr = users[hold], s.cols[hold].copy(), s.vals[hold].astype(np.float64)
    s.close()
    nnz = len(cols)
    hot = int(np.bincount(cols, minlength=I).max())
    plan = ctx.svd_plan_csr(U, I, rp, cols, vals, k)
    plan.set_tile_claim(claim)
    if cap or wg or ring:
        plan.set_tiles(workgroups=wg, run_cap=cap, ring=ring)
    if gb_fold is not None:
        plan.set_gb_fold(gb_fold)
    if cold is not None:  # (experiment) cold runs' write-through (rs_svd_plan_set_cold_store)
        plan.set_cold_store(cold)
    if damp:  # (experiment) the damped kernel with R = deg x damp runs in flight (rs_svd_plan_set_damp_concurrency)
        plan.set_damp_concurrency(damp)
    plan.init_normal(0.0, 0.1, seed=1)
    gb0 = float(np.mean(vals, dtype=np.float64))
    plan.upload(gb=gb0)
    ref_curve = None
    if with_oracle:
        import oracle as O
        P0, Q0, bu0, bi0, _ = plan.download()
        uu = np.repeat(np.arange(U, dtype=np.int32), np.diff(rp))
        # the reference visits its TrainSet in data order, which KFold has shuffled (data.go:49-70): a seeded
        # permutation of the ratings (round 5; round 4 used the user-major CSR order, which trains worse)
        perm = np.random.default_rng(7).permutation(len(cols))
        ou, oi, ov = uu[perm], cols[perm].astype(np.int32), vals[perm].astype(np.float64)
        P, Q, bu, bi, g = P0, Q0, bu0, bi0, gb0
        ref_curve = []
        for _ in range(ep):
            P, Q, bu, bi, g = O.svd_fit(ou, oi, ov, P, Q, bu, bi, g, epochs=1)
            ref_curve.append(float(np.sqrt(np.mean((O.svd_predict(hu, hi, P, Q, bu, bi, g) - hr) ** 2))))
    r0 = plan.evaluate(hu, hi, hr)[0]
    curve = []
    plan.set_timing(True)
    ms = 0.0
    for _ in range(ep):
        plan.epochs(1)
        m, _n = plan.last_kernel_ms()
        ms += m
        curve.append(plan.evaluate(hu, hi, hr)[0])
    try:
        plan.download()
        numeric = "ok"
    except rsgpu.RsError as e:
        numeric = f"RS_ERR {e.code}"
    refits = plan.refits()
    plan.close()
    out = {"nnz": nnz, "hot_share": hot / nnz, "k": k, "rmse0": r0, "curve": curve, "ref_curve": ref_curve,
           "numeric": numeric, "epoch_ms": ms / ep, "refits": refits}
    log(f"{name:12s} claim {claim} cap {cap or 'auto'} wg {wg or 'all'}: nnz {nnz} hottest {hot} ({100.0 * hot / nnz:.2f} %) k {k} "
        f"epoch {ms / ep:.2f} ms  held-out {r0:.4f} -> " + " ".join(f"{x:.4f}" for x in curve) +
        (("  | reference " + " ".join(f"{x:.4f}" for x in ref_curve)) if ref_curve else "") +
        f"  [{numeric}, refits {refits}, {time.time() - t0:.0f} s]")
    return out


def run_fit(ctx, name, log):
    """The Go drop-in (rs_svd_fit: host COO in, guarded refits) on the same set: held-out RMSE and refits."""
    U, I, deg, zs, k, ep, _ = CASES[name]
    s = rsgpu.Synth(U, I, mean_deg=deg, zipf_s=zs, seed=20250901, n_threads=16)
    users = np.repeat(np.arange(U, dtype=np.int32), np.diff(s.rowptr))
    hold = np.random.default_rng(0).random(s.nnz) < 0.05
    keep = ~hold
    u, i, r = users[keep], s.cols[keep].copy(), s.vals[keep].astype(np.float64)
    hu, hi, hr = users[hold], s.cols[hold].copy(), s.vals[hold].astype(np.float64)
    s.close()
    rng = np.random.default_rng(1)
    P0, Q0 = rng.normal(0, 0.1, (U, k)), rng.normal(0, 0.1, (I, k))
    t0 = time.time()
    try:
        got = ctx.svd_fit(rsgpu.Ratings(u, i, r, U, I), P0, Q0, n_epochs=ep)
        import oracle as O
        e = float(np.sqrt(np.mean((O.svd_predict(hu, hi, *got) - hr) ** 2)))
        res = f"held-out RMSE after {ep} epochs {e:.4f}"
    except rsgpu.RsError as x:
        e = None
        res = f"RS_ERR {x.code}"
    log(f"{name:12s} rs_svd_fit: {res}, refits {ctx.fit_refits()} ({time.time() - t0:.1f} s)")
    return {"rmse": e, "refits": ctx.fit_refits()}


def run_diag(ctx, name, wg=0, epochs=None, log=print):
    """Guard off: per epoch the held-out RMSE, the largest |factor| / |bias| and where (item's rating rank),
    to find the rows that run away without the guard's redo."""
    U, I, deg, zs, k, ep, _ = CASES[name]
    ep = epochs or ep
    s = rsgpu.Synth(U, I, mean_deg=deg, zipf_s=zs, seed=20250901, n_threads=16)
    d = np.diff(s.rowptr)
    users = np.repeat(np.arange(U, dtype=np.int32), d)
    hold = np.random.default_rng(0).random(s.nnz) < 0.05
    keep = ~hold
    rp = np.concatenate([[0], np.cumsum(np.bincount(users[keep], minlength=U))]).astype(np.int64)
    cols, vals = s.cols[keep].copy(), s.vals[keep].copy()
    hu, hi, hr = users[hold], s.cols[hold].copy(), s.vals[hold].astype(np.float64)
    s.close()
    cnt = np.bincount(cols, minlength=I)
    rank = np.empty(I, np.int64)
    rank[np.argsort(-cnt, kind="stable")] = np.arange(I)
    plan = ctx.svd_plan_csr(U, I, rp, cols, vals, k)
    plan.set_guard(False)
    if wg:
        plan.set_tiles(workgroups=wg)
    plan.init_normal(0.0, 0.1, seed=1)
    plan.upload(gb=float(np.mean(vals, dtype=np.float64)))
    for e in range(ep):
        plan.epochs(1)
        try:
            P, Q, bu, bi, g = plan.download()
        except rsgpu.RsError as x:
            log(f"{name} wg {wg or 'auto'} epoch {e + 1}: download RS_ERR {x.code}")
            break
        qa = np.abs(Q).max(1)
        top = np.argsort(-qa)[:3]
        rm = plan.evaluate(hu, hi, hr)[0]
        log(f"{name} wg {wg or 'auto'} epoch {e + 1}: held-out {rm:.4f} gb {g:.3f} max|P| {np.abs(P).max():.3f} "
            f"max|bu| {np.abs(bu).max():.3f} max|bi| {np.abs(bi).max():.3f} (item rank {rank[int(np.argmax(np.abs(bi)))]}) "
            f"max|Q| rows " + ", ".join(f"{qa[t]:.3f}@rank{rank[t]}({cnt[t]})" for t in top))
    plan.close()


def nnz_of(name):
    """the training ratings of a case (95 % of the generated set)"""
    U, I, deg, zs, k, ep, _ = CASES[name]
    s = rsgpu.Synth(U, I, mean_deg=deg, zipf_s=zs, seed=20250901, n_threads=16)
    n = s.nnz
    s.close()
    return 0.95 * n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*", default=list(CASES))
    ap.add_argument("--claim", type=int, default=4)
    ap.add_argument("--cap", type=int, default=0)
    ap.add_argument("--wg", type=int, default=0, help="workgroups (0: one per CU)")
    ap.add_argument("--gb-fold", type=int, default=None, help="0 mean, 1 smoothed (default: library)")
    ap.add_argument("--ring", type=int, default=0, help="q rows prefetched per wave (0: library)")
    ap.add_argument("--cold", type=float, default=None, help="cold-store runs in flight (default: library)")
    ap.add_argument("--damp", type=float, default=0.0, help="force the damped kernel, R = deg x DAMP x nnz (natural: grid x waves)")
    ap.add_argument("--fit", action="store_true", help="through rs_svd_fit (the guarded Go drop-in)")
    ap.add_argument("--diag", action="store_true", help="guard off, per-epoch extremes (run_diag)")
    args = ap.parse_args()
    ctx = rsgpu.Context(0)
    for c in args.cases:
        if args.diag:
            run_diag(ctx, c, args.wg)
        elif args.fit:
            run_fit(ctx, c, lambda m: print(m, flush=True))
        else:
            run(ctx, c, args.claim, args.cap, lambda m: print(m, flush=True), args.wg, damp=args.damp / nnz_of(c) if args.damp else 0.0,
                gb_fold=args.gb_fold, cold=args.cold, ring=args.ring)
    ctx.close()


if __name__ == "__main__":
    main()
