#!/usr/bin/env python3
"""Measures the BASELINE.json configurations that bench.py does not cover (bench.py = configs[1]):

  0    configs[0]: SVD nFactors=20, 5-fold ML-100K (the reference's own u.data), CPU: the C fp64
       restatement of core/svd.go:63-132 on one core (the Go Fit() plumbing of benchmark.go:12-52),
       with the GPU fit of the same folds beside it
  2    configs[2]: SVD++ nFactors=128 on an ML-1M-shaped set (FAST lazy-y kernel K2)
  3    configs[3]: KNN item-based Cosine on an ML-20M-shaped set (int8-MFMA K4)
  4    configs[4]: SVD nFactors=256 on the 1/8 item shard of the 10M x 1M x 1e9 synthetic set (one
       GPU's share of the item-sharded fit), library defaults (tile schedule K1)
  nmf  NMF nFactors=15 on the ML-1M-shaped set (K3; no BASELINE config)

Each line: kernel-only device time (HIP events on the launch stream, rs_last_kernel_ms), the
roofline fraction against the bound SURVEY §8d names, and a CPU baseline timed on this host on a
bounded sample of the same workload (the oracle: C fp64 restatement of the reference, 1 thread).
Writes JSON lines to stdout (and --out).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the oracle's nJobs restatements fork/join once per rating (svd.go:399-422): spinning OpenMP workers
# stand in for Go's spinning scheduler threads (a sleeping pool would charge a wake-up per rating)
os.environ.setdefault("OMP_WAIT_POLICY", "ACTIVE")
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle")]

HBM_PEAK = 8000.0      # GB/s, MI355X_MICROARCH.md chip table
I8_PEAK = 5000.0       # dense int8 MFMA TOP/s: 2x the ~2.5 PF dense bf16 rate (microarch: i8 2x bf16)


def emit(d, out):
    line = json.dumps(d)
    print(line, flush=True)
    if out:
        with open(out, "a") as f:
            f.write(line + "\n")


def host_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "cpu_model": model}


def cpu_jobs():
    """Threads for the reference's nJobs = runtime.NumCPU() fan-out: the CPUs this process may use,
    capped at the box's per-GPU share (OMP_NUM_THREADS, 16 on the GPU box)."""
    avail = len(os.sched_getaffinity(0))
    return max(1, min(avail, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def config0(ctx, out, k=20, epochs=20):
    import oracle as O
    import rsgpu
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from helpers import folds, rmse
    d = np.load(os.path.join(REPO, "tests", "golden", "ml100k.npz"))
    U, I, R = d["users"].astype(np.int64), d["items"].astype(np.int64), d["ratings"].astype(np.float64)
    fl = folds(U, I, R)
    cpu_s, gpu_s, cpu_rmse, gpu_rmse, n_upd = 0.0, 0.0, [], [], 0
    for f in fl:
        rng = np.random.default_rng(7)
        P0, Q0 = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
        t0 = time.perf_counter()
        m = O.svd_fit(f.iu, f.ii, f.r, P0, Q0, epochs=epochs)
        cpu_s += time.perf_counter() - t0
        cpu_rmse.append(rmse(O.svd_predict(f.tu, f.ti, *m), f.te_r))
        rr = rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni)
        ctx.svd_fit(rr, P0, Q0, n_epochs=1)  # warm-up (code objects, allocator)
        t0 = time.perf_counter()
        g = ctx.svd_fit(rr, P0, Q0, n_epochs=epochs)
        gpu_s += time.perf_counter() - t0
        gpu_rmse.append(rmse(O.svd_predict(f.tu, f.ti, *g), f.te_r))
        n_upd += len(f.r) * epochs
    emit({"config": "SVD nFactors=20, 5-fold CV on ML-100K (BASELINE configs[0], reference's own u.data)",
          "cpu": {"fit_s_5_folds": cpu_s, "updates_per_s": n_upd / cpu_s, "cores": 1, "kind": "port",
                  "what": "oracle C fp64 restatement of core/svd.go:63-132 (reference visit order), "
                          "one thread, 20 epochs per fold", **host_info()},
          "rmse_cpu_mean": float(np.mean(cpu_rmse)),
          "gpu": {"fit_s_5_folds": gpu_s, "updates_per_s": n_upd / gpu_s,
                  "what": "rs_svd_fit (one-shot Fit through the C-ABI, FAST tile schedule), wall "
                          "time per call incl. host packing and H2D/D2H"},
          "rmse_gpu_mean": float(np.mean(gpu_rmse)),
          "reference_bound": "core/base_test.go:35 checks RMSE <= 0.942 on this CV"}, out)


def config2(ctx, out, epochs=5):
    import oracle as O
    import rsgpu
    from rsgpu import synth
    u, i, r, nu, ni = synth.ml1m_like()
    k = 128
    rng = np.random.default_rng(3)
    P0, Q0, Y0 = (rng.normal(0, 0.1, (m, k)) for m in (nu, ni, ni))
    R = rsgpu.Ratings(u, i, r, nu, ni)
    ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=1)            # warm-up (code objects, allocator)
    t0 = time.perf_counter()
    ctx.svdpp_fit(R, P0, Q0, Y0, n_epochs=epochs)
    wall = time.perf_counter() - t0
    ms = ctx.last_kernel_ms() / epochs
    nnz = len(r)
    ab = nnz * (16 + 8 * k) + nu * (16 + 8 * k) + nnz * (4 + 12 * k)
    # CPU: the literal svd.go:316-427 restatement with the reference's own parallelism -- the y-update
    # of every rating split over nJobs threads (svd.go:399-422, one fork/join per rating) -- on a
    # uniform sample of the epoch: ratings of the shuffled set with their FULL N(u) (the epoch's
    # per-rating cost depends only on |N(u)|), timed as a slice of a real epoch
    jobs = cpu_jobs()
    m = 4000
    t0 = time.perf_counter()
    O.svdpp_fit_sample(u, i, r, nu, P0, Q0, Y0, m, n_jobs=jobs)
    t_rating = (time.perf_counter() - t0) / m
    t0 = time.perf_counter()
    O.svdpp_fit_sample(u, i, r, nu, P0, Q0, Y0, m // 4, n_jobs=1)
    t_rating1 = (time.perf_counter() - t0) / (m // 4)
    emit({"config": "SVD++ nFactors=128 ML-1M-shaped (BASELINE configs[2])", "kernel": "svdpp_epoch_fast_kernel<E=3,D=8>",
          "updates_per_s": nnz / (ms / 1e3), "epoch_ms_kernel": ms, "fit_wall_s": wall,
          "roofline": {"bound": "hbm", "achieved_GBs": ab / (ms / 1e3) / 1e9, "peak_GBs": HBM_PEAK,
                       "frac": ab / (ms / 1e3) / 1e9 / HBM_PEAK, "algorithmic_bytes": ab},
          "cpu_baseline": {"value": 1.0 / t_rating, "unit": "updates/s", "cores": jobs, "kind": "port",
                           "sample": f"literal svd.go:352-424 restatement with svd.go:399-422's nJobs = {jobs} "
                                     f"split of every rating's y-update (OpenMP fork/join per rating), the first "
                                     f"{m} ratings of the shuffled ML-1M-shaped epoch against the full N(u); "
                                     f"1 thread: {1.0 / t_rating1:.3g} updates/s",
                           **host_info()}}, out)


def config3(ctx, out):
    import oracle as O
    import rsgpu
    from rsgpu import synth
    u, i, r, nu, ni = synth.ml20m_like()
    order = np.argsort(i, kind="stable")
    rowptr = np.zeros(ni + 1, np.int64)
    np.add.at(rowptr, i.astype(np.int64) + 1, 1)
    rowptr = np.cumsum(rowptr)
    ids, rr = u[order], r[order]
    L, R = ni, nu
    t0 = time.perf_counter()
    S = ctx.knn_sims(rsgpu.SIM_COSINE, rowptr, ids, rr, R)
    wall = time.perf_counter() - t0
    ms = ctx.last_kernel_ms()
    Lp = (L + 127) // 128 * 128
    T = Lp // 128
    kpad = (R + 63) // 64 * 64
    executed = 3 * 2 * (T * (T + 1) // 2) * 128 * 128 * kpad     # 3 int8 contractions, triangle tiles
    algorithmic = 2 * 2 * L * (L + 1) // 2 * R                    # G=2, unique pairs
    # CPU: the reference-style merge (sim.go:10-25) on nJobs threads over a 512-row block (knn.go:192-216
    # splits the rows into contiguous ranges, one per goroutine), every row against every partner,
    # extrapolated to the unique pairs of the full matrix (knn.go skips computed mirrors) -- BASELINE.md
    srt = np.lexsort((ids, np.repeat(np.arange(L), np.diff(rowptr))))
    sid, sr = ids[srt], rr[srt]
    rows, jobs = 512, cpu_jobs()
    t0 = time.perf_counter()
    blk = O.knn_sims_rows_mt(O.COSINE, rowptr, sid, sr, 0, rows, jobs)
    t_blk = time.perf_counter() - t0
    t_full = t_blk * (L / rows) / 2
    same = np.array_equal(np.isnan(blk), np.isnan(S[:rows])) and np.array_equal(
        blk[~np.isnan(blk)].view(np.uint64), S[:rows][~np.isnan(blk)].view(np.uint64))
    emit({"config": "KNN item-based Cosine ML-20M-shaped (BASELINE configs[3])",
          "kernel": "knn_sims_mfma_kernel<Cosine> (v_mfma_i32_32x32x32_i8)",
          "L": L, "R": R, "nnz": int(len(r)), "kernel_ms": ms, "fit_wall_s": wall,
          "pairs_per_s": L * (L - 1) / 2 / (ms / 1e3),
          "roofline": {"bound": "mfma", "achieved_TOPs_executed": executed / (ms / 1e3) / 1e12,
                       "achieved_TOPs_algorithmic": algorithmic / (ms / 1e3) / 1e12,
                       "peak_TOPs": I8_PEAK, "frac": algorithmic / (ms / 1e3) / 1e12 / I8_PEAK,
                       "frac_executed": executed / (ms / 1e3) / 1e12 / I8_PEAK,
                       "executed_int8_ops": executed, "algorithmic_int8_ops": algorithmic},
          "parity_rows_0_511_bitwise": bool(same),
          "cpu_baseline": {"value": L * (L - 1) / 2 / t_full, "unit": "pairs/s", "cores": jobs,
                           "kind": "port", "sample": f"rows 0-{rows - 1} x {L} partners, merge "
                           f"restatement on {jobs} threads (knn.go:192-216's contiguous row split) "
                           f"{t_blk:.1f} s, extrapolated x{L / rows / 2:.1f} to the unique pairs "
                           f"({t_full:.0f} s)", **host_info()}}, out)


def config4(ctx, out, epochs=5):
    import rsgpu
    n_users, n_items, k = 10_000_000, 1_000_000, 256
    t0 = time.perf_counter()
    s = rsgpu.Synth(n_users, n_items, mean_deg=100.0, seed=20250826, item_lo=0, item_hi=n_items // 8,
                    n_threads=16)
    t_gen = time.perf_counter() - t0
    t0 = time.perf_counter()
    plan = ctx.svd_plan_csr(n_users, n_items, s.rowptr, s.cols, s.vals, k)
    t_build = time.perf_counter() - t0
    plan.init_normal(0.0, 0.1, seed=1)
    plan.epochs(1)
    plan.set_timing(True)
    plan.epochs(epochs)
    ms, nl = plan.last_kernel_ms()
    plan.set_timing(False)
    P, Q, bu, bi, gb = plan.download()
    finite = bool(np.isfinite(Q).all() and np.isfinite(P).all() and np.isfinite(gb))
    nnz = s.nnz
    ab = nnz * (16 + 8 * k) + n_users * (16 + 8 * k)
    t_ep = ms / nl / 1e3
    plan.close()
    s.close()
    emit({"config": "SVD nFactors=256, 1/8 item shard of the 10M x 1M x 1e9 synthetic set (BASELINE configs[4], one GPU's share)",
          "kernel": "svd_epoch_tile_kernel<E=5,NW=16,RQ=2> (library defaults)",
          "nnz": int(nnz), "epoch_ms_kernel": t_ep * 1e3, "updates_per_s": nnz / t_ep,
          "plan_build_s": t_build, "synth_s": t_gen, "finite": finite,
          "roofline": {"bound": "hbm", "achieved_GBs": ab / t_ep / 1e9, "peak_GBs": HBM_PEAK,
                       "frac": ab / t_ep / 1e9 / HBM_PEAK, "algorithmic_bytes": ab}}, out)


def nmf(ctx, out, epochs=50):
    import oracle as O
    import rsgpu
    from rsgpu import synth
    u, i, r, nu, ni = synth.ml1m_like()
    k = 15
    rng = np.random.default_rng(5)
    P0, Q0 = rng.uniform(0, 1, (nu, k)), rng.uniform(0, 1, (ni, k))
    R = rsgpu.Ratings(u, i, r, nu, ni)
    ctx.nmf_fit(R, P0, Q0, n_epochs=1, as_written=False)
    ctx.nmf_fit(R, P0, Q0, n_epochs=epochs, as_written=False)
    ms = ctx.last_kernel_ms() / epochs
    nnz = len(r)
    ab = nnz * (8 + 20 * k) + nu * 28 * k + ni * 24 * k
    t0 = time.perf_counter()
    O.nmf_fit(u, i, r, P0, Q0, epochs=1, as_written=False)
    t_cpu = time.perf_counter() - t0
    emit({"config": "NMF nFactors=15 ML-1M-shaped (no BASELINE config)", "kernel": "nmf_chunk_kernel<16,1> + nmf_combine_kernel, item and user pass",
          "updates_per_s": nnz / (ms / 1e3), "epoch_ms_kernel": ms,
          "roofline": {"bound": "hbm", "achieved_GBs": ab / (ms / 1e3) / 1e9, "peak_GBs": HBM_PEAK,
                       "frac": ab / (ms / 1e3) / 1e9 / HBM_PEAK, "algorithmic_bytes": ab},
          "cpu_baseline": {"value": nnz / t_cpu, "unit": "updates/s", "cores": 1, "kind": "port",
                           "sample": "1 epoch, svd.go:178-250 restatement"}}, out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="0,2,3,4,nmf")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import rsgpu
    ctx = rsgpu.Context(0)
    which = a.only.split(",")
    for name, fn in (("0", config0), ("2", config2), ("nmf", nmf), ("3", config3), ("4", config4)):
        if name in which:
            print(f"running {name}", file=sys.stderr, flush=True)
            fn(ctx, a.out)
    ctx.close()


if __name__ == "__main__":
    main()
