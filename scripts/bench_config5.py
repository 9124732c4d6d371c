#!/usr/bin/env python3
"""BASELINE configs[4]: SVD nFactors=256 on the synthetic 10M users x 1M items x ~1B ratings set,
item-sharded (north_star).  Not the driver's bench line (bench.py is configs[1]); a separate
measurement script.

Single process:  python scripts/bench_config5.py [--shard p/n] [--users U --items I --mean-deg D]
  --shard 0/1  the whole set on one GPU (FAST epochs, rs_svd_plan_epochs)
  --shard p/n  item range [p I / n, (p + 1) I / n) only, run in the multi-GPU delta mode
               (rs_svd_plan_epoch_delta + apply_delta; with one process the all-reduce is the
               identity): the per-GPU work of an n-GPU run, measured on one GPU
torch.distributed (WORLD_SIZE > 1, backend nccl = RCCL): every rank generates its own item shard
  (rs_synth_create with the item range: the same full set, filtered) and runs rsgpu.multi's
  ItemShardedStep (one all-reduce of n_users x ld fp32 per epoch).

Data: rs_synth_create (lognormal user degree mean 100, Zipf(0.9) items over permuted ids, no repeated
(u, i), ratings 1..5 from a planted rank-4 model, seed 20250826); 0.1 % of the ratings are held out
(hash mask) for a device-side RMSE (rs_svd_plan_evaluate).  Factors: device init N(0, 0.1).
Hot items (Zipf head, up to ~1e7 ratings each) get row copies (rs_svd_plan_set_item_split) so the
memory-side float atomics of one row are not serialised.
Prints one JSON line per run (progress lines go to stderr).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle")]

HBM_PEAK = 8000.0


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def algorithmic_bytes(nnz, n_users, k):
    return nnz * (16 + 8 * k) + n_users * (16 + 8 * k)


def cpu_baseline(rowptr, cols, vals, n_users, n_items, k, budget_s, lr, reg):
    """C fp64 restatement of core/svd.go:92-130 (oracle), one thread, on the first users' ratings
    (CSR prefix) until ~budget_s of CPU work; updates/s."""
    import oracle as O
    m = int(np.searchsorted(rowptr, 2_000_000))
    u = np.repeat(np.arange(m, dtype=np.int32), np.diff(rowptr[:m + 1]))
    items, i = np.unique(cols[:len(u)], return_inverse=True)  # compact ids of the sample's items
    i, r = i.astype(np.int32), vals[:len(u)].astype(np.float64)
    rng = np.random.default_rng(0)
    P, Q = rng.normal(0, 0.1, (m, k)), rng.normal(0, 0.1, (len(items), k))
    done, t = 0, 0.0
    while t < budget_s:
        t0 = time.perf_counter()
        P, Q, *_ = O.svd_fit(u, i, r, P, Q, epochs=1, lr=lr, reg=reg)
        t += time.perf_counter() - t0
        done += len(u)
    return {"value": done / t, "unit": "updates/s", "cores": 1, "kind": "port",
            "sample": f"{done} updates over the first {m} users' {len(u)} ratings (CSR prefix), "
                      f"C fp64 restatement of core/svd.go:92-130, single thread, {t:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--mean-deg", type=float, default=100.0)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--shard", default="0/1")
    ap.add_argument("--partition", choices=("items", "users"), default="items",
                    help="items: north_star item-range shards + user-delta all-reduce; users: the dual "
                         "partition (user-range shards + item-delta all-reduce)")
    ap.add_argument("--item-cap", type=int, default=1 << 16)
    ap.add_argument("--split", type=int, default=-1, help="user split cap (-1: plan default)")
    ap.add_argument("--fixed-q", type=int, default=-1, help="fixed-point Q (-1: plan default)")
    ap.add_argument("--hot", type=int, default=-1, help="hot replicas n_hot (-1: plan default)")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--lr", type=float, default=0.005)
    ap.add_argument("--reg", type=float, default=0.02)
    args = ap.parse_args()

    import rsgpu
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        p, n = rank, world
    else:
        p, n = (int(x) for x in args.shard.split("/"))
    U_all, I, k = args.users, args.items, args.k
    by_users = args.partition == "users"
    lo, hi = (0, I) if by_users else (I * p // n, I * (p + 1) // n)
    ulo, uhi = (U_all * p // n, U_all * (p + 1) // n) if by_users else (0, U_all)
    U = uhi - ulo  # rows of this rank's plan

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = local if world > 1 else 0
    torch.cuda.set_device(dev)
    torch.cuda.init()
    ctx = rsgpu.Context(dev)  # device first: fail before minutes of data generation

    t0 = time.perf_counter()
    s = rsgpu.Synth(U_all, I, mean_deg=args.mean_deg, sigma=1.0, min_deg=1, max_deg=I // 2, zipf_s=0.9,
                    seed=20250826, item_lo=lo, item_hi=hi, user_lo=ulo, user_hi=uhi,
                    n_threads=args.threads)
    t_gen = time.perf_counter() - t0
    log(f"rank {rank}: generated users [{ulo}, {uhi}) x items [{lo}, {hi}): {s.nnz} ratings in {t_gen:.1f} s")
    deg = np.diff(s.rowptr)
    # hold out every 1024th rating of the CSR (rows are in random draw order)
    hold = np.zeros(s.nnz, bool)
    hold[::1024] = True
    users_h = np.repeat(np.arange(U, dtype=np.int32), deg)[hold]
    items_h, r_h = s.cols[hold].copy(), s.vals[hold].astype(np.float64)
    keep = ~hold
    tr_deg = deg - np.bincount(users_h, minlength=U)
    tr_rowptr = np.zeros(U + 1, np.int64)
    np.cumsum(tr_deg, out=tr_rowptr[1:])
    cols, vals = s.cols[keep], s.vals[keep]
    del keep, hold
    nnz = len(cols)
    item_cnt = np.bincount(cols, minlength=I)
    max_item = int(item_cnt.max()) if nnz else 0
    log(f"rank {rank}: train {nnz}, held out {len(r_h)}, max user deg {int(deg.max())}, "
        f"max item deg {max_item}")
    cpu = None
    if rank == 0 and args.cpu_budget > 0:
        cpu = cpu_baseline(tr_rowptr, cols, vals, U, I, k, args.cpu_budget, args.lr, args.reg)
        log(f"cpu baseline {cpu['value']:.3e} upd/s")
    s.close()

    t0 = time.perf_counter()
    plan = ctx.svd_plan_csr(U, I, tr_rowptr, cols, vals, k)
    if args.item_cap > 0:
        plan.set_item_split(args.item_cap)
    if args.split >= 0:
        plan.set_split(args.split)
    if args.fixed_q >= 0:
        plan.set_fixed_q(args.fixed_q)
    if args.hot >= 0:
        plan.set_hot_replicas(args.hot, 8)
    plan.init_normal(0.0, 0.1, seed=1)
    t_plan = time.perf_counter() - t0
    log(f"rank {rank}: plan built in {t_plan:.1f} s")
    del cols, vals
    stream = torch.cuda.current_stream(dev).cuda_stream
    delta = n > 1
    if delta:
        import rsgpu.multi as multi

        class _Solo:  # one process stands in for the n-way collective (identity all-reduce)
            @staticmethod
            def all_reduce(t, op=None):
                return None
        d = dist or _Solo
        local = item_cnt if by_users else tr_deg
        w, total_nnz = multi.count_weights(local, d, device=f"cuda:{dev}")
        if not dist:
            total_nnz = float(nnz) * n  # one process: one shard of an n-way run
        Step = multi.UserShardedStep if by_users else multi.ItemShardedStep
        step = Step(plan, d, w, total_nnz, device=f"cuda:{dev}", stream=stream)
        run = lambda e: step.run(e, args.lr, args.reg)
    else:
        run = lambda e: plan.epochs(e, args.lr, args.reg, stream)

    rmse0, _ = plan.evaluate(users_h, items_h, r_h)
    run(args.warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    run(args.epochs)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    log(f"rank {rank}: {args.epochs} epochs in {dt:.3f} s")
    plan.set_timing(True)
    run(1)
    kms, nl = plan.last_kernel_ms()
    plan.set_timing(False)
    rmse, mae = plan.evaluate(users_h, items_h, r_h)
    ab = algorithmic_bytes(nnz, U, k)
    total = nnz * (world if world > 1 else 1)
    if dist:
        tt = torch.tensor([float(nnz)], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(tt)
        total = float(tt.item())
    if rank == 0:
        line = {
            "config": "SVD nFactors=256 synthetic 10M x 1M x ~1B, item-sharded (BASELINE configs[4])",
            "shard": f"{p}/{n}" if world == 1 else f"all/{world}",
            "partition": args.partition,
            "n_gpus": world, "n_users": U_all, "users_this_rank": U, "n_items": I, "items_this_rank": hi - lo,
            "nnz_this_rank": nnz, "nnz_total": total, "n_factors": k,
            "max_user_deg": int(deg.max()), "max_item_deg": max_item, "item_cap": args.item_cap,
            "mode": "delta (multi-GPU protocol)" if delta else "single plan",
            "epochs": args.epochs, "epoch_s": dt / args.epochs,
            "updates_per_s": total * args.epochs / dt,
            "kernel_ms_per_epoch": kms / max(1, nl),
            "roofline": {"bound": "hbm", "algorithmic_bytes_per_launch": ab,
                         "achieved_GBs": ab / (kms / max(1, nl) / 1e3) / 1e9, "peak_GBs": HBM_PEAK,
                         "frac": ab / (kms / max(1, nl) / 1e3) / 1e9 / HBM_PEAK},
            "allreduce_bytes_per_epoch": ((I if by_users else U) * plan.ld * 4 + 8) if delta else 0,
            "holdout": {"n": int(len(r_h)), "rmse_init": rmse0, "rmse": rmse, "mae": mae,
                        "epochs_trained": args.warmup + args.epochs + 1},
            "gen_s": t_gen, "plan_build_s": t_plan,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    plan.close()
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
