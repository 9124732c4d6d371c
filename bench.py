#!/usr/bin/env python3
"""bench.py -- SGD updates/s of SVD k=100 on a MovieLens-1M-shaped set (BASELINE.json configs[1]).

One step = one fast-mode SGD epoch (core/svd.go:92-130) over all 1,000,209 ratings, inputs resident
in HBM (user-CSR + factors uploaded before the timed region).  N>1 GPUs: one process per GPU
(torch.distributed for the barriers and the max-over-ranks clock); each rank owns its own item-range
shard of ML-1M size (weak scaling, the 6040 users shared) and the library's own RCCL communicator
(rs_svd_plan_join) runs north_star's protocol: one full-shard epoch per rank, then one RCCL all-reduce of the
count-weighted user deltas (RS_EXCHANGE_AVERAGE, one user block).  The exact stratum rotation (RS_EXCHANGE_ROTATE,
rs_svd_fit_multi's choice for item shards) trains each rank's epoch as N x 2 user-block launches; on an ML-1M-sized
shard those cost 144 / 299 / 916 us per epoch at 1 / 2 / 8 ranks' blocks (profiles/r06/rotate_blocks_ml1m.log), a
launch-size cost that a weak-scaling line of ML-1M shards would mostly measure.

Launch: under torch.distributed.run (WORLD_SIZE set) every process is one rank.  `--gpus N` with
N > 1 and no WORLD_SIZE starts the N rank processes itself from a parent that makes no GPU call, and
fails when fewer than N GPUs are visible.

Extra fields of the same line:
  strong_scaling  BASELINE configs[4] at full size (10M users x 1M items x ~1e9 ratings, k = 256), user
                  ranges over the N ranks, the ranks' item moves all-reduced 16 times per epoch (RS_EXCHANGE_QDELTA,
                  fp16 moves, each all-reduce behind the next block's kernel) -- the north_star scaling question;
                  the driver's N = 1, 2, 4, 8 lines give its curve.  One timed call of 20 epochs (a default Fit,
                  core/svd.go:66).  About a minute at N = 1 (generation ~35 s, plan ~10-30 s, 21 epochs of ~0.6 s).
  ordered         N = 1: throughput of the ORDERED mode (the reference visit order, the mode that
                  meets north_star's 1e-5 factor contract) on the same ML-1M-shaped set.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "recommend-sys_amd"))

METRIC = "SGD updates/sec, SVD k=100 MovieLens-1M, 1/2/4/8 GPU; % HBM roofline"
K = 100
LR, REG = 0.005, 0.02
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
EXCHANGE_NAMES = {0: "RS_EXCHANGE_ROTATE (stratum rotation)", 1: "RS_EXCHANGE_AVERAGE", 2: "RS_EXCHANGE_ROTATE_Q",
                  3: "RS_EXCHANGE_QDELTA"}
# what each exchange sends between the ranks (include/rsgpu.h)
EXCHANGE_WIRE = {0: "RCCL send/recv of P rank-blocks per sub-epoch",
                 1: "RCCL all-reduce of count-weighted user deltas once per epoch (one user block)",
                 2: "RCCL send/recv of Q rank-blocks and hot-item copies per sub-epoch",
                 3: "RCCL all-reduce of weighted fp16 item moves per merge"}


def algorithmic_bytes(nnz, n_users, k):
    """nnz*(16 + 8k) + U*(16 + 8k) per epoch (fp32 factors, int32 idx, fp32 rating)."""
    return nnz * (16 + 8 * k) + n_users * (16 + 8 * k)


def cpu_baseline(u, i, r, n_users, n_items, budget_s=10.0):
    """Times the C restatement of core/svd.go:63-132 (oracle, fp64, single thread) on whole epochs
    of the same workload until ~budget_s of CPU work has run."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    rng = np.random.default_rng(0)
    P, Q = rng.normal(0, 0.1, (n_users, K)), rng.normal(0, 0.1, (n_items, K))
    bu, bi, gb = np.zeros(n_users), np.zeros(n_items), 0.0
    epochs, t_total = 0, 0.0
    while t_total < budget_s and epochs < 100:
        t0 = time.perf_counter()
        P, Q, bu, bi, gb = O.svd_fit(u, i, r, P, Q, bu, bi, gb, epochs=1, lr=LR, reg=REG)
        t_total += time.perf_counter() - t0
        epochs += 1
    return {"value": len(r) * epochs / t_total, "unit": "updates/s", "cores": 1, "kind": "port",
            "sample": f"{epochs} full epoch(s) of the same {len(r)}-rating set, C fp64 restatement "
                      f"of core/svd.go:92-130 (oracle/), single thread, {t_total:.1f} s"}


def strong_scaling(ctx, rank, world, dist, dev, stream, epochs=20, warmup=1):
    """BASELINE configs[4] at its own size: SVD nFactors=256 on the synthetic 10M users x 1M items x ~1e9
    ratings set (rs_synth, seed 20250826 -- the set tests/test_config4_gpu.py fits), library defaults.  Rank r
    generates and holds users [U r / N, U (r + 1) / N) (global ids, every item); with N > 1 the library's RCCL
    communicator runs RS_EXCHANGE_QDELTA (each rank trains its users against the whole Q in 16 blocks; after each
    block the ranks' weighted item moves are all-reduced as fp16 while the next block trains, csrc/multi.hip).
    One timed call of `epochs` epochs: a default Fit is 20 (core/svd.go:66), and P's ranges are broadcast once
    per call."""
    import torch
    import rsgpu
    n_users, n_items, k = 10_000_000, 1_000_000, 256
    lo, hi = n_users * rank // world, n_users * (rank + 1) // world
    t0 = time.perf_counter()
    s = rsgpu.Synth(n_users, n_items, mean_deg=100.0, sigma=1.0, min_deg=1, max_deg=n_items // 2, zipf_s=0.9,
                    seed=20250826, user_lo=lo, user_hi=hi, n_threads=16)
    rp = np.empty(n_users + 1, np.int64)  # this range's CSR as rows 0..U-1 (empty rows elsewhere)
    rp[:lo + 1] = 0
    rp[lo + 1:hi + 1] = s.rowptr[1:]
    rp[hi + 1:] = s.rowptr[-1]
    nnz, vsum = s.nnz, float(np.sum(s.vals, dtype=np.float64))
    probe_u = np.repeat(np.arange(lo, hi, dtype=np.int32), np.diff(s.rowptr))[:4096]
    probe_i, probe_r = s.cols[:len(probe_u)].copy(), s.vals[:len(probe_u)].astype(np.float64)
    gen_s = time.perf_counter() - t0
    print(f"bench: strong_scaling rank {rank}/{world}: users [{lo}, {hi}), {nnz} ratings generated in {gen_s:.1f} s",
          file=sys.stderr, flush=True)
    plan = ctx.svd_plan_csr(n_users, n_items, rp, s.cols, s.vals, k)
    s.close()
    del rp
    plan.init_normal(0.0, 0.1, seed=1)  # rows drawn by row id: every rank's P / Q equal one plan's
    tot = torch.tensor([float(nnz), vsum], dtype=torch.float64, device=f"cuda:{dev}")
    if dist:
        dist.all_reduce(tot)
    plan.upload(gb=float(tot[1] / tot[0]))  # the training mean: the same GlobalBias on every rank
    if dist:
        plan.set_exchange(rsgpu.EXCHANGE_QDELTA)
        uid = [rsgpu.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        plan.join(uid[0], rank, world)
        _, _, _, n_blocks = plan.shard_info()
        run = lambda n: plan.epochs_sharded(n, LR, REG, stream)
    else:
        n_blocks = 1
        run = lambda n: plan.epochs(n, LR, REG, stream)
    setup_s = time.perf_counter() - t0
    print(f"bench: strong_scaling rank {rank}/{world}: plan ready at {setup_s:.1f} s ({n_blocks} blocks)", file=sys.stderr,
          flush=True)
    run(warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(epochs)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    try:  # RMSE over this rank's first ratings: the device's fixed-point / non-finite check of the factors
        finite = bool(np.isfinite(plan.evaluate(probe_u, probe_i, probe_r)[0]))
    except rsgpu.RsError:
        finite = False
    plan.close()
    total = int(tot[0].item())
    return {"workload": "BASELINE configs[4]: SVD nFactors=256 on the synthetic 10M users x 1M items x "
                        f"{total} ratings set (rs_synth seed 20250826, lognormal user degrees mean 100, Zipf 0.9 "
                        f"items), library defaults, user ranges over {world} GPU(s)",
            "scaling": "strong", "n_gpus": world, "epochs": epochs, "warmup": warmup,
            "value": total * epochs / dt, "unit": "updates/s", "ms_per_epoch": dt / epochs * 1e3,
            "gen_s_rank0": gen_s, "setup_s_rank0": setup_s, "finite": finite, "item_blocks": n_blocks,
            "exchange": f"rs_svd_plan_join + rs_svd_plan_epochs_sharded, RS_EXCHANGE_QDELTA ({n_blocks} merges per "
                        "epoch: RCCL all-reduce of the ranks' weighted item moves as fp16, each behind the next "
                        "block's kernel; P ranges broadcast once per call)"
                        if world > 1 else "none (one GPU, one plan over the whole set)"}


def ordered_throughput(ctx, u, i, r, n_users, n_items):
    """ORDERED mode (core/svd.go:93-129 in the reference's visit order), one epoch, kernel time."""
    import rsgpu
    rng = np.random.default_rng(1)
    P0, Q0 = rng.normal(0, 0.1, (n_users, K)), rng.normal(0, 0.1, (n_items, K))
    R = rsgpu.Ratings(u, i, r, n_users, n_items)
    n_w = min(len(r), 20000)  # warm-up on a prefix: the first launch of the kernel loads its code object
    ctx.svd_fit(rsgpu.Ratings(u[:n_w], i[:n_w], r[:n_w], n_users, n_items), P0[:, :K], Q0, n_epochs=1,
                mode=rsgpu.SGD_ORDERED)
    ctx.svd_fit(R, P0[:, :K], Q0, n_epochs=1, mode=rsgpu.SGD_ORDERED)
    ms = ctx.last_kernel_ms()
    return {"value": len(r) / (ms / 1e3), "unit": "updates/s", "epoch_ms_kernel": ms,
            "note": "one workgroup walks the ratings in the reference order in conflict-free batches (no user "
                    "or item twice, <= 64 ratings, a 16-lane group per rating; rows prefetched a batch ahead, the "
                    "previous batch's rows "
                    "forwarded through LDS, the GlobalBias chain as a lane-parallel scan; factors within 1e-5 "
                    "of the oracle; csrc/sgd_ordered.hip); kernel-only time of one epoch"}


def load_traffic():
    """HBM bytes per SGD launch measured by rocprofv3 --pmc (separate pass, committed summary)."""
    p = os.path.join(REPO, "profiles", "sgd_traffic.json")
    if os.path.exists(p):
        try:
            return json.load(open(p)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def measure_traffic():
    """HBM bytes per SGD launch, measured now: two rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE: they
    do not fit one pass's TCC slots), kernel trace only, each a child process running the same workload
    without torch (scripts/experiments/tile_epochs.py; PMC passes under torch's runtime hung on this image),
    summarised with the gfx950 FETCH_SIZE x 2 correction (scripts/pmc_summary.py).  Returns (bytes, None) or
    (None, reason).  RS_BENCH_PMC=0 skips it."""
    import shutil
    import subprocess
    import tempfile
    if os.environ.get("RS_BENCH_PMC", "1") == "0":
        return None, "skipped (RS_BENCH_PMC=0)"
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None, "bench.py itself runs under a profiler"
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    out = tempfile.mkdtemp(prefix="rs_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp", EPOCHS="4")
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        cmd = [prof, "--pmc", c, "--kernel-trace", "--output-format", "csv", "-d", os.path.join(out, c), "-o", "run",
               "--", sys.executable, os.path.join(REPO, "scripts", "experiments", "tile_epochs.py")]
        # own process group: a pass that hangs is killed with everything it started (the profiled workload)
        proc = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                start_new_session=True)
        try:
            rc = proc.wait(timeout=150)
        except subprocess.TimeoutExpired:
            import signal
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait()
            return None, f"rocprofv3 --pmc {c} timed out"
        print(f"bench: PMC pass {c} rc={rc}", file=sys.stderr, flush=True)
        if rc != 0:
            return None, f"rocprofv3 --pmc {c} exited {rc}"
    try:
        res = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "pmc_summary.py"), out,
                              "svd_epoch_tile_kernel"], capture_output=True, text=True, timeout=60)
        b = json.loads(res.stdout.strip().splitlines()[-1]).get("hbm_bytes_per_launch")
    except Exception as e:  # noqa: BLE001 -- any parse failure falls back to the committed figure
        return None, f"PMC summary failed: {e}"
    return (b, None) if b else (None, "no PMC rows for svd_epoch_tile_kernel")


def spawn_ranks(n, argv, need_gpus=True):
    """`--gpus n` without a launcher: n rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*),
    started from this parent, which touches no GPU (device_count does not initialise HIP here)."""
    import socket
    import subprocess
    if need_gpus:
        import torch
        visible = torch.cuda.device_count()
        if visible < n:
            sys.exit(f"bench.py --gpus {n}: only {visible} GPU(s) visible")
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rcs = [p.wait() for p in procs]
    sys.exit(next((c for c in rcs if c != 0), 0))


def launch_check(gpus):
    """Every rank joins a gloo group and all-reduces its rank; rank 0 prints what the group saw."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank), 1.0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"gpus": gpus, "world": world, "rank_sum": int(t[0]), "ranks": int(t[1]),
                          "local_rank0": int(os.environ.get("LOCAL_RANK", "0"))}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-strong", action="store_true", help="skip the configs[4] strong-scaling field")
    ap.add_argument("--no-ordered", action="store_true", help="skip the ORDERED-mode field")
    ap.add_argument("--launch-check", action="store_true",
                    help="CPU check of the N-rank launch: gloo ranks report themselves, no GPU work")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args.gpus, sys.argv[1:], need_gpus=not args.launch_check)
    if args.launch_check:
        launch_check(args.gpus)
        return

    import torch
    import rsgpu
    from rsgpu import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py --gpus {args.gpus} launched with WORLD_SIZE={world}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = local if world > 1 else 0
    torch.cuda.set_device(dev)

    # Weak scaling: each rank owns an ML-1M-sized item shard; users are shared (replicated).
    u, i, r, n_users, n_items = synth.ml1m_like(seed=20250824 + rank)
    nnz = len(r)
    ctx = rsgpu.Context(dev)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, n_users, n_items), K)
    rng = np.random.default_rng(1)
    P0 = rng.normal(0, 0.1, (n_users, K))  # identical on every rank (replicated user factors)
    Q0 = np.random.default_rng(100 + rank).normal(0, 0.1, (n_items, K))
    # GlobalBias warm start of the FAST schedule (rs_svd_fit does the same, common.hpp)
    plan.upload(P0, Q0, np.zeros(n_users), np.zeros(n_items), float(np.mean(r)))
    stream = torch.cuda.current_stream(dev).cuda_stream

    if world > 1:  # the library's own RCCL communicator (csrc/multi.hip), id sent over torch.distributed
        uid = [rsgpu.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        plan.set_exchange(rsgpu.EXCHANGE_AVERAGE)  # north_star's once-per-epoch all-reduce (module docstring)
        plan.join(uid[0], rank, world, n_blocks=1)
        comm_rank, comm_ranks, comm_exchange, comm_blocks = plan.shard_info()
        run = lambda n: plan.epochs_sharded(n, LR, REG, stream)
    else:
        comm_ranks, comm_blocks, comm_exchange = 1, 1, None
        run = lambda n: plan.epochs(n, LR, REG, stream)
    rccl_version, rccl_path = rsgpu.comm_info()

    for _ in range(args.warmup):
        run(1)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    P, Q, bu, bi, gb = plan.download()
    finite = bool(np.isfinite(P).all() and np.isfinite(Q).all() and np.isfinite(gb))
    # kernel-only timing of the SGD kernel (HIP events on the launch stream), separate pass: plain
    # single-GPU epochs of this rank's shard (the dominant kernel; no exchange)
    plan.set_timing(True)
    plan.epochs(5, LR, REG, stream)
    kms, nl = plan.last_kernel_ms()
    plan.set_timing(False)
    avg_kernel_s = kms / 1e3 / nl
    plan.close()
    strong = None if args.no_strong else strong_scaling(ctx, rank, world, dist, dev, stream)

    if rank == 0:
        total_updates = nnz * world * args.steps
        ab = algorithmic_bytes(nnz, n_users, K)
        achieved = ab / avg_kernel_s / 1e9
        traffic, traffic_src = None, None
        if world == 1:
            traffic, why = measure_traffic()
            if traffic:
                traffic_src = ("measured in this run: FETCH_SIZE x 2 + WRITE_SIZE per launch of the SGD kernel, two "
                               "rocprofv3 --pmc child passes over the same ML-1M workload (scripts/pmc_summary.py)")
            else:
                traffic = load_traffic()
                traffic_src = (f"committed PMC figure ({why}): FETCH_SIZE x 2 + WRITE_SIZE per launch from separate "
                               "rocprofv3 --pmc passes over the same workload (scripts/pmc_sgd.sh -> "
                               "profiles/sgd_traffic.json)")
        line = {
            "metric": METRIC,
            "value": total_updates / dt,
            "unit": "updates/s",
            "n_gpus": world,
            "nranks": comm_ranks,  # as the library's RCCL communicator reports it (1: no communicator)
            "rccl": {"version": rccl_version, "path": rccl_path},
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32/fx24",  # fp32 arithmetic; P (LDS) and Q (HBM) stored as int32 round(v * 2^24)
            "storage": "P rows int32 fixed point 2^-24 in LDS during the epoch; Q int32 fixed point 2^-24 "
                       "in HBM during a call (fp32 outside); the deltas are integer LDS / memory-side atomics",
            "data": "synthetic ML-1M-shaped ratings (rsgpu/synth.py: 6040 users x 3706 items, "
                    "1,000,209 ratings per rank, seed 20250824+rank); random-init factors N(0,0.1); "
                    "strong_scaling: rs_synth generator (csrc/synth.cpp)",
            "config": {"workload": "SVD nFactors=100 fast-mode SGD, 1 epoch over ML-1M-shaped set "
                                   "per step (BASELINE configs[1])",
                       "n_users": n_users, "n_items_per_rank": n_items, "nnz_per_rank": nnz,
                       "n_factors": K, "lr": LR, "reg": REG,
                       "parallelism": (f"item-sharded x{world}: {EXCHANGE_NAMES.get(comm_exchange, comm_exchange)}, "
                                       f"{comm_blocks} user blocks ({EXCHANGE_WIRE.get(comm_exchange, '?')})")
                                      if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "svd_epoch_tile_kernel<E=2,NW=16,RQ=2,CH=4> (tile schedule: user tiles in "
                                   "LDS, integer LDS atomics, one memory-side atomic per (item, tile) run, waves "
                                   "claim 4 runs at a time from the tile's run queue)",
                         "avg_kernel_us": avg_kernel_s * 1e6,
                         "timed_span": "HIP events around each epoch's SGD kernel on the launch stream "
                                       "(the per-epoch epilogue and the per-call Q fixed-point conversions "
                                       "are outside it but inside `value`; rocprofv3 lists them, profiles/)",
                         "algorithmic_bytes_per_launch": ab},
            "finite": finite,
        }
        if strong is not None:
            line["strong_scaling"] = strong
        if world == 1 and not args.no_ordered:
            line["ordered"] = ordered_throughput(ctx, u, i, r, n_users, n_items)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(u, i, r, n_users, n_items, args.cpu_budget)
        print(json.dumps(line), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
