#!/usr/bin/env python3
"""BASELINE configs[4] as a sharded fit at full size on ONE MI355X: SVD nFactors=256 on the synthetic
10M users x 1M items x ~1e9 ratings set (rs_synth, seed 20250826), library defaults, 8 shards through
the in-process group (rs_svd_group on plans sharing device 0), next to the whole set fitted by one plan.

The exchange is RS_EXCHANGE_ROTATE_Q (U > I: the Q item rank-blocks rotate, the users stay; the shards
are user ranges of near-equal ratings, as rs_svd_fit_multi cuts them).  Both fits start from the same
factors (rs_svd_plan_init_normal draws rows by row id, so every shard's P / Q equal the single plan's)
and the same GlobalBias (the training mean).  0.1 % of the ratings (every 1024th of each user range's
CSR) are held out.  Reports the held-out RMSE after every epoch for both fits, the epoch times, and --
with --strata -- one extra epoch per shard with every stratum launched alone (rs_svd_plan_time_blocks):
the per-stratum kernel times an 8-GPU run's sub-epochs wait on, and the Q bytes each sub-epoch moves.

    python scripts/config4_sharded.py [--epochs 5] [--shards 8] [--strata] [--users U --items I]
(the test helper of tests/test_config4_gpu.py; scripts/config4_sharded.py is its command line)
Prints JSON lines (progress on stderr).  Reference: core/svd.go:92-130.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "recommend-sys_amd")]
import rsgpu  # noqa: E402

LR, REG = 0.005, 0.02


def log(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def generate(U, I, n, seed, threads=16, zipf=0.9):
    """n user ranges of near-equal users (rs_synth rows [lo, hi)), each with every 1024th rating held out."""
    parts = []
    for p in range(n):
        lo, hi = U * p // n, U * (p + 1) // n
        s = rsgpu.Synth(U, I, mean_deg=100.0, sigma=1.0, min_deg=1, max_deg=I // 2, zipf_s=zipf, seed=seed,
                        user_lo=lo, user_hi=hi, n_threads=threads)
        deg = np.diff(s.rowptr)
        hold = np.zeros(s.nnz, bool)
        hold[::1024] = True
        rows = np.repeat(np.arange(hi - lo, dtype=np.int32), deg)
        hu, hi_, hr = rows[hold] + lo, s.cols[hold].copy(), s.vals[hold].astype(np.float64)
        keep = ~hold
        rp = np.zeros(hi - lo + 1, np.int64)
        np.cumsum(np.bincount(rows[keep], minlength=hi - lo), out=rp[1:])
        parts.append(dict(lo=lo, hi=hi, rowptr=rp, cols=s.cols[keep].copy(), vals=s.vals[keep].copy(),
                          hu=hu, hi_=hi_, hr=hr))
        s.close()
        log(f"range {p}: users [{lo}, {hi}) {int(rp[-1])} training ratings")
    return parts


def padded_rowptr(part, U):
    """A user range's CSR as rows 0..U-1 (empty rows outside the range)."""
    rp = np.zeros(U + 1, np.int64)
    rp[part["lo"] + 1:part["hi"] + 1] = part["rowptr"][1:]
    rp[part["hi"] + 1:] = part["rowptr"][-1]
    return rp


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--seed", type=int, default=20250826)
    ap.add_argument("--zipf", type=float, default=0.9, help="item popularity exponent (0: uniform items)")
    ap.add_argument("--strata", action="store_true", help="time every stratum alone (one extra epoch per shard)")
    ap.add_argument("--no-whole", action="store_true", help="skip the single-plan fit")
    ap.add_argument("--wg", type=int, default=0, help="workgroups per shard launch (0: one per CU)")
    ap.add_argument("--blocks", type=int, default=0, help="item blocks in all (0: automatic)")
    ap.add_argument("--hot-share", type=float, default=None, help="rs_svd_plan_set_hot_split share (default: library)")
    ap.add_argument("--hot-min", type=int, default=None, help="rs_svd_plan_set_hot_split min stratum ratings")
    ap.add_argument("--hot-merge", type=int, default=None, help="0 scaled (default), 1 average, 2 sum")
    ap.add_argument("--exchange", choices=["rotq", "qdelta"], default="rotq",
                    help="RS_EXCHANGE_ROTATE_Q (Q item blocks rotate) or RS_EXCHANGE_QDELTA (one all-reduce of item moves)")
    ap.add_argument("--wire", type=int, default=16, choices=[16, 32], help="QDELTA moves on the wire: fp16 or int32")
    ap.add_argument("--hot", type=float, default=None, help="QDELTA hot threshold, ratings per rank and block")
    ap.add_argument("--cold-every", type=int, default=None, help="QDELTA most blocks between a cold item's merges")
    ap.add_argument("--curv", type=float, default=None, help="QDELTA factor merge-weight curvature (library default 0.25)")
    ap.add_argument("--cold", type=float, default=None, help="rs_svd_plan_set_cold_store threshold (runs in flight) "
                                                             "for the shard plans (default: library)")
    ap.add_argument("--whole-cold", type=float, default=None, help="the same for the whole-set plan")
    ap.add_argument("--variants", default=None,
                    help="JSON list of option dicts (blocks, wire, hot, cold_every, curv, epochs): several sharded "
                         "fits of the one generated set, each after the whole-set fit")
    return ap.parse_args(argv)


def run(args, say=log):
    """The whole-set fit and the sharded fit of the same set; returns the summary dict (tests/ call this)."""
    U, I, k, n = args.users, args.items, args.k, args.shards
    global log
    log = say
    ctx = rsgpu.Context(0)
    t0 = time.perf_counter()
    parts = generate(U, I, n, args.seed, zipf=args.zipf)
    t_gen = time.perf_counter() - t0
    hu = np.concatenate([p["hu"] for p in parts])
    hi_ = np.concatenate([p["hi_"] for p in parts])
    hr = np.concatenate([p["hr"] for p in parts])
    nnz = int(sum(int(p["rowptr"][-1]) for p in parts))
    gb0 = float(sum(float(np.sum(p["vals"], dtype=np.float64)) for p in parts) / nnz)
    log(f"generated {nnz} training + {len(hr)} held-out ratings in {t_gen:.1f} s, mean {gb0:.4f}")
    out = {"config": "BASELINE configs[4]: SVD nFactors=256, synthetic 10M x 1M x ~1e9 (rs_synth seed "
                     f"{args.seed}), library defaults", "n_users": U, "n_items": I, "nnz_train": nnz,
           "n_holdout": int(len(hr)), "epochs": args.epochs, "lr": LR, "reg": REG, "gen_s": t_gen}

    variants = json.loads(args.variants) if args.variants else [{}]
    ep_whole = max([args.epochs] + [int(v.get("epochs", 0)) for v in variants])
    whole = None
    if not args.no_whole:  # the same set as one plan: one CSR over all users
        t0 = time.perf_counter()
        rp = np.concatenate([[0]] + [p["rowptr"][1:] + sum(int(q["rowptr"][-1]) for q in parts[:x])
                                     for x, p in enumerate(parts)]).astype(np.int64)
        cols = np.concatenate([p["cols"] for p in parts])
        vals = np.concatenate([p["vals"] for p in parts])
        plan = ctx.svd_plan_csr(U, I, rp, cols, vals, k)
        del cols, vals, rp
        if args.whole_cold is not None:
            plan.set_cold_store(args.whole_cold)
        plan.init_normal(0.0, 0.1, seed=1)
        plan.upload(gb=gb0)
        t_plan = time.perf_counter() - t0
        r0 = plan.evaluate(hu, hi_, hr)[0]
        curve, ep_s = [], []
        for e in range(ep_whole):
            t = time.perf_counter()
            plan.epochs(1, LR, REG)
            ctx.check(rsgpu.lib().rs_synchronize(ctx.h))
            ep_s.append(time.perf_counter() - t)
            curve.append(plan.evaluate(hu, hi_, hr)[0])
            log(f"whole set epoch {e + 1}: {ep_s[-1]:.3f} s, held-out RMSE {curve[-1]:.4f}")
        plan.close()
        whole = {"plan_build_s": t_plan, "rmse_init": r0, "rmse_per_epoch": curve, "epoch_s": ep_s}
        out["whole"] = whole
        print(json.dumps({"whole": whole}), flush=True)

    out["variants"] = []
    for vi, var in enumerate(variants):
        a = argparse.Namespace(**{**vars(args), **var})
        log(f"variant {vi}: {var}")
        sh = sharded(a, ctx, parts, hu, hi_, hr, gb0, whole)
        sh["variant"] = var
        out["variants"].append(sh)
        out["sharded"] = sh
    ctx.close()
    return out


def sharded(args, ctx, parts, hu, hi_, hr, gb0, whole):
    """The sharded fit of the generated set (one variant of the options)."""
    U, I, k, n = args.users, args.items, args.k, args.shards
    # the sharded fit: n plans over user ranges (global ids, all items), Q item blocks rotate
    t0 = time.perf_counter()
    plans = []
    for p in parts:
        pl = ctx.svd_plan_csr(U, I, padded_rowptr(p, U), p["cols"], p["vals"], k)
        pl.set_exchange(rsgpu.EXCHANGE_QDELTA if args.exchange == "qdelta" else rsgpu.EXCHANGE_ROTATE_Q)
        if args.exchange == "qdelta":
            pl.set_qdelta_wire(args.wire)
            if args.hot is not None or args.cold_every is not None:
                pl.set_qdelta_split(4.0 if args.hot is None else args.hot, 2 if args.cold_every is None else args.cold_every)
            if args.curv is not None:
                pl.set_qdelta_curvature(args.curv)
        if args.cold is not None:
            pl.set_cold_store(args.cold)
        if args.wg:
            pl.set_tiles(workgroups=args.wg)
        if args.hot_share is not None or args.hot_min is not None or args.hot_merge is not None:
            pl.set_hot_split(0.02 if args.hot_share is None else args.hot_share,
                             (1 << 17) if args.hot_min is None else args.hot_min, args.hot_merge or 0)
        pl.init_normal(0.0, 0.1, seed=1)
        pl.upload(gb=gb0)
        plans.append(pl)
    g = rsgpu.SvdGroup(plans, n_blocks=args.blocks)
    t_join = time.perf_counter() - t0
    _, _, exch, nblk = plans[0].shard_info()
    qinfo = plans[0].qdelta_info() if args.exchange == "qdelta" else None
    log(f"{n} shard plans + group in {t_join:.1f} s: exchange {exch}, {nblk} blocks"
        + (f", {qinfo[0]} hot items, a full merge every {qinfo[1]} blocks" if qinfo else ""))
    r0 = plans[0].evaluate(hu, hi_, hr)[0]
    curve, ep_s = [], []
    for e in range(args.epochs):
        t = time.perf_counter()
        try:
            g.epochs(1, LR, REG)
        except rsgpu.RsError as x:  # (diagnostic: where the shards' replicas differ)
            log(f"sharded epoch {e + 1}: {x}")
            Qs = [pl.download()[1] for pl in plans]
            cnt = np.bincount(np.concatenate([p_["cols"] for p_ in parts]), minlength=I)
            for sidx in range(1, len(Qs)):
                d = np.abs(Qs[sidx] - Qs[0]).max(1)
                bad = np.nonzero(d > 0)[0]
                log(f"shard {sidx} vs 0: {len(bad)} item rows differ, max {d.max():.3g}; first "
                    + ", ".join(f"{int(b)}(deg {int(cnt[b])}, {d[b]:.3g})" for b in bad[:8]))
            raise
        ep_s.append(time.perf_counter() - t)
        curve.append(plans[0].evaluate(hu, hi_, hr)[0])
        log(f"sharded epoch {e + 1}: {ep_s[-1]:.3f} s, held-out RMSE {curve[-1]:.4f}")
    sh = {"n_shards": n, "exchange": f"RS_EXCHANGE_QDELTA (wire {args.wire} bits)" if args.exchange == "qdelta"
          else "RS_EXCHANGE_ROTATE_Q",
          "item_blocks": nblk, "setup_s": t_join, "qdelta_hot_items": qinfo[0] if qinfo else None,
          "qdelta_cold_every": qinfo[1] if qinfo else None,
          "rmse_init": r0, "rmse_per_epoch": curve, "epoch_s_one_gpu": ep_s}
    if whole:
        wc = whole["rmse_per_epoch"]
        sh["rmse_diff_vs_whole"] = curve[-1] - wc[len(curve) - 1] if len(wc) >= len(curve) else None
        sh["rmse_diff_per_epoch"] = [a - b for a, b in zip(curve, wc)]
    g.close()
    if args.strata and args.exchange == "qdelta":  # one epoch of each shard alone: what an 8-GPU epoch waits on
        t = np.array([pl.time_blocks(nblk, LR, REG) for pl in plans]).sum(1)  # the shard's user blocks, summed
        sh["shard_epoch_ms"] = t.tolist()
        sh["shard_epoch_max_ms"] = float(t.max())
        sh["imbalance_max_over_mean"] = float(t.max() / t.mean())
        sh["allreduce_bytes_per_merge"] = int(I * ((k + 1 + 3) // 4 * 4) * args.wire // 8)
        sh["merges_per_epoch"] = nblk
        log(f"shard epochs {t.min():.1f}-{t.max():.1f} ms (max/mean {sh['imbalance_max_over_mean']:.3f}); "
            f"{nblk} all-reduces of {sh['allreduce_bytes_per_merge'] / 1e9:.2f} GB per epoch")
    elif args.strata:  # per-stratum kernel times: shard g trains item rank-block (g + s) mod n in sub-epoch s
        pieces = nblk // n
        t = np.array([pl.time_blocks(nblk, LR, REG) for pl in plans])  # [shard, item block] ms
        rb = t.reshape(n, n, pieces).sum(2)  # [shard, item rank-block]
        sub = np.array([[rb[gg, (gg + s) % n] for gg in range(n)] for s in range(n)])  # [sub-epoch, shard]
        ld = plans[0].ld
        sh["stratum_ms"] = t.tolist()
        sh["sub_epoch_ms_per_shard"] = sub.tolist()
        sh["sub_epoch_max_ms"] = sub.max(1).tolist()
        sh["sub_epoch_mean_ms"] = sub.mean(1).tolist()
        sh["imbalance_max_over_mean"] = float((sub.max(1) / sub.mean(1)).mean())
        sh["q_bytes_per_sub_epoch"] = int(I / n * ld * 4)
        sh["p_bytes_per_sub_epoch_if_p_rotated"] = int(U / n * ld * 4)
        log(f"sub-epoch max/mean stratum time {sh['imbalance_max_over_mean']:.3f}; "
            f"epoch on {n} GPUs ~ {sum(sh['sub_epoch_max_ms']):.1f} ms of SGD")
    # finite: the download's fixed-point / non-finite check of Q (RS_ERR_NUMERIC) and the RMSE of every shard
    # (P of 10M x 256 doubles is not brought to the host)
    finite = all(np.isfinite(x) for x in curve)
    for pl in plans:
        try:
            e = pl.evaluate(hu[:1000], hi_[:1000], hr[:1000])[0]
            finite = finite and bool(np.isfinite(e))
        except rsgpu.RsError:
            finite = False
        pl.close()
    sh["finite"] = finite
    print(json.dumps({"sharded": sh}), flush=True)
    return sh


if __name__ == "__main__":
    print(json.dumps(run(parse())), flush=True)
