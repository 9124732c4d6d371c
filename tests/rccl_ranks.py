"""Several RCCL ranks on ONE GPU: the multi-GPU exchanges of csrc/multi.hip with real collectives between
processes, on the one-GPU box (test infrastructure; tests/test_rccl_ranks_gpu.py drives it).

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected": same host hash and bus id).  Each
rank process therefore gets its own NCCL_HOSTID, so RCCL sees N hosts with one GPU each and connects them with
its network transport (sockets over the loopback interface).  The collectives -- ncclAllReduce of the QDELTA
item moves (int32 or fp16 sums) and of the GlobalBias partials, ncclSend / ncclRecv of ROTATE / ROTATE_Q's
rank-blocks, the P-range and rank-block broadcasts, the join's count all-reduce -- then run as RCCL kernels on
the device and move their bytes through RCCL's proxy: everything but xGMI itself.

Each rank process runs `python tests/rccl_ranks.py CASE RANK N ID_FILE OUT`: rank 0 writes the communicator id
(rs_comm_unique_id), every rank builds its shard plan, rs_svd_plan_join + rs_svd_plan_epochs_sharded, and saves
its downloaded model.  `group(case, n)` runs the same shards through the in-process exchange
(rs_svd_group on plans of one device) for comparison.  Reference loop: core/svd.go:92-130.
"""
from __future__ import annotations

import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "recommend-sys_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import rsgpu  # noqa: E402

K, EPOCHS, N_RATINGS = 24, 2, 30000
# case -> (exchange, QDELTA wire bits, blocks (0: the library's), seed)
CASES = {
    "qdelta32": (rsgpu.EXCHANGE_QDELTA, 32, 4, 90),
    "qdelta16": (rsgpu.EXCHANGE_QDELTA, 16, 4, 91),
    "rotate_q": (rsgpu.EXCHANGE_ROTATE_Q, 32, 0, 92),
    "rotate": (rsgpu.EXCHANGE_ROTATE, 32, 0, 93),
    "average": (rsgpu.EXCHANGE_AVERAGE, 32, 2, 94),
    "qdelta_diverge": (rsgpu.EXCHANGE_QDELTA, 16, 4, 95),  # rank 1 perturbs its replica: every rank must fail
}


def data(case):
    """ML-100K fold 3's first 30k ratings (tests/golden/ml100k.npz: the reference's u.data), start factors."""
    from helpers import folds
    d = np.load(os.path.join(REPO, "tests", "golden", "ml100k.npz"))
    f = folds(d["users"].astype(np.int64), d["items"].astype(np.int64), d["ratings"].astype(np.float64))[2]
    u, i, r, nu, ni = f.iu[:N_RATINGS], f.ii[:N_RATINGS], f.r[:N_RATINGS], f.nu, f.ni
    rng = np.random.default_rng(CASES[case][3])
    return u, i, r, nu, ni, rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))


def _bounds(keys, n, parts):
    cum = np.concatenate([[0], np.cumsum(np.bincount(keys, minlength=n))])
    return np.array([np.searchsorted(cum, cum[-1] * b // parts, side="left") for b in range(parts)] + [n])


def shard(case, s, n):
    """Shard s of n: user ranges of near-equal ratings (QDELTA, ROTATE_Q; global ids, all items) or item
    ranges (ROTATE, AVERAGE: shard-local item ids).  Returns (ratings, start rows of P / Q / b_i, item offset)."""
    u, i, r, nu, ni, P0, Q0 = data(case)
    mode = CASES[case][0]
    if mode in (rsgpu.EXCHANGE_QDELTA, rsgpu.EXCHANGE_ROTATE_Q):
        b = _bounds(u, nu, n)
        m = (u >= b[s]) & (u < b[s + 1])
        return rsgpu.Ratings(u[m], i[m], r[m], nu, ni), P0, Q0, 0
    b = rsgpu.item_shards(i, ni, n)
    m = (i >= b[s]) & (i < b[s + 1])
    return rsgpu.Ratings(u[m], i[m] - b[s], r[m], nu, int(b[s + 1] - b[s])), P0, Q0[b[s]:b[s + 1]], int(b[s])


def plan(ctx, case, s, n):
    mode, wire, _, _ = CASES[case]
    rt, P0, Q0, _ = shard(case, s, n)
    pl = ctx.svd_plan(rt, K)
    pl.set_tiles(workgroups=1, waves=1)  # one wave per shard: deterministic, so the runs compare bit for bit
    pl.set_exchange(mode)
    if mode == rsgpu.EXCHANGE_QDELTA:
        pl.set_qdelta_wire(wire)
    pl.upload(P0, Q0, np.zeros(rt.n_users), np.zeros(rt.n_items), 3.5)
    return pl


def group(ctx, case, n):
    """The same shards through the in-process exchange: every shard's download."""
    plans = [plan(ctx, case, s, n) for s in range(n)]
    g = rsgpu.SvdGroup(plans, n_blocks=CASES[case][2])
    g.epochs(EPOCHS)
    g.close()
    out = [pl.download() for pl in plans]
    for pl in plans:
        pl.close()
    return out


def rank_env(rank):
    env = dict(os.environ)
    env.update(NCCL_HOSTID=f"rsgpu-rank-{rank}",  # one "host" per rank: no duplicate-GPU refusal, net transport
               NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", NCCL_DEBUG=env.get("NCCL_DEBUG", "WARN"))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def launch(case, n, workdir, timeout=120, log_dir=None):
    """Starts n rank processes of `case` on device 0 and waits for them; returns every rank's download.
    Raises on a non-zero exit or a timeout (the rank processes are killed).  Each rank's output (progress lines,
    RCCL's warnings) goes to log_dir/<case>_<n>_r<rank>.log (default: gpurun_out/rccl_ranks under the repo)."""
    log_dir = log_dir or os.path.join(REPO, "gpurun_out", "rccl_ranks")
    os.makedirs(log_dir, exist_ok=True)
    id_file = os.path.join(workdir, f"{case}_{n}.id")
    if os.path.exists(id_file):
        os.remove(id_file)
    procs, outs, logs = [], [], []
    for r in range(n):
        out = os.path.join(workdir, f"{case}_{n}_r{r}.npz")
        outs.append(out)
        logs.append(os.path.join(log_dir, f"{case}_{n}_r{r}.log"))
        with open(logs[-1], "w") as lf:
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), case, str(r), str(n), id_file, out],
                                          env=rank_env(r), stdout=lf, stderr=subprocess.STDOUT))
    deadline = time.time() + timeout

    def tails():
        return "\n".join(f"--- rank {r} ({p}):\n" + open(p, errors="replace").read()[-3000:] for r, p in enumerate(logs))

    for p in procs:
        try:
            p.wait(timeout=max(1.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            for q in procs:
                q.wait()
            raise RuntimeError(f"{case} x{n}: rank processes timed out after {timeout} s\n" + tails())
    bad = [(r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0]
    if bad:
        raise RuntimeError(f"{case} x{n}: ranks failed {bad}\n" + tails())
    res = []
    for o in outs:
        z = np.load(o)
        res.append(int(z["code"]) if "code" in z else (z["P"], z["Q"], z["bu"], z["bi"], float(z["gb"])))
    return res, tails()


def main(case, rank, n, id_file, out):
    t0 = time.time()

    def say(m):
        print(f"[{time.time() - t0:7.2f} s] rank {rank}/{n} {case}: {m}", flush=True)

    ctx = rsgpu.Context(0)
    pl = plan(ctx, case, rank, n)  # the plan first: rank 0's id must not wait for the other ranks' plans
    say("plan built")
    if rank == 0:
        cid = rsgpu.comm_unique_id()
        with open(id_file + ".tmp", "wb") as f:
            f.write(cid)
        os.replace(id_file + ".tmp", id_file)
        say("communicator id written")
    else:
        t0 = time.time()
        while not os.path.exists(id_file):
            if time.time() - t0 > 120:
                raise SystemExit("no communicator id from rank 0")
            time.sleep(0.05)
        with open(id_file, "rb") as f:
            cid = f.read()
    say("joining")
    pl.join(cid, rank, n, CASES[case][2])
    say("joined")
    info = pl.shard_info()
    assert info[:3] == (rank, n, CASES[case][0]), info
    if case.endswith("_diverge"):  # the consistency check must fail on every rank, not only the perturbed one
        if rank == 1:
            pl.inject_fault(rsgpu.FAULT_DIVERGE)
        try:
            pl.epochs_sharded(EPOCHS)
            code, msg = 0, ""
        except rsgpu.RsError as e:
            code, msg = e.code, str(e)
        pl.leave()
        pl.close()
        ctx.close()
        np.savez(out, code=code)
        print(f"rank {rank}/{n} {case}: call returned {code} {msg}", flush=True)
        return
    pl.epochs_sharded(EPOCHS)
    say("epochs done")
    pl.leave()
    P, Q, bu, bi, gb = pl.download()
    pl.close()
    ctx.close()
    np.savez(out, P=P, Q=Q, bu=bu, bi=bi, gb=gb)
    print(f"rank {rank}/{n} {case}: done, shard_info {info}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5])
