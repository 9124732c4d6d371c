"""Multi-GPU schedules on CPU: world_size-2/3 gloo tests with a host model of the plan (a shard's epoch is
the oracle's restatement of the kernel's schedule), checked against a single-process computation of the
same rule -- the ROTATE exchange (the library's default, its schedule from rs_rotation_step), the
AVERAGE delta protocol, the user-sharded dual partition and the KNN part split."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from rsgpu import multi

K, EPOCHS = 8, 3


class HostPlan:
    """CPU stand-in for SvdPlan's delta interface (the GPU test covers the kernels themselves)."""

    def __init__(self, users, items, r, n_users, n_items, P0, Q0, gb0):
        self.k = P0.shape[1]
        self.n_users, self.ld = n_users, self.k + 1
        self.rowptr, self.items, self.r = O.csr_by(users, n_users, items, r)
        self.P, self.Q = P0.copy(), Q0.copy()
        self.bu, self.bi, self.gb = np.zeros(n_users), np.zeros(n_items), gb0
        self.w = None

    def set_user_weights(self, w):
        self.w = np.asarray(w, np.float64)

    def epoch_delta_t(self, dP, gbsum, lr, reg, stream=None):
        P, Q, bu, bi, g = O.svd_fit_chunked(self.rowptr, self.items, self.r, self.P, self.Q, 1 << 30,
                                            bu=self.bu, bi=self.bi, gb=self.gb, epochs=1, lr=lr,
                                            reg=reg, warm=False)
        self.Q, self.bi = Q, bi
        d = np.zeros((self.n_users, self.ld))
        d[:, :self.k] = self.w[:, None] * (P - self.P)
        d[:, self.k] = self.w * (bu - self.bu)
        dP.copy_(torch.from_numpy(d.astype(np.float32)))
        deg = np.diff(self.rowptr).astype(np.float64)
        nnz = deg.sum()
        gbsum.copy_(torch.tensor([(g - self.gb) * nnz]))  # fold of the local chains (one fold)

    def apply_delta_t(self, dP, gbsum, inv_total, stream=None):
        d = dP.numpy().astype(np.float64)
        self.P = self.P + d[:, :self.k]
        self.bu = self.bu + d[:, self.k]
        self.gb = self.gb + float(gbsum.item()) * inv_total


def make_data(seed=0, n_users=40, n_items=60, nnz=700):
    rng = np.random.default_rng(seed)
    pairs = rng.choice(n_users * n_items, nnz, replace=False)
    u, i = (pairs // n_items).astype(np.int32), (pairs % n_items).astype(np.int32)
    return u, i, rng.integers(1, 6, nnz).astype(float), n_users, n_items


def reference_merge(u, i, r, nu, ni, P0, Q0, n_shards, epochs=EPOCHS):
    """Single process: every shard's epoch from the same start, count-weighted user-delta merge."""
    sh = multi.item_shard_of(ni, n_shards)
    plans = [HostPlan(*multi.take_shard(u, i, r, sh, s), nu, ni, P0, Q0, 3.0) for s in range(n_shards)]
    cnt = np.stack([np.bincount(multi.take_shard(u, i, r, sh, s)[0], minlength=nu) for s in range(n_shards)])
    tot = cnt.sum(0)
    for s, p in enumerate(plans):
        p.set_user_weights(np.divide(cnt[s], tot, out=np.zeros(nu), where=tot > 0))
    for _ in range(epochs):
        ds, gs = [], []
        for p in plans:
            dP, g = torch.zeros((nu, p.ld)), torch.zeros(1, dtype=torch.float64)
            p.epoch_delta_t(dP, g, 0.005, 0.02)
            ds.append(dP)
            gs.append(g)
        dsum, gsum = sum(ds), sum(gs)
        for p in plans:
            p.apply_delta_t(dsum, gsum, 1.0 / len(r))
    return plans


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    u, i, r, nu, ni = make_data()
    rng = np.random.default_rng(1)
    P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    sh = multi.item_shard_of(ni, world)
    lu, li, lr_ = multi.take_shard(u, i, r, sh, rank)
    plan = HostPlan(lu, li, lr_, nu, ni, P0, Q0, 3.0)
    w, total = multi.user_weights(lu, nu, dist)
    assert total == len(r)
    step = multi.ItemShardedStep(plan, dist, w, total)
    step.run(EPOCHS)
    out[rank] = (plan.P, plan.Q, plan.bu, plan.bi, plan.gb)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_item_shards_partition_items():
    sh = multi.item_shard_of(1000, 4)
    assert set(np.unique(sh)) == {0, 1, 2, 3}
    assert max(np.bincount(sh)) - min(np.bincount(sh)) <= 1


def test_two_rank_gloo_matches_single_process_merge():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    u, i, r, nu, ni = make_data()
    rng = np.random.default_rng(1)
    P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    plans = reference_merge(u, i, r, nu, ni, P0, Q0, 2)
    for rank in (0, 1):
        P, Q, bu, bi, gb = res[rank]
        # replicated state identical on both ranks and equal to the single-process merge
        np.testing.assert_allclose(P, plans[rank].P, atol=1e-6)
        np.testing.assert_allclose(bu, plans[rank].bu, atol=1e-6)
        assert abs(gb - plans[rank].gb) < 1e-9
        np.testing.assert_array_equal(res[0][0], res[1][0])
        # each rank's item shard equals the shard trained in the single-process run
        mine = multi.item_shard_of(ni, 2) == rank
        np.testing.assert_allclose(Q[mine], plans[rank].Q[mine], atol=1e-6)


# ---- ROTATE (the library's default exchange): strata rotation with P rank-blocks sent around ------
# Host model of rs_svd_plan_epochs_sharded's ROTATE path (csrc/multi.hip) on world_size 2 and 3 over
# gloo: the schedule is the library's own (rs_rotation_step, host-only C-ABI); a stratum's epoch is the
# oracle's per-rating SGD (svd.go:93-129) with one work-local GlobalBias; P rank-blocks go to rank g-1
# by send/recv, GlobalBias partials are all-reduced once per epoch, the rank-blocks broadcast at the end.

def _rot_blocks(u, nu, n):
    """Rank-blocks of near-equal ratings over all users (the library's user_block_bounds rule)."""
    cum = np.concatenate([[0], np.cumsum(np.bincount(u, minlength=nu))])
    return np.array([np.searchsorted(cum, cum[-1] * b // n, side="left") for b in range(n)] + [nu])


def _stratum(u, i, r, ub, lo, hi, b):
    """Ratings of users in rank-block b and items in [lo, hi), user-CSR order (data order per user)."""
    m = (u >= ub[b]) & (u < ub[b + 1]) & (i >= lo) & (i < hi)
    order = np.argsort(u[m], kind="stable")
    return u[m][order], i[m][order], r[m][order]


def _train_stratum(P, Q, bu, bi, gb, su, si, sr):
    """One stratum: the sequential SGD with a work-local GlobalBias; returns its fold partial."""
    if len(sr) == 0:
        return P, Q, bu, bi, 0.0
    P, Q, bu, bi, g = O.svd_fit_works(su, si, sr, np.array([0, len(sr)], np.int64), P, Q, bu, bi, gb, epochs=1)
    return P, Q, bu, bi, len(sr) * (g - gb)


def _rot_worker(rank, world, port, out):
    import rsgpu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    u, i, r, nu, ni = make_data(seed=5)
    rng = np.random.default_rng(4)
    P, Q = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    bu, bi, gb = np.zeros(nu), np.zeros(ni), 3.0
    lo, hi = ni * rank // world, ni * (rank + 1) // world  # this rank's item shard
    ub = _rot_blocks(u, nu, world)
    for _ in range(EPOCHS):
        part = 0.0
        for st in range(world):
            train, send_to, recv, recv_from = rsgpu.rotation_step(rank, world, st)
            P, Q, bu, bi, p = _train_stratum(P, Q, bu, bi, gb, *_stratum(u, i, r, ub, lo, hi, train))
            part += p
            a, z = ub[train], ub[train + 1]
            blk = torch.from_numpy(np.concatenate([P[a:z], bu[a:z, None]], 1).copy())
            ra, rz = ub[recv], ub[recv + 1]
            inc = torch.zeros((rz - ra, K + 1), dtype=torch.float64)
            reqs = [dist.isend(blk, send_to), dist.irecv(inc, recv_from)]
            for q in reqs:
                q.wait()
            P[ra:rz], bu[ra:rz] = inc[:, :K].numpy(), inc[:, K].numpy()
        t = torch.tensor([part], dtype=torch.float64)
        dist.all_reduce(t)
        gb += float(t.item()) / len(r)
    for b in range(world):  # rank-block b is current on rank b
        blk = torch.from_numpy(np.concatenate([P[ub[b]:ub[b + 1]], bu[ub[b]:ub[b + 1], None]], 1).copy())
        dist.broadcast(blk, b)
        P[ub[b]:ub[b + 1]], bu[ub[b]:ub[b + 1]] = blk[:, :K].numpy(), blk[:, K].numpy()
    out[rank] = (P, Q[lo:hi], bu, bi[lo:hi], gb)
    dist.destroy_process_group()


def _rot_reference(world):
    """Single process: the strata in rotation order (sub-epoch, then rank), one GlobalBias fold per epoch."""
    u, i, r, nu, ni = make_data(seed=5)
    rng = np.random.default_rng(4)
    P, Q = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    bu, bi, gb = np.zeros(nu), np.zeros(ni), 3.0
    ub = _rot_blocks(u, nu, world)
    for _ in range(EPOCHS):
        part = 0.0
        for st in range(world):
            for g in range(world):
                lo, hi = ni * g // world, ni * (g + 1) // world
                P, Q, bu, bi, p = _train_stratum(P, Q, bu, bi, gb, *_stratum(u, i, r, ub, lo, hi, (g + st) % world))
                part += p
        gb += part / len(r)
    return P, Q, bu, bi, gb, ni


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_rotation_matches_single_process(world):
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rot_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    P, Q, bu, bi, gb, ni = _rot_reference(world)
    for rank in range(world):
        rP, rQ, rbu, rbi, rgb = res[rank]
        lo, hi = ni * rank // world, ni * (rank + 1) // world
        np.testing.assert_allclose(rP, P, atol=1e-12)
        np.testing.assert_allclose(rbu, bu, atol=1e-12)
        np.testing.assert_allclose(rQ, Q[lo:hi], atol=1e-12)
        np.testing.assert_allclose(rbi, bi[lo:hi], atol=1e-12)
        assert abs(rgb - gb) < 1e-12
        np.testing.assert_array_equal(res[0][0], rP)  # P replicated bit for bit after the broadcast


def test_rotation_step_covers_every_stratum_once():
    """rs_rotation_step (the library's schedule): over an epoch every (rank, rank-block) stratum is
    trained exactly once, no two ranks train one rank-block in the same sub-epoch, and the block a rank
    receives is the one it trains next (sent by the rank that just trained it)."""
    import rsgpu
    for n in (1, 2, 3, 8):
        seen = set()
        for st in range(n):
            trained = set()
            for g in range(n):
                train, send_to, recv, recv_from = rsgpu.rotation_step(g, n, st)
                assert (g, train) not in seen
                seen.add((g, train))
                trained.add(train)
                if st + 1 < n:
                    assert rsgpu.rotation_step(g, n, st + 1)[0] == recv
                assert rsgpu.rotation_step(recv_from, n, st)[0] == recv
                assert rsgpu.rotation_step(send_to, n, st)[3] == g
            assert len(trained) == n
        assert len(seen) == n * n


# ---- user-sharded (dual) partition: users split by range, item deltas all-reduced ---------------

class HostUserPlan:
    """CPU stand-in for SvdPlan's Q-delta interface over a user range (local user ids)."""

    def __init__(self, users, items, r, n_users, n_items, P0, Q0, gb0):
        self.k = P0.shape[1]
        self.n_items, self.ld = n_items, self.k + 1
        self.rowptr, self.items, self.r = O.csr_by(users, n_users, items, r)
        self.P, self.Q = P0.copy(), Q0.copy()
        self.bu, self.bi, self.gb = np.zeros(n_users), np.zeros(n_items), gb0
        self.w = None

    def set_item_weights(self, w):
        self.w = np.asarray(w, np.float64)

    def epoch_qdelta_t(self, dQ, gbsum, lr, reg, stream=None):
        P, Q, bu, bi, g = O.svd_fit_chunked(self.rowptr, self.items, self.r, self.P, self.Q, 1 << 30,
                                            bu=self.bu, bi=self.bi, gb=self.gb, epochs=1, lr=lr,
                                            reg=reg, warm=False)
        self.P, self.bu = P, bu
        d = np.zeros((self.n_items, self.ld))
        d[:, :self.k] = self.w[:, None] * (Q - self.Q)
        d[:, self.k] = self.w * (bi - self.bi)
        dQ.copy_(torch.from_numpy(d.astype(np.float32)))
        nnz = float(self.rowptr[-1])
        gbsum.copy_(torch.tensor([(g - self.gb) * nnz]))

    def apply_qdelta_t(self, dQ, gbsum, inv_total, stream=None):
        d = dQ.numpy().astype(np.float64)
        self.Q = self.Q + d[:, :self.k]
        self.bi = self.bi + d[:, self.k]
        self.gb = self.gb + float(gbsum.item()) * inv_total


def user_ranges(nu, world):
    return [(nu * p // world, nu * (p + 1) // world) for p in range(world)]


def user_shard(u, i, r, lo, hi):
    m = (u >= lo) & (u < hi)
    return (u[m] - lo).astype(np.int32), i[m], r[m]


def reference_user_merge(u, i, r, nu, ni, P0, Q0, world, epochs=EPOCHS):
    plans = []
    cnt = []
    for lo, hi in user_ranges(nu, world):
        su, si, sr = user_shard(u, i, r, lo, hi)
        plans.append(HostUserPlan(su, si, sr, hi - lo, ni, P0[lo:hi], Q0, 3.0))
        cnt.append(np.bincount(si, minlength=ni))
    tot = np.sum(cnt, 0)
    for s, p in enumerate(plans):
        p.set_item_weights(np.divide(cnt[s], tot, out=np.zeros(ni), where=tot > 0))
    for _ in range(epochs):
        ds, gs = [], []
        for p in plans:
            dQ, g = torch.zeros((ni, p.ld)), torch.zeros(1, dtype=torch.float64)
            p.epoch_qdelta_t(dQ, g, 0.005, 0.02)
            ds.append(dQ)
            gs.append(g)
        dsum, gsum = sum(ds), sum(gs)
        for p in plans:
            p.apply_qdelta_t(dsum, gsum, 1.0 / len(r))
    return plans


def _user_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    u, i, r, nu, ni = make_data(seed=3)
    rng = np.random.default_rng(2)
    P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    lo, hi = user_ranges(nu, world)[rank]
    su, si, sr = user_shard(u, i, r, lo, hi)
    plan = HostUserPlan(su, si, sr, hi - lo, ni, P0[lo:hi], Q0, 3.0)
    w, total = multi.count_weights(np.bincount(si, minlength=ni), dist)
    assert total == len(r)
    multi.UserShardedStep(plan, dist, w, total).run(EPOCHS)
    out[rank] = (plan.P, plan.Q, plan.bu, plan.bi, plan.gb)
    dist.destroy_process_group()


def test_two_rank_gloo_user_sharded_matches_single_process_merge():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_user_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    u, i, r, nu, ni = make_data(seed=3)
    rng = np.random.default_rng(2)
    P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    plans = reference_user_merge(u, i, r, nu, ni, P0, Q0, 2)
    for rank in (0, 1):
        P, Q, bu, bi, gb = res[rank]
        np.testing.assert_allclose(Q, plans[rank].Q, atol=1e-6)       # replicated item state
        np.testing.assert_allclose(bi, plans[rank].bi, atol=1e-6)
        np.testing.assert_array_equal(res[0][1], res[1][1])
        assert abs(gb - plans[rank].gb) < 1e-9 and res[0][4] == res[1][4]
        np.testing.assert_allclose(P, plans[rank].P, atol=1e-6)       # the rank's own users
        np.testing.assert_allclose(bu, plans[rank].bu, atol=1e-6)


# ---- KNN sims across ranks: disjoint parts, one shared file, no collective ----------

def test_knn_part_blocks_partition_and_balance():
    """Every 128-row block has exactly one owner and the triangle work (T - t tiles for block t) is
    spread within 10 % (ML-20M: T = 209) for 2..8 parts."""
    for L, n in ((26744, 2), (26744, 4), (26744, 8), (700, 3), (1, 2), (0, 4)):
        T = (L + 127) // 128
        own = np.stack([multi.knn_part_blocks(L, p, n) for p in range(n)]) if T else np.zeros((n, 0))
        assert (own.sum(0) == 1).all()
        if L == 26744:
            work = own @ (T - np.arange(T))
            assert work.max() <= 1.1 * work.min()


def _host_part(kind, rowptr, ids, rr):
    """CPU stand-in for ctx.knn_sims(..., part, n_parts, out): the oracle's Sims, entries of the part
    only (rows of its blocks from the diagonal rightwards, and their mirrors)."""
    full = O.knn_sims(kind, rowptr, ids, rr)
    L = len(rowptr) - 1

    def compute(part, n_parts, out):
        own = multi.knn_part_blocks(L, part, n_parts)
        for t in np.nonzero(own)[0]:
            a0, a1 = 128 * t, min(L, 128 * t + 128)
            out[a0:a1, a0:] = full[a0:a1, a0:]
            out[a0:, a0:a1] = full[a0:, a0:a1]
    return compute, full


def _knn_worker(rank, world, port, path, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rowptr, ids, rr = _knn_lists()
    compute, _ = _host_part(0, rowptr, ids, rr)
    S = multi.knn_sims_shared(compute, len(rowptr) - 1, path, rank, world, dist)
    out[rank] = np.array(S)
    dist.destroy_process_group()


def _knn_lists():
    rng = np.random.default_rng(5)
    L, Rn = 300, 400
    rows, cols = np.nonzero(rng.random((L, Rn)) < 0.05)
    return O.csr_by(rows, L, cols, rng.integers(1, 6, len(rows)).astype(float))


def test_two_rank_gloo_knn_sims_shared_file(tmp_path):
    port = _free_port()
    path = str(tmp_path / "sims.npy")
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_knn_worker, args=(2, port, path, out), nprocs=2, join=True)
        res = dict(out)
    rowptr, ids, rr = _knn_lists()
    full = O.knn_sims(0, rowptr, ids, rr)
    for rank in (0, 1):
        got = res[rank]
        assert np.array_equal(np.isnan(full), np.isnan(got))
        m = ~np.isnan(full)
        assert np.array_equal(full[m], got[m])


def test_rs_item_shards_balanced_ranges():
    """rs_item_shards (host, no GPU): contiguous item ranges covering every item, split points at the
    first item whose cumulative count reaches r/n of the ratings."""
    import rsgpu
    rng = np.random.default_rng(4)
    ni = 500
    items = rng.zipf(1.3, 40000) % ni
    for n in (1, 2, 3, 8):
        b = rsgpu.item_shards(items, ni, n)
        assert b[0] == 0 and b[-1] == ni and np.all(np.diff(b) >= 0)
        cum = np.concatenate([[0], np.cumsum(np.bincount(items, minlength=ni))])
        for r in range(1, n):
            assert b[r] == np.searchsorted(cum, len(items) * r // n, side="left")


# ---- ROTATE_Q (the exchange rs_svd_fit_multi picks at configs[4]): user ranges stay, item blocks rotate -------
# Host model of epochs_rotate(RS_EXCHANGE_ROTATE_Q) (csrc/multi.hip; rules restated in tests/rotq_model.py) on
# world_size 2 and 3 over gloo: the library's rs_rotation_step schedule, Q item blocks plus their hot copies by
# isend/irecv, the hot copies' summed moves all-reduced and merged with RS_HOT_SCALED's weights, the GlobalBias
# partials all-reduced, the item rank-blocks and P ranges broadcast at the end.  Checked against the
# single-process sequential run over the strata (rotq_model.sequential).  tests/test_multi_gpu.py checks the
# same sequential model against the library's in-process group on one GPU (1e-5).

RQ_PIECES, RQ_HOT = 2, 0.05


def _rq_data():
    rng = np.random.default_rng(11)
    nu, ni, nnz = 60, 50, 1400
    pop = 1.0 / np.arange(1, ni + 1) ** 1.1  # a Zipf head, so that hot items exist
    pairs = set()
    while len(pairs) < nnz:
        pairs.add((int(rng.integers(0, nu)), int(rng.choice(ni, p=pop / pop.sum()))))
    pairs = sorted(pairs, key=lambda _: rng.random())
    u = np.array([a for a, _ in pairs], np.int32)
    i = np.array([b for _, b in pairs], np.int32)
    return u, i, rng.integers(1, 6, nnz).astype(float), nu, ni


def _rq_setup(world):
    import rotq_model as RQ
    u, i, r, nu, ni = _rq_data()
    rng = np.random.default_rng(6)
    P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    lay = RQ.Layout(u, i, ni, world, RQ_PIECES, hot_share=RQ_HOT, min_stratum=0)
    ub = RQ.block_bounds(u, nu, world)  # the ranks' user ranges (rs_svd_fit_multi's user_block_bounds)
    return RQ, u, i, r, nu, ni, P0, Q0, lay, ub


def _rq_works(RQ, lay, u, i, r, ub):
    def works(g, b):
        m = (u >= ub[g]) & (u < ub[g + 1])
        return [RQ.stratum_csr(lay, u[m], i[m], r[m], b)]
    return works


def _rq_worker(rank, world, port, out):
    import rsgpu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    RQ, u, i, r, nu, ni, P0, Q0, lay, ub = _rq_setup(world)
    works = _rq_works(RQ, lay, u, i, r, ub)
    h, nb, H = lay.h, lay.nb, lay.H
    P, bu = P0.copy(), np.zeros(nu)
    Q = np.zeros((lay.rows(), K))
    Q[:ni] = Q0
    bi = np.zeros(lay.rows())
    lay.seed(Q, bi)
    gb = 3.0

    def block_rows(rb):  # item rows of rank-block rb, then its blocks' copy rows
        a, z = lay.ib[rb * h], lay.ib[rb * h + h]
        rows = list(range(a, z)) + [lay.copy_row(b, x) for b in range(rb * h, rb * h + h) for x in range(H)]
        return np.array(rows, np.int64)

    for _ in range(EPOCHS):
        part = 0.0
        for st in range(world):
            train, send_to, recv, recv_from = rsgpu.rotation_step(rank, world, st)
            for j in range(h):
                P, Q, bu, bi, p = RQ.train_works(P, Q, bu, bi, gb, works(rank, train * h + j))
                part += p
            out_rows, in_rows = block_rows(train), block_rows(recv)
            blk = torch.from_numpy(np.concatenate([Q[out_rows], bi[out_rows, None]], 1).copy())
            inc = torch.zeros((len(in_rows), K + 1), dtype=torch.float64)
            for q in [dist.isend(blk, send_to), dist.irecv(inc, recv_from)]:
                q.wait()
            Q[in_rows], bi[in_rows] = inc[:, :K].numpy(), inc[:, K].numpy()
        if H:  # rank g holds item rank-block g again: its copies' moves, summed over the ranks
            t = torch.from_numpy(lay.partial(Q, bi, rank * h, rank * h + h))
            dist.all_reduce(t)
            lay.write(Q, bi, t.numpy(), rank * h, rank * h + h)
        t = torch.tensor([part], dtype=torch.float64)
        dist.all_reduce(t)
        gb += float(t.item()) / len(r)
    for g in range(world):  # item rank-block g is current on rank g, P range g too
        a, z = lay.ib[g * h], lay.ib[g * h + h]
        blk = torch.from_numpy(np.concatenate([Q[a:z], bi[a:z, None]], 1).copy())
        dist.broadcast(blk, g)
        Q[a:z], bi[a:z] = blk[:, :K].numpy(), blk[:, K].numpy()
        pr = torch.from_numpy(np.concatenate([P[ub[g]:ub[g + 1]], bu[ub[g]:ub[g + 1], None]], 1).copy())
        dist.broadcast(pr, g)
        P[ub[g]:ub[g + 1]], bu[ub[g]:ub[g + 1]] = pr[:, :K].numpy(), pr[:, K].numpy()
    out[rank] = (P, Q[:ni], bu, bi[:ni], gb, H)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_rotation_q_matches_single_process(world):
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_rq_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    RQ, u, i, r, nu, ni, P0, Q0, lay, ub = _rq_setup(world)
    assert lay.H >= 2 and any(c > 1 for _, c in lay.meta)  # the hot split is exercised
    P, Q, bu, bi, gb = RQ.sequential(lay, u, i, r, nu, P0, Q0, 3.0, EPOCHS, ub, _rq_works(RQ, lay, u, i, r, ub))
    for rank in range(world):
        rP, rQ, rbu, rbi, rgb, H = res[rank]
        assert H == lay.H
        np.testing.assert_allclose(rP, P, atol=1e-12)
        np.testing.assert_allclose(rbu, bu, atol=1e-12)
        np.testing.assert_allclose(rQ, Q, atol=1e-12)
        np.testing.assert_allclose(rbi, bi, atol=1e-12)
        assert abs(rgb - gb) < 1e-12
        for x in range(4):  # replicated bit for bit after the broadcasts
            np.testing.assert_array_equal(res[0][x], res[rank][x])


def test_rotation_q_layout_rules():
    """The restated hot rules: every hot item's copies sit nb // copies blocks apart from its natural block,
    every rating of a hot item lands on a used copy, and a copy's block is a function of the user only."""
    import rotq_model as RQ
    u, i, r, nu, ni = _rq_data()
    lay = RQ.Layout(u, i, ni, 3, RQ_PIECES, hot_share=RQ_HOT, min_stratum=0)
    assert lay.H > 0
    for h, x in enumerate(lay.hot):
        nat, c = lay.meta[h]
        assert lay.ib[nat] <= x < lay.ib[nat + 1]
        assert sum(lay.copy_used(b, h) for b in range(lay.nb)) == c
        for a in np.unique(u[i == x]):
            b = lay.block_of(a, x)
            assert lay.copy_used(b, h) and b == lay.block_of(a, x)
    assert RQ.mix32(0) == (0xE220A8397B1DCDAF >> 16) & 0xFFFFFFFF  # splitmix64(0)'s published first output


# ---- QDELTA (round 5): user ranges, every item, one all-reduce of the weighted item moves per merge ---------
# Host model of epochs_qdelta (csrc/multi.hip) on world_size 2 and 3 over gloo: every rank trains its user
# range (the oracle's sequential SGD in user-CSR order, work-local GlobalBias) from the same Q, the item moves
# w_i (q_end - q_start) with w_i = kappa_i / c_i are summed by one all-reduce (with the GlobalBias partials);
# `merges` user blocks per epoch each end in a merge, pipelined: a rank keeps its own weighted moves at once and
# adds the others' (sum - own) and the GlobalBias fold after its next block, so the all-reduce overlaps that
# block; after the last merge every rank holds the same Q; the P ranges are broadcast at the end.  Checked against the single-process run of the same rule.

QD_MERGES = 2


def _qd_data():
    """A Zipf head over 200 items and 400 users (unique pairs), so that some items pass the hot threshold (4
    ratings per rank and block) and the tail stays cold."""
    rng = np.random.default_rng(12)
    nu, ni, nnz = 400, 200, 4000
    pop = 1.0 / np.arange(1, ni + 1) ** 1.1
    pairs = set()
    while len(pairs) < nnz:
        pairs.add((int(rng.integers(0, nu)), int(rng.choice(ni, p=pop / pop.sum()))))
    pairs = sorted(pairs, key=lambda _: rng.random())
    u = np.array([a for a, _ in pairs], np.int32)
    i = np.array([b for _, b in pairs], np.int32)
    return u, i, rng.integers(1, 6, nnz).astype(float), nu, ni


def _qd_setup(world):
    import rotq_model as RQ
    import qdelta_model as QM
    u, i, r, nu, ni = _qd_data()
    rng = np.random.default_rng(8)
    P0, Q0 = rng.normal(0, 0.1, (nu, K)), rng.normal(0, 0.1, (ni, K))
    ub = RQ.block_bounds(u, nu, world)
    shards = [((u >= ub[g]) & (u < ub[g + 1])) for g in range(world)]
    cnt = np.bincount(i, minlength=ni).astype(np.float64)
    c = np.sum([np.bincount(i[m], minlength=ni) > 0 for m in shards], 0).astype(np.float64)
    hot = QM.hot_items(cnt, c, QD_MERGES)
    w = QM.weights(cnt, c, 0.005, QD_MERGES, hot, k=K)
    blocks = []  # per rank: its merges' user blocks (user_block_bounds over the rank's own ratings)
    for g, m in enumerate(shards):
        bb = RQ.block_bounds(u[m], nu, QD_MERGES)
        blocks.append([_stratum_rows(u[m], i[m], r[m], bb[b], bb[b + 1]) for b in range(QD_MERGES)])
    return RQ, QM, u, i, r, nu, ni, P0, Q0, ub, w, hot, blocks


def _stratum_rows(u, i, r, lo, hi):
    m = (u >= lo) & (u < hi)
    o = np.argsort(u[m], kind="stable")
    return u[m][o].astype(np.int32), i[m][o].astype(np.int32), r[m][o]


def _qd_train(RQ, P, rows, bu, gb, blk):
    """One block of a rank: (P, b_u, the rank's [Q | b_i] after it, its GlobalBias partial)."""
    P, Qn, bu, bin_, part = RQ.train_works(P, rows[:, :K].copy(), bu, rows[:, K].copy(), gb, [blk])
    return P, bu, np.concatenate([Qn, bin_[:, None]], 1), part


def _qd_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    RQ, QM, u, i, r, nu, ni, P0, Q0, ub, w, hot, blocks = _qd_setup(world)
    P, bu, gb = P0.copy(), np.zeros(nu), 3.0
    rows = np.concatenate([Q0, np.zeros((ni, 1))], 1)
    st = QM.Rank(rows)
    pend_gb = None  # merge m - 1's GlobalBias partials, folded after block m
    n_merges = EPOCHS * QD_MERGES
    for m in range(n_merges):
        X, _ = QM.merge_set(m, QD_MERGES, hot)
        P, bu, rows, part = _qd_train(RQ, P, rows, bu, gb, blocks[rank][m % QD_MERGES])
        rows = st.merge(rows, X, w)
        t = torch.from_numpy(st.own.copy())
        g = torch.tensor([part], dtype=torch.float64)
        dist.all_reduce(t)  # (the library all-reduces only the rows of X; the others' moves are zero here)
        dist.all_reduce(g)
        st.settle(t.numpy(), X)
        if pend_gb is not None:
            gb += pend_gb / len(r)
        pend_gb = float(g.item())
    rows = st.flush(rows)
    gb += pend_gb / len(r)
    for g in range(world):  # P range g is current on rank g
        pr = torch.from_numpy(np.concatenate([P[ub[g]:ub[g + 1]], bu[ub[g]:ub[g + 1], None]], 1).copy())
        dist.broadcast(pr, g)
        P[ub[g]:ub[g + 1]], bu[ub[g]:ub[g + 1]] = pr[:, :K].numpy(), pr[:, K].numpy()
    out[rank] = (P, rows[:, :K], bu, rows[:, K], gb)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_qdelta_matches_single_process(world):
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_qd_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    RQ, QM, u, i, r, nu, ni, P0, Q0, ub, w, hot, blocks = _qd_setup(world)
    # the single-process run of the same rules: the ranks train one after another (disjoint users), each from
    # its own rows, and the merges' sums are formed here
    P, bu, gb = P0.copy(), np.zeros(nu), 3.0
    rows = [np.concatenate([Q0, np.zeros((ni, 1))], 1) for _ in range(world)]
    st = [QM.Rank(x) for x in rows]
    pend_gb, n_merges = None, EPOCHS * QD_MERGES
    assert hot.any() and not hot.all()  # both hot merges and full merges move rows
    for m in range(n_merges):
        X, _ = QM.merge_set(m, QD_MERGES, hot)
        part = 0.0
        for g in range(world):
            P, bu, rows[g], p = _qd_train(RQ, P, rows[g], bu, gb, blocks[g][m % QD_MERGES])
            rows[g] = st[g].merge(rows[g], X, w)
            part += p
        total = sum(x.own for x in st)
        for x in st:
            x.settle(total, X)
        if pend_gb is not None:
            gb += pend_gb / len(r)
        pend_gb = part
    rows = [x.flush(y) for x, y in zip(st, rows)]
    gb += pend_gb / len(r)
    Q, bi = rows[0][:, :K], rows[0][:, K]
    assert ((0.0 < w) & (w < 1.0)).any()  # items on several ranks: weighted merges are exercised
    for rank in range(world):
        rP, rQ, rbu, rbi, rgb = res[rank]
        np.testing.assert_allclose(rP, P, atol=1e-12)
        np.testing.assert_allclose(rbu, bu, atol=1e-12)
        np.testing.assert_allclose(rQ, Q, atol=1e-12)
        np.testing.assert_allclose(rbi, bi, atol=1e-12)
        assert abs(rgb - gb) < 1e-12
        for x in (0, 2):  # the P ranges are broadcast; Q in this fp64 model is start + own + (sum - own): equal to
            np.testing.assert_array_equal(res[0][x], res[rank][x])  # rounding here, bit-equal in the int32 path
