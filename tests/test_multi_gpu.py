"""GPU tests of the item-sharded multi-GPU path behind the C-ABI (csrc/multi.hip; north_star's item
sharding, core/svd.go:92-130 per shard).

The one-GPU box runs N shards of one device through the in-process exchange (rs_svd_group with plans
sharing a device) and the RCCL code with a single rank (rs_svd_group of one device, rs_svd_plan_join
with n_ranks = 1): the schedule, the GlobalBias fold and the final broadcast are the same code as with
8 GPUs; only RCCL's p2p transfers between two devices are unexercised ("unmeasured on hardware").

ROTATE (the default exchange) checker: with one workgroup of one wave per shard the epoch is the
sequential SGD of svd.go:93-129 over the strata in rotation order -- sub-epoch s, shard g, rank-block
(g + s) mod N, its tiles in the exported order -- with the work-local GlobalBias fold of the FAST
schedules; the oracle restates exactly that (or_svd_fit_works).  The strata of one sub-epoch share no
P or Q row, so their order inside the sub-epoch is immaterial.  Accuracy with the default schedule
(16 waves): P2, RMSE within 0.003 of the reference visit order at 2, 4 and 8 shards.

AVERAGE (round 2's protocol, selectable): the delta protocol run by hand on plans of the same
schedule, as before.
"""
import os

import numpy as np
import pytest

import oracle as O
import qdelta_model as QM
import rsgpu
from helpers import folds, rmse
from rsgpu import synth

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _maxdiff(a, b):
    return max(float(np.max(np.abs(np.asarray(x) - np.asarray(y)))) for x, y in zip(a, b))


def _shards(u, i, r, nu, ni, n):
    b = rsgpu.item_shards(i, ni, n)
    out = []
    for s in range(n):
        m = (i >= b[s]) & (i < b[s + 1])
        out.append((u[m], i[m] - b[s], r[m], nu, int(b[s + 1] - b[s]), int(b[s])))
    return out


def _bounds(shards, nu, blocks):
    """The library's common user-block bounds: from every user's ratings over all shards, the b-th
    bound is the first user whose ratings start at or past b/blocks of them."""
    cnt = sum(np.bincount(su, minlength=nu) for su, *_ in shards)
    cum = np.concatenate([[0], np.cumsum(cnt)])
    return np.array([np.searchsorted(cum, cum[-1] * b // blocks, side="left") for b in range(blocks)] + [nu])


def _plans(ctx, shards, k, P0, Q0, blocks, waves=1, wg=1, mode=rsgpu.EXCHANGE_ROTATE, gb0=3.5):
    plans = []
    bounds = _bounds(shards, shards[0][3], blocks)
    for su, si, sr, nu, ni_s, lo in shards:
        pl = ctx.svd_plan(rsgpu.Ratings(su, si, sr, nu, ni_s), k)
        pl.set_tiles(workgroups=wg, waves=waves)
        pl.set_user_blocks(blocks, bounds)
        pl.set_exchange(mode)
        pl.upload(P0, Q0[lo:lo + ni_s], np.zeros(nu), np.zeros(ni_s), gb0)
        plans.append(pl)
    return plans


def _rotation_oracle(plans, shards, bounds, pieces, P0, Q0, gb0, epochs):
    """or_svd_fit_works over the strata in rotation order (global user / item ids)."""
    n = len(plans)
    strata = {}  # (shard, user block) -> (u, i, r, works)
    for g, (pl, (su, si, sr, nu, ni_s, lo)) in enumerate(zip(plans, shards)):
        rowptr, items, rr = O.csr_by(su, nu, si, sr)
        cu = np.repeat(np.arange(nu, dtype=np.int32), np.diff(rowptr))
        pos, off = pl.tile_order()
        uu, ii, r_ = cu[pos], np.asarray(items, np.int32)[pos] + lo, np.asarray(rr)[pos]
        for w in range(len(off) - 1):
            if off[w + 1] == off[w]:
                continue
            b = int(np.searchsorted(bounds, uu[off[w]], side="right") - 1)
            strata.setdefault((g, b), []).append((off[w], off[w + 1], uu, ii, r_))
    U, I, R, W = [], [], [], [0]
    for st in range(n):
        for g in range(n):
            for j in range(pieces):
                b = ((g + st) % n) * pieces + j
                for a, z, uu, ii, r_ in strata.get((g, b), []):
                    U.append(uu[a:z])
                    I.append(ii[a:z])
                    R.append(r_[a:z])
                    W.append(W[-1] + (z - a))
    U, I, R = np.concatenate(U), np.concatenate(I), np.concatenate(R)
    return O.svd_fit_works(U, I, R, np.array(W, np.int64), P0, Q0, np.zeros(P0.shape[0]),
                           np.zeros(Q0.shape[0]), gb0, epochs=epochs)


@pytest.mark.parametrize("n_shards,pieces", [(2, 1), (2, 2), (3, 1), (4, 2), (8, 1)])
def test_rotation_one_wave_equals_oracle(ctx, ml100k, n_shards, pieces):
    """ROTATE through the in-process exchange (shards on device 0), one wave per shard: equal to the
    sequential SGD over the strata in rotation order (1e-5), P / b_u / GlobalBias bitwise identical on
    every shard after the call (the final broadcast)."""
    f = folds(*ml100k)[2]
    n = 30000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    k = 24
    rng = np.random.default_rng(n_shards + 10 * pieces)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    sh = _shards(u, i, r, nu, ni, n_shards)
    blocks = n_shards * pieces
    got = _plans(ctx, sh, k, P0, Q0, blocks)
    g = rsgpu.SvdGroup(got, n_blocks=blocks)
    g.epochs(2)
    ref = _rotation_oracle(got, sh, _bounds(sh, nu, blocks), pieces, P0, Q0, 3.5, 2)
    g.close()
    b = [pl.download() for pl in got]
    for pl in got:
        pl.close()
    Qg = np.concatenate([x[1] for x in b])
    big = np.concatenate([x[3] for x in b])
    assert _maxdiff((ref[0], ref[1], ref[2], ref[3]), (b[0][0], Qg, b[0][2], big)) <= TOL
    assert abs(ref[4] - b[0][4]) <= TOL  # a run's GlobalBias steps are summed in fp32 (sgd_tile.hip)
    for y in b[1:]:  # the replicated state is bitwise identical across shards
        assert np.array_equal(b[0][0], y[0]) and np.array_equal(b[0][2], y[2]) and b[0][4] == y[4]


def _block_bounds(keys, n, blocks):
    """The library's block bounds over rows counted by `keys` (user_block_bounds): the b-th bound is the
    first row whose ratings start at or past b/blocks of them."""
    cum = np.concatenate([[0], np.cumsum(np.bincount(keys, minlength=n))])
    return np.array([np.searchsorted(cum, cum[-1] * b // blocks, side="left") for b in range(blocks)] + [n])


def _user_shards(u, i, r, nu, n):
    """ROTATE_Q shards: the ratings of contiguous user ranges of near-equal ratings, global ids."""
    b = _block_bounds(u, nu, n)
    return [(u[(u >= b[s]) & (u < b[s + 1])], i[(u >= b[s]) & (u < b[s + 1])], r[(u >= b[s]) & (u < b[s + 1])])
            for s in range(n)]


@pytest.mark.parametrize("n_shards,pieces", [(2, 1), (2, 2), (3, 1), (4, 2), (8, 1)])
def test_rotation_q_one_wave_equals_oracle(ctx, ml100k, n_shards, pieces):
    """ROTATE_Q (user ranges stay, item rank-blocks rotate) through the in-process exchange, one wave per
    shard: equal to the sequential SGD over the strata in rotation order -- sub-epoch s, shard g, item
    blocks of rank-block (g + s) mod N, each stratum's tiles in the exported order -- (1e-5), and P, Q,
    the biases and GlobalBias bitwise identical on every shard after the call (the final broadcast)."""
    f = folds(*ml100k)[2]
    n = 30000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    k = 24
    rng = np.random.default_rng(50 + n_shards + 10 * pieces)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    sh = _user_shards(u, i, r, nu, n_shards)
    blocks = n_shards * pieces
    ib = _block_bounds(i, ni, blocks)
    plans = []
    for su, si, sr in sh:
        pl = ctx.svd_plan(rsgpu.Ratings(su, si, sr, nu, ni), k)
        pl.set_tiles(workgroups=1, waves=1)
        pl.set_exchange(rsgpu.EXCHANGE_ROTATE_Q)
        pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
        plans.append(pl)
    g = rsgpu.SvdGroup(plans, n_blocks=blocks)
    assert all(pl.shard_info()[2:] == (rsgpu.EXCHANGE_ROTATE_Q, blocks) for pl in plans)
    g.epochs(2)
    strata = {}  # (shard, item block) -> works
    for gi, (pl, (su, si, sr)) in enumerate(zip(plans, sh)):
        rowptr, items, rr = O.csr_by(su, nu, si, sr)
        cu = np.repeat(np.arange(nu, dtype=np.int32), np.diff(rowptr))
        pos, off = pl.tile_order()
        assert np.array_equal(np.sort(pos), np.arange(len(sr)))
        uu, ii, r_ = cu[pos], np.asarray(items, np.int32)[pos], np.asarray(rr)[pos]
        for w in range(len(off) - 1):
            if off[w + 1] > off[w]:
                b = int(np.searchsorted(ib, ii[off[w]], side="right") - 1)
                assert np.all((ii[off[w]:off[w + 1]] >= ib[b]) & (ii[off[w]:off[w + 1]] < ib[b + 1]))
                strata.setdefault((gi, b), []).append((off[w], off[w + 1], uu, ii, r_))
    U, I, R, W = [], [], [], [0]
    for st in range(n_shards):
        for gi in range(n_shards):
            for j in range(pieces):
                for a, z, uu, ii, r_ in strata.get((gi, ((gi + st) % n_shards) * pieces + j), []):
                    U.append(uu[a:z])
                    I.append(ii[a:z])
                    R.append(r_[a:z])
                    W.append(W[-1] + (z - a))
    ref = O.svd_fit_works(np.concatenate(U), np.concatenate(I), np.concatenate(R), np.array(W, np.int64), P0, Q0,
                          np.zeros(nu), np.zeros(ni), 3.5, epochs=2)
    g.close()
    b = [pl.download() for pl in plans]
    for pl in plans:
        pl.close()
    assert _maxdiff(ref[:4], b[0][:4]) <= TOL and abs(ref[4] - b[0][4]) <= TOL
    for y in b[1:]:
        assert all(np.array_equal(b[0][x], y[x]) for x in range(4)) and b[0][4] == y[4]


@pytest.mark.parametrize("n_shards,pieces", [(2, 2), (3, 1)])
def test_rotation_q_hot_copies_equal_host_model(ctx, ml100k, n_shards, pieces):
    """ROTATE_Q with a forced hot split (share 1 %, no stratum minimum: ML-100K's head items get per-block
    copies), in-process exchange, one wave per shard: equal (1e-5) to tests/rotq_model.py's sequential
    model -- the same model the world-size 2 / 3 gloo run of tests/test_multi.py matches -- with every
    stratum's ratings in the tile order the shard exports, the copies' moves merged once per epoch with
    RS_HOT_SCALED's weights, and the replicated state bitwise identical on every shard."""
    import rotq_model as RQ
    f = folds(*ml100k)[2]
    n = 30000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    k = 24
    rng = np.random.default_rng(70 + n_shards)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    ub = _block_bounds(u, nu, n_shards)
    sh = _user_shards(u, i, r, nu, n_shards)
    lay = RQ.Layout(u, i, ni, n_shards, pieces, hot_share=0.01, min_stratum=0)
    assert lay.H >= 4 and any(c > 1 for _, c in lay.meta)
    plans = []
    for su, si, sr in sh:
        pl = ctx.svd_plan(rsgpu.Ratings(su, si, sr, nu, ni), k)
        pl.set_tiles(workgroups=1, waves=1)
        pl.set_exchange(rsgpu.EXCHANGE_ROTATE_Q)
        pl.set_hot_split(0.01, 0, 0)
        pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
        plans.append(pl)
    g = rsgpu.SvdGroup(plans, n_blocks=n_shards * pieces)
    g.epochs(2)
    strata = {}  # (shard, block) -> works in the shard's visit order
    for gi, (pl, (su, si, sr)) in enumerate(zip(plans, sh)):
        rowptr, items, rr = O.csr_by(su, nu, si, sr)
        cu = np.repeat(np.arange(nu, dtype=np.int32), np.diff(rowptr))
        pos, off = pl.tile_order()
        uu, ii, r_ = cu[pos], np.asarray(items, np.int32)[pos], np.asarray(rr)[pos]
        for w in range(len(off) - 1):
            a, z = off[w], off[w + 1]
            if z == a:
                continue
            blk = {lay.block_of(x, y) for x, y in zip(uu[a:z], ii[a:z])}
            assert len(blk) == 1  # a work lies in one stratum
            b = blk.pop()
            rows = np.array([lay.row_of(b, y) for y in ii[a:z]], np.int32)
            strata.setdefault((gi, b), []).append((uu[a:z], rows, r_[a:z]))
    ref = RQ.sequential(lay, u, i, r, nu, P0, Q0, 3.5, 2, ub, lambda gi, b: strata.get((gi, b), []))
    g.close()
    got = [pl.download() for pl in plans]
    for pl in plans:
        pl.close()
    assert _maxdiff(ref[:4], got[0][:4]) <= TOL and abs(ref[4] - got[0][4]) <= TOL
    for y in got[1:]:
        assert all(np.array_equal(got[0][x], y[x]) for x in range(4)) and got[0][4] == y[4]


@pytest.mark.parametrize("n_shards,merges", [(2, 1), (3, 1), (8, 1), (2, 3), (4, 2), (2, 8)])
def test_qdelta_one_wave_equals_host_model(ctx, ml100k, n_shards, merges):
    """RS_EXCHANGE_QDELTA through the in-process exchange (int32 wire), one wave per shard: each shard trains
    its user range block by block (the oracle's sequential SGD in the shard's exported tile order, P in place)
    and merges the hot items after every block and every item after every cold_every-th block, with the
    kappa / c weights and pipelined corrections (tests/qdelta_model.py) -- equal to that host model to 1e-5,
    with the library's hot-item count, and P, Q, the biases and GlobalBias identical on every shard after the
    call (the P-range broadcast; Q and GlobalBias are the same integer sums everywhere)."""
    f = folds(*ml100k)[2]
    n = 30000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    k, lr, epochs = 24, 0.005, 2
    rng = np.random.default_rng(90 + n_shards)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    sh = _user_shards(u, i, r, nu, n_shards)
    plans = []
    for su, si, sr in sh:
        pl = ctx.svd_plan(rsgpu.Ratings(su, si, sr, nu, ni), k)
        pl.set_tiles(workgroups=1, waves=1)
        pl.set_exchange(rsgpu.EXCHANGE_QDELTA)
        pl.set_qdelta_wire(32)  # exact integer sums (the fp16 wire: test_qdelta_fp16_wire_tracks_int32)
        pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
        plans.append(pl)
    g = rsgpu.SvdGroup(plans, n_blocks=merges)
    assert all(pl.shard_info()[2] == rsgpu.EXCHANGE_QDELTA for pl in plans)
    g.epochs(epochs, lr=lr)
    works = []  # per shard and merge: (users, items, ratings, work offsets) in the shard's visit order
    for pl, (su, si, sr) in zip(plans, sh):
        rowptr, items, rr = O.csr_by(su, nu, si, sr)
        cu = np.repeat(np.arange(nu, dtype=np.int32), np.diff(rowptr))
        pos, off = pl.tile_order()
        uu, ii, r_ = cu[pos], np.asarray(items, np.int32)[pos], np.asarray(rr)[pos]
        ub = _block_bounds(su, nu, merges)  # the merges' user blocks (user_block_bounds of the shard's ratings)
        per = [[] for _ in range(merges)]
        for x in range(len(off) - 1):
            if off[x + 1] > off[x]:
                per[int(np.searchsorted(ub, uu[off[x]], side="right") - 1)].append((off[x], off[x + 1]))
        for b in range(merges):
            seg = per[b]
            sel = np.concatenate([np.arange(a, z) for a, z in seg]) if seg else np.zeros(0, np.int64)
            wo = np.concatenate([[0], np.cumsum([z - a for a, z in seg])]).astype(np.int64)
            per[b] = (uu[sel], ii[sel], r_[sel], wo)
        works.append(per)
    cnt = np.bincount(i, minlength=ni).astype(np.float64)
    c = np.sum([np.bincount(x[1], minlength=ni) > 0 for x in sh], 0).astype(np.float64)
    hot = QM.hot_items(cnt, c, merges)
    w = QM.weights(cnt, c, lr, merges, hot, k=k).astype(np.float32).astype(np.float64)  # (the library's defaults)
    assert all(pl.qdelta_info() == (int(hot.sum()), QM.cold_every(merges)) for pl in plans)
    if merges in (2, 8):  # hot merges and full merges both move rows
        assert 0 < hot.sum() < ni
    # the merge rules of tests/qdelta_model.py: each shard trains its block from its own rows, merges the hot
    # rows (or every row, at a full merge) with its own weighted moves and the corrections pending from the
    # rows' previous merges; GlobalBias folds merge m's partials after block m + 1
    P, bu, gb = P0.copy(), np.zeros(nu), 3.5
    rows = [np.concatenate([Q0, np.zeros((ni, 1))], 1) for _ in sh]
    st = [QM.Rank(x) for x in rows]
    pend_gb = None
    for m in range(epochs * merges):
        b = m % merges
        X, _ = QM.merge_set(m, merges, hot)
        part = 0.0
        for x, per in enumerate(works):
            uu, ii, r_, off = per[b]
            if len(r_):
                P, Qg, bu, big, gg = O.svd_fit_works(uu, ii, r_, off, P, rows[x][:, :k], bu, rows[x][:, k], gb, epochs=1,
                                                     lr=lr)
                rows[x] = np.concatenate([Qg, big[:, None]], 1)
                part += (gg - gb) * len(r_)
            rows[x] = st[x].merge(rows[x], X, w)
        total = sum(y.own for y in st)
        for y in st:
            y.settle(total, X)
        if pend_gb is not None:
            gb += pend_gb / len(r)
        pend_gb = part
    rows = [y.flush(z) for y, z in zip(st, rows)]
    gb += pend_gb / len(r)
    Q, bi = rows[0][:, :k], rows[0][:, k]
    g.close()
    got = [pl.download() for pl in plans]
    for pl in plans:
        pl.close()
    assert _maxdiff((P, Q, bu, bi), got[0][:4]) <= TOL and abs(gb - got[0][4]) <= TOL
    for y in got[1:]:
        assert all(np.array_equal(got[0][x], y[x]) for x in range(4)) and got[0][4] == y[4]


@pytest.mark.parametrize("n_shards,merges", [(2, 1), (4, 3), (8, 4)])
def test_qdelta_fp16_wire_tracks_int32(ctx, ml100k, n_shards, merges):
    """The default fp16 wire (rs_svd_plan_set_qdelta_wire 16): every shard ends with the same bits (each applies
    the same rounded moves), and the fit stays within 2e-3 of the exact int32-wire fit (fp16 keeps 11 bits of
    each merge's move) with held-out RMSE within 1e-3 of it.  The in-process sum is the arithmetic of RCCL's ring
    (qdelta_sum_kernel<16>): per chunk a rotated start rank, the ranks in ring order, rounded to fp16 after every
    add -- 7 roundings per value at 8 shards, as an 8-GPU all-reduce makes them."""
    f = folds(*ml100k)[1]
    u, i, r, nu, ni = f.iu, f.ii, f.r, f.nu, f.ni
    k, lr, epochs = 32, 0.005, 5
    rng = np.random.default_rng(7)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    sh = _user_shards(u, i, r, nu, n_shards)
    res = {}
    for bits in (32, 16):
        plans = []
        for su, si, sr in sh:
            pl = ctx.svd_plan(rsgpu.Ratings(su, si, sr, nu, ni), k)
            pl.set_tiles(workgroups=1, waves=1)  # deterministic: the two runs differ only by the wire
            pl.set_exchange(rsgpu.EXCHANGE_QDELTA)
            pl.set_qdelta_wire(bits)
            pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), float(np.mean(r)))
            plans.append(pl)
        g = rsgpu.SvdGroup(plans, n_blocks=merges)
        g.epochs(epochs, lr=lr)
        g.close()
        got = [pl.download() for pl in plans]
        for y in got[1:]:
            bad = [(x, float(np.max(np.abs(got[0][x] - y[x]))), int(np.sum(got[0][x] != y[x]))) for x in range(4)
                   if not np.array_equal(got[0][x], y[x])]
            assert not bad and got[0][4] == y[4], (bits, bad, got[0][4], y[4])
        res[bits] = (got[0], rmse(O.svd_predict(f.tu, f.ti, *got[0]), f.te_r))
        for pl in plans:
            pl.close()
    assert _maxdiff(res[16][0][:4], res[32][0][:4]) <= 2e-3
    assert abs(res[16][1] - res[32][1]) <= 1e-3, (res[16][1], res[32][1])


@pytest.mark.parametrize("mode", [rsgpu.EXCHANGE_QDELTA, rsgpu.EXCHANGE_ROTATE_Q, rsgpu.EXCHANGE_ROTATE])
def test_replica_check_catches_a_diverged_shard(ctx, ml100k, mode):
    """The consistency check after a sharded call (multi.hip check_replicas): one shard's replicated factors
    changed by one word (test hook RS_FAULT_DIVERGE) make the call fail with RS_ERR_NUMERIC on the group; the
    same call without the fault passes the check, and a later call on the same group is checked again."""
    f = folds(*ml100k)[0]
    u, i, r, nu, ni = f.iu[:20000], f.ii[:20000], f.r[:20000], f.nu, f.ni
    k = 16
    rng = np.random.default_rng(33)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    if mode == rsgpu.EXCHANGE_ROTATE:
        plans = _plans(ctx, _shards(u, i, r, nu, ni, 3), k, P0, Q0, 3, wg=0, waves=16, mode=mode)
    else:
        plans = []
        for su, si, sr in _user_shards(u, i, r, nu, 3):
            pl = ctx.svd_plan(rsgpu.Ratings(su, si, sr, nu, ni), k)
            pl.set_exchange(mode)
            pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
            plans.append(pl)
    g = rsgpu.SvdGroup(plans, n_blocks=3 if mode == rsgpu.EXCHANGE_ROTATE else 0)
    g.epochs(1)  # clean: passes
    plans[1].inject_fault(rsgpu.FAULT_DIVERGE)
    with pytest.raises(rsgpu.RsError) as e:
        g.epochs(1)
    assert e.value.code == rsgpu.RS_ERR_NUMERIC and "disagree" in str(e.value)
    g.close()
    for pl in plans:
        pl.close()


def test_qdelta_edge_shards(ctx, ml100k):
    """QDELTA edge cases, in-process group: a shard whose user range holds no ratings (its plan trains nothing
    and still takes part in every merge), more merges than a shard has users, and an item no shard rates --
    the fit stays finite, every shard ends with the same bits, and the empty shard's start P rows for its
    (unrated) users come back unchanged."""
    f = folds(*ml100k)[4]
    u, i, r, nu, ni = f.iu[:20000], f.ii[:20000], f.r[:20000], f.nu, f.ni + 3  # 3 items nobody rates
    k = 16
    rng = np.random.default_rng(21)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    lo = int(np.max(u)) + 1  # users past the last rated one: an empty range for the third shard
    sh = [(u[u < nu // 3], i[u < nu // 3], r[u < nu // 3]), (u[u >= nu // 3], i[u >= nu // 3], r[u >= nu // 3]),
          (np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0))]
    plans = []
    for su, si, sr in sh:
        pl = ctx.svd_plan(rsgpu.Ratings(su, si, sr, nu, ni), k)
        pl.set_exchange(rsgpu.EXCHANGE_QDELTA)
        pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
        plans.append(pl)
    g = rsgpu.SvdGroup(plans, n_blocks=64)
    g.epochs(3)
    g.close()
    got = [pl.download() for pl in plans]
    for pl in plans:
        pl.close()
    assert all(np.all(np.isfinite(x)) for x in got[0][:4]) and np.isfinite(got[0][4])
    for y in got[1:]:
        assert all(np.array_equal(got[0][x], y[x]) for x in range(4)) and got[0][4] == y[4]
    assert np.allclose(got[0][1][-3:], Q0[-3:], atol=1e-7)  # unrated items: the start rows (2^-24 fixed point)
    assert not np.array_equal(got[0][0][: nu // 3], P0[: nu // 3])
    if lo < nu:
        assert np.allclose(got[0][0][lo:], P0[lo:], atol=1e-6)


def test_rccl_single_rank_qdelta_equals_group_of_one(ctx, ml100k):
    """QDELTA through the RCCL join with one rank (communicator, comm stream, events; no collective runs at
    N = 1): the same blocks, GlobalBias folds and results as the in-process group of one plan (one wave)."""
    f = folds(*ml100k)[1]
    n = 20000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    k = 24
    rng = np.random.default_rng(5)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    out = []
    for join in (True, False):
        pl = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
        pl.set_tiles(workgroups=1, waves=1)
        pl.set_exchange(rsgpu.EXCHANGE_QDELTA)
        pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
        if join:
            pl.join(rsgpu.comm_unique_id(), 0, 1, 4)
            assert pl.shard_info()[1:] == (1, rsgpu.EXCHANGE_QDELTA, 4)
            pl.epochs_sharded(2)
            pl.leave()
        else:
            g = rsgpu.SvdGroup([pl], n_blocks=4)
            g.epochs(2)
            g.close()
        out.append(pl.download())
        pl.close()
    assert _maxdiff(out[0][:4], out[1][:4]) <= TOL and abs(out[0][4] - out[1][4]) <= TOL


def test_rotation_fewer_users_than_blocks(ctx):
    """ROTATE with more user blocks than users (4 shards x 2 pieces, 5 users): empty blocks send and
    receive nothing and the fit still equals a single plan's users trained (finite, every rating seen)."""
    rng = np.random.default_rng(4)
    nu, ni, k = 5, 40, 8
    u = rng.integers(0, nu, 300).astype(np.int32)
    i = rng.integers(0, ni, 300).astype(np.int32)
    r = rng.integers(1, 6, 300).astype(float)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    sh = _shards(u, i, r, nu, ni, 4)
    plans = _plans(ctx, sh, k, P0, Q0, 8)
    g = rsgpu.SvdGroup(plans, n_blocks=8)
    g.epochs(3)
    g.close()
    b = [pl.download() for pl in plans]
    for pl in plans:
        pl.close()
    assert all(np.all(np.isfinite(x)) for y in b for x in y[:4])
    assert not np.array_equal(b[0][0], P0)


@pytest.mark.parametrize("api", ["group", "join"])
def test_rccl_single_rank_rotation_equals_oracle(ctx, ml100k, api):
    """The RCCL exchange (communicator, comm stream, events, GlobalBias fold) with one rank: the
    rotation degenerates to the user blocks in order, equal to the oracle in tile order (1e-5)."""
    f = folds(*ml100k)[3]
    n = 30000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    k = 40
    rng = np.random.default_rng(11)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    sh = _shards(u, i, r, nu, ni, 1)
    got = _plans(ctx, sh, k, P0, Q0, 3)
    if api == "group":
        g = rsgpu.SvdGroup(got, n_blocks=3)
        g.epochs(3)
        ref = _rotation_oracle(got, sh, _bounds(sh, nu, 3), 3, P0, Q0, 3.5, 3)
        g.close()
    else:
        got[0].join(rsgpu.comm_unique_id(), 0, 1, 3)
        got[0].epochs_sharded(3)
        ref = _rotation_oracle(got, sh, _bounds(sh, nu, 3), 3, P0, Q0, 3.5, 3)
        got[0].leave()
    b = got[0].download()
    got[0].close()
    assert _maxdiff(ref[:4], b[:4]) <= TOL and abs(ref[4] - b[4]) <= TOL


def test_rotation_shard_failure_releases_the_others(ctx, ml100k):
    """A shard that throws mid-epoch (test hook rs_svd_plan_inject_fault) makes rs_svd_group_epochs return
    its error instead of leaving the other shards blocked at the exchange."""
    f = folds(*ml100k)[0]
    k = 16
    rng = np.random.default_rng(3)
    P0, Q0 = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
    sh = _shards(f.iu, f.ii, f.r, f.nu, f.ni, 3)
    plans = _plans(ctx, sh, k, P0, Q0, 3)
    g = rsgpu.SvdGroup(plans, n_blocks=3)
    plans[1].inject_fault(2)  # the last sub-epoch
    with pytest.raises(rsgpu.RsError) as e:
        g.epochs(1)
    assert "shard 1" in str(e.value) or "another shard" in str(e.value)
    g.close()
    for pl in plans:
        pl.close()


@pytest.mark.parametrize("n_dev", [2, 8])
def test_fit_multi_rmse_parity_ml100k(ctx, ml100k, n_dev):
    """P2 for rs_svd_fit_multi (ROTATE, default tile schedule, 16 waves) with 2 and 8 item shards on
    device 0: 5-fold ML-100K held-out RMSE within 0.003 of the reference visit order and under
    core/base_test.go:35's bound (0.934 + 0.008)."""
    k = 100
    ref_r, gpu_r = [], []
    for f in folds(*ml100k):
        rng = np.random.default_rng(7)
        P0, Q0 = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
        ref_r.append(rmse(O.svd_predict(f.tu, f.ti, *O.svd_fit(f.iu, f.ii, f.r, P0, Q0)), f.te_r))
        got = rsgpu.svd_fit_multi([0] * n_dev, rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), P0, Q0)
        assert all(np.all(np.isfinite(x)) for x in got[:4])
        gpu_r.append(rmse(O.svd_predict(f.tu, f.ti, *got), f.te_r))
    g, ref = float(np.mean(gpu_r)), float(np.mean(ref_r))
    print(f"n_dev={n_dev}: fit_multi RMSE {g:.4f} vs reference order {ref:.4f}")
    assert abs(g - ref) <= 0.003, (g, ref)
    assert g <= 0.934 + 0.008


_ML1M = {}


def _ml1m_holdout():
    if not _ML1M:
        u, i, r, nu, ni = synth.ml1m_like()
        n = len(r)
        te = np.zeros(n, bool)
        te[np.random.default_rng(9).permutation(n)[: n // 10]] = True
        tr = ~te
        rng = np.random.default_rng(5)
        P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
        ref = O.svd_fit(u[tr], i[tr], r[tr], P0, Q0, epochs=20)
        _ML1M.update(u=u, i=i, r=r, nu=nu, ni=ni, tr=tr, te=te, P0=P0, Q0=Q0,
                     e_ref=rmse(O.svd_predict(u[te], i[te], *ref), r[te]))
    return _ML1M


@pytest.mark.parametrize("n_dev", [2, 4, 8])
def test_fit_multi_rmse_parity_ml1m_holdout(ctx, n_dev):
    """P2 at config-2 scale for the sharded fit: ML-1M-shaped set, 90/10 split, k=100, 20 epochs, 2/4/8
    item shards on device 0; held-out RMSE within 0.003 of the reference visit order's."""
    d = _ml1m_holdout()
    u, i, r, tr, te = d["u"], d["i"], d["r"], d["tr"], d["te"]
    got = rsgpu.svd_fit_multi([0] * n_dev, rsgpu.Ratings(u[tr], i[tr], r[tr], d["nu"], d["ni"]), d["P0"], d["Q0"])
    e = rmse(rsgpu.svd_predict(u[te], i[te], *got), r[te])
    print(f"n_dev={n_dev}: ML-1M held-out RMSE {e:.4f} vs reference order {d['e_ref']:.4f}")
    assert abs(e - d["e_ref"]) <= 0.003, (e, d["e_ref"])


# ---- AVERAGE (round 2's delta protocol, selectable) ---------------------------------------------

def _manual(plans, shards, nu, epochs):
    """The delta protocol by hand (torch buffers, sum in shard order)."""
    import torch
    tot = np.zeros(nu)
    for su, *_ in shards:
        tot += np.bincount(su, minlength=nu)
    total = sum(len(sr) for _, _, sr, *_ in shards)
    for pl, (su, *_) in zip(plans, shards):
        c = np.bincount(su, minlength=nu)
        pl.set_user_weights(np.divide(c, tot, out=np.zeros(nu), where=tot > 0).astype(np.float32))
    ld = plans[0].ld
    dPs = [torch.zeros((nu, ld), dtype=torch.float32, device="cuda") for _ in plans]
    gs = [torch.zeros(1, dtype=torch.float64, device="cuda") for _ in plans]
    for _ in range(epochs):
        for pl, dP, g in zip(plans, dPs, gs):
            pl.epoch_delta_t(dP, g, 0.005, 0.02)
        torch.cuda.synchronize()
        sdP, sg = dPs[0].clone(), gs[0].clone()
        for dP, g in zip(dPs[1:], gs[1:]):
            sdP += dP
            sg += g
        for pl in plans:
            pl.apply_delta_t(sdP, sg, 1.0 / total)
        torch.cuda.synchronize()


@pytest.mark.parametrize("n_shards,blocks", [(2, 1), (2, 3), (3, 4)])
def test_average_group_on_one_device_equals_manual_protocol(ctx, ml100k, n_shards, blocks):
    f = folds(*ml100k)[2]
    u, i, r, nu, ni = f.iu, f.ii, f.r, f.nu, f.ni
    k = 24
    rng = np.random.default_rng(n_shards + blocks)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    sh = _shards(u, i, r, nu, ni, n_shards)
    ref = _plans(ctx, sh, k, P0, Q0, blocks, mode=rsgpu.EXCHANGE_AVERAGE)
    _manual(ref, sh, nu, epochs=2)
    got = _plans(ctx, sh, k, P0, Q0, blocks, mode=rsgpu.EXCHANGE_AVERAGE)
    g = rsgpu.SvdGroup(got, n_blocks=blocks)
    g.epochs(2)
    g.close()
    a = [pl.download() for pl in ref]
    b = [pl.download() for pl in got]
    for pl in ref + got:
        pl.close()
    for x, y in zip(a, b):
        assert _maxdiff(x[:4], y[:4]) <= TOL and abs(x[4] - y[4]) <= 1e-9
    for y in b[1:]:
        assert np.array_equal(b[0][0], y[0]) and np.array_equal(b[0][2], y[2]) and b[0][4] == y[4]


def test_average_rccl_single_rank_equals_manual_protocol(ctx, ml100k):
    f = folds(*ml100k)[3]
    u, i, r, nu, ni = f.iu, f.ii, f.r, f.nu, f.ni
    k = 40
    rng = np.random.default_rng(11)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    sh = _shards(u, i, r, nu, ni, 1)
    ref = _plans(ctx, sh, k, P0, Q0, 3, mode=rsgpu.EXCHANGE_AVERAGE)
    _manual(ref, sh, nu, epochs=3)
    got = _plans(ctx, sh, k, P0, Q0, 3, mode=rsgpu.EXCHANGE_AVERAGE)
    got[0].join(rsgpu.comm_unique_id(), 0, 1, 3)
    got[0].epochs_sharded(3)
    got[0].leave()
    a, b = ref[0].download(), got[0].download()
    for pl in ref + got:
        pl.close()
    assert _maxdiff(a[:4], b[:4]) <= TOL and abs(a[4] - b[4]) <= 1e-9


def test_one_librccl_mapped(ctx):
    """Exactly one librccl is mapped into the process and the library runs against it."""
    ver, path = rsgpu.comm_info()
    maps = open("/proc/self/maps").read().split("\n")
    libs = {ln.split()[-1] for ln in maps if "librccl" in ln and ln.split()[-1].startswith("/")}
    assert len(libs) == 1, libs
    assert os.path.realpath(path) == os.path.realpath(libs.pop()) and ver > 0


def test_group_lowers_the_shift_and_destroy_restores_it(ctx, ml100k):
    """a group runs at its shards' smallest fixed-point shift (Q rows move between them as words); a
    star-scale shard (2^-24) grouped with a 1-100 one (2^-20) runs at 2^-20 and gets its own 2^-24 back when the
    group is destroyed, and then trains on its own (finite, the guard not redoing)."""
    f = folds(*ml100k)[0]
    n = 30000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    k = 16
    rng = np.random.default_rng(5)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    lo = i < ni // 2
    stars = ctx.svd_plan(rsgpu.Ratings(u[lo], i[lo], r[lo], nu, ni), k)
    wide = ctx.svd_plan(rsgpu.Ratings(u[~lo], i[~lo], 20.0 * r[~lo], nu, ni), k)
    assert (stars.fixed_point(), wide.fixed_point()) == (24, 20)
    for pl in (stars, wide):
        pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
    g = rsgpu.SvdGroup([stars, wide], n_blocks=2)
    assert (stars.fixed_point(), wide.fixed_point()) == (20, 20)
    g.close()
    assert (stars.fixed_point(), wide.fixed_point()) == (24, 20)
    stars.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
    stars.epochs(2)
    P, Q, bu, bi, gb = stars.download()
    assert np.isfinite(P).all() and np.isfinite(Q).all() and stars.refits() == 0
    stars.close()
    wide.close()
