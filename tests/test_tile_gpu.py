"""GPU tests of the tile schedule (RS_SGD_WB_TILE, the FAST default; csrc/sgd_tile.hip) of K1, the SGD
epoch of core/svd.go:92-130.

Exactness: with one wave per workgroup the tile kernel is the sequential SGD of svd.go:93-129 in the
schedule's own visit order (rs_svd_plan_tile_order) with a work-local GlobalBias per (tile, wave)
stream folded after the epoch (the smoothed fold of the single-GPU epoch: sgd_tile.hip header).  The oracle
restates exactly that (or_svd_fit_works2 with compose = 2, the reference's per-rating update and aliasing Q1
over explicit work segments), so:
  * one workgroup, one wave, real ML-100K data (users and items shared everywhere): equal to 1e-5;
  * several workgroups, one wave each, on race-free input (private items): equal to 1e-5.
The P rows live in LDS as int32 fixed point (2^-24) and Q as int32 fixed point between calls, inside the
1e-5 tolerance.  With 16 waves per tile the waves of a tile share P rows through integer LDS atomics
(no update lost, Hogwild timing), so the default schedule is checked by RMSE parity (P2, in
test_svd_gpu.py and below) and by size-independent properties.
"""
import numpy as np
import pytest

import oracle as O
import rsgpu
from helpers import folds, rmse
from rsgpu import synth

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _maxdiff(a, b):
    return max(float(np.max(np.abs(np.asarray(x) - np.asarray(y)))) for x, y in zip(a, b))


def _csr(u, i, r, nu):
    rowptr, items, rr = O.csr_by(u, nu, i, r)
    users = np.repeat(np.arange(nu, dtype=np.int32), np.diff(rowptr))
    return users, np.asarray(items, np.int32), np.asarray(rr, np.float64)


def _oracle_in_tile_order(plan, u, i, r, nu, P0, Q0, bu0, bi0, gb0, epochs):
    cu, ci, cr = _csr(u, i, r, nu)
    pos, off = plan.tile_order()
    assert np.array_equal(np.sort(pos), np.arange(len(r)))  # every rating exactly once
    return O.svd_fit_works(cu[pos], ci[pos], cr[pos], off, P0, Q0, bu0, bi0, gb0, epochs=epochs, compose=2)


@pytest.mark.parametrize("k,epochs,target,run_cap", [(20, 1, 3000, 0), (100, 1, 5000, 0),
                                                     (100, 3, 2000, 3), (256, 2, 20000, 0)])
def test_one_wave_is_sequential_sgd(ctx, ml100k, k, epochs, target, run_cap):
    """One workgroup of one wave: the kernel is svd.go:93-129 in the tile order (1e-5), on real
    ML-100K fold-1 data (a 20k-rating prefix), several tiles, runs of hot items cut at run_cap."""
    f = folds(*ml100k)[0]
    n = 20000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    rng = np.random.default_rng(k + epochs)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    bu0, bi0 = rng.normal(0, 0.1, nu), rng.normal(0, 0.1, ni)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    plan.set_tiles(workgroups=1, waves=1, target=target, run_cap=run_cap)
    plan.upload(P0, Q0, bu0, bi0, 3.2)
    plan.epochs(epochs)
    got = plan.download()
    ref = _oracle_in_tile_order(plan, u, i, r, nu, P0, Q0, bu0, bi0, 3.2, epochs)
    plan.close()
    assert _maxdiff(ref[:4], got[:4]) <= TOL and abs(ref[4] - got[4]) <= TOL


@pytest.mark.parametrize("claim,ring", [(4, 3), (8, 3), (8, 2), (4, 2)])
def test_one_wave_claims_any_ring(ctx, ml100k, claim, ring):
    """Claimed runs with every ring the API accepts (a ring of 3 runs on 4- or 8-run claims is taken
    as the 4-deep ring on chunks of 8, which the ring divides): one wave equals the oracle in the
    exported order (1e-5).  A ring that did not divide the chunk trained the next chunk's runs twice
    and added q deltas to the wrong rows (advisor round 4)."""
    f = folds(*ml100k)[0]
    n = 12000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    k = 40
    rng = np.random.default_rng(claim * 10 + ring)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    bu0, bi0 = rng.normal(0, 0.1, nu), rng.normal(0, 0.1, ni)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    plan.set_tile_claim(claim)
    plan.set_tiles(workgroups=1, waves=1, target=2500, ring=ring)
    plan.upload(P0, Q0, bu0, bi0, 3.4)
    plan.epochs(2)
    got = plan.download()
    ref = _oracle_in_tile_order(plan, u, i, r, nu, P0, Q0, bu0, bi0, 3.4, 2)
    plan.close()
    assert _maxdiff(ref[:4], got[:4]) <= TOL and abs(ref[4] - got[4]) <= TOL


@pytest.mark.parametrize("k,kconc", [(40, 1.0), (100, 0.25)])
def test_damped_runs_one_wave_equal_oracle(ctx, ml100k, k, kconc):
    """The hot-run damping (svd_epoch_tile_kernel<..., DAMP = true>) pinned: the test hook
    rs_svd_plan_set_damp_concurrency makes one wave -- whose runs never overlap -- take the damped kernel with
    R = deg x kconc runs in flight, and the result equals the oracle's restatement of the rule
    (or_svd_fit_works_damped: each run's move scaled by min(1, 1 / (R f)) on the factors and on b_i) to 1e-5,
    on real ML-100K ratings; the damping moved the item rows away from the undamped epoch."""
    f = folds(*ml100k)[0]
    n = 20000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    rng = np.random.default_rng(k)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    bu0, bi0 = rng.normal(0, 0.1, nu), rng.normal(0, 0.1, ni)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    plan.set_tiles(workgroups=1, waves=1, target=4000)  # one wave: runs uncut (no automatic cap)
    plan.set_damp_concurrency(kconc)
    plan.upload(P0, Q0, bu0, bi0, 3.2)
    plan.epochs(2)
    got = plan.download()
    cu, ci, cr = _csr(u, i, r, nu)
    pos, off = plan.tile_order()
    deg = np.bincount(i, minlength=ni).astype(np.int32)
    ref = O.svd_fit_works_damped(cu[pos], ci[pos], cr[pos], off, deg, float(np.float32(kconc)), P0, Q0, bu0, bi0, 3.2,
                                 epochs=2, compose=2)
    plain = O.svd_fit_works(cu[pos], ci[pos], cr[pos], off, P0, Q0, bu0, bi0, 3.2, epochs=2, compose=2)
    plan.set_damp_concurrency(0)
    plan.close()
    assert _maxdiff(ref[:4], got[:4]) <= TOL and abs(ref[4] - got[4]) <= TOL
    assert _maxdiff(ref[1:2], plain[1:2]) > 1e-3 and _maxdiff(ref[3:4], plain[3:4]) > 1e-3  # the rule acted


@pytest.mark.parametrize("k", [20, 100])
def test_cold_store_one_wave_equals_oracle(ctx, ml100k, k):
    """Cold runs (rs_svd_plan_set_cold_store: here every item cold) end in write-through stores of the new row; with
    one wave no other run of the item is in flight, so the store is the atomic's sum and the epoch stays the
    sequential SGD in tile order (1e-5)."""
    f = folds(*ml100k)[3]
    n = 20000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    rng = np.random.default_rng(k + 1)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    bu0, bi0 = rng.normal(0, 0.1, nu), rng.normal(0, 0.1, ni)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    plan.set_tiles(workgroups=1, waves=1, target=3000)
    plan.set_cold_store(1e9)
    plan.upload(P0, Q0, bu0, bi0, 3.3)
    plan.epochs(2)
    got = plan.download()
    ref = _oracle_in_tile_order(plan, u, i, r, nu, P0, Q0, bu0, bi0, 3.3, 2)
    plan.close()
    assert _maxdiff(ref[:4], got[:4]) <= TOL and abs(ref[4] - got[4]) <= TOL


def test_gb_fold_switch_one_wave(ctx, ml100k):
    """rs_svd_plan_set_gb_fold: with the mean fold (GB_FOLD_MEAN, rounds 1-5 and the multi-GPU exchanges) one wave
    equals the oracle's mean-of-moves fold (or_svd_fit_works2 compose 0), with the smoothed default compose 2; the
    factors are the same sequential SGD either way within an epoch, the folds differ in GlobalBias."""
    f = folds(*ml100k)[1]
    n = 20000
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    rng = np.random.default_rng(11)
    P0, Q0 = rng.normal(0, 0.1, (nu, 32)), rng.normal(0, 0.1, (ni, 32))
    bu0, bi0 = rng.normal(0, 0.1, nu), rng.normal(0, 0.1, ni)
    got = {}
    for fold in (rsgpu.GB_FOLD_MEAN, rsgpu.GB_FOLD_SMOOTH):
        plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), 32)
        plan.set_tiles(workgroups=1, waves=1, target=3000)
        plan.set_gb_fold(fold)
        plan.upload(P0, Q0, bu0, bi0, 3.3)
        plan.epochs(2)
        got[fold] = plan.download()
        cu, ci, cr = _csr(u, i, r, nu)
        pos, off = plan.tile_order()
        ref = O.svd_fit_works(cu[pos], ci[pos], cr[pos], off, P0, Q0, bu0, bi0, 3.3, epochs=2,
                              compose=0 if fold == rsgpu.GB_FOLD_MEAN else 2)
        plan.close()
        assert _maxdiff(ref[:4], got[fold][:4]) <= TOL and abs(ref[4] - got[fold][4]) <= TOL, fold
    assert got[rsgpu.GB_FOLD_MEAN][4] != got[rsgpu.GB_FOLD_SMOOTH][4]


def _private_items(n_users=300, per_user=25, seed=4):
    rng = np.random.default_rng(seed)
    deg = rng.integers(1, 2 * per_user, n_users)
    users = np.repeat(np.arange(n_users), deg)
    items = np.arange(len(users))
    perm = rng.permutation(len(users))
    r = rng.integers(1, 6, len(users)).astype(float)
    return users[perm], items[perm], r[perm], n_users, len(users)


@pytest.mark.parametrize("k", [8, 63, 64, 100, 127, 300, 510])
@pytest.mark.parametrize("wg", [3, 0])
def test_workgroups_race_free(ctx, k, wg):
    """Several workgroups (3, or one per CU), one wave each, many tiles per workgroup, private items
    (no two tiles share a row): equal to the restatement over the same work items (1e-5)."""
    u, i, r, nu, ni = _private_items(seed=k)
    rng = np.random.default_rng(k)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    bu0, bi0 = rng.normal(0, 0.1, nu), rng.normal(0, 0.1, ni)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    plan.set_tiles(workgroups=wg, waves=1, target=300)
    plan.upload(P0, Q0, bu0, bi0, 3.0)
    plan.epochs(2)
    got = plan.download()
    ref = _oracle_in_tile_order(plan, u, i, r, nu, P0, Q0, bu0, bi0, 3.0, 2)
    plan.close()
    assert _maxdiff(ref[:4], got[:4]) <= TOL and abs(ref[4] - got[4]) <= TOL


def test_delta_mode_equals_direct(ctx, ml100k):
    """The item-sharded multi-GPU path with one shard holding every item (user weights 1):
    epoch_delta + apply_delta gives the epoch of plain epochs() (one wave: deterministic) -- the same factors
    and biases; GlobalBias is folded by the mean of the streams' moves in delta mode and smoothed in the plain
    single-GPU epoch, each equal to the oracle's fold of that name in the exported tile order."""
    import torch
    f = folds(*ml100k)[1]
    u, i, r, nu, ni = f.iu, f.ii, f.r, f.nu, f.ni
    k = 32
    rng = np.random.default_rng(2)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    plans = []
    for _ in range(2):
        pl = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
        pl.set_tiles(workgroups=1, waves=1)
        pl.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.5)
        plans.append(pl)
    plans[0].epochs(1)
    plans[1].set_user_weights(np.ones(nu))
    dP = torch.zeros((nu, plans[1].ld), dtype=torch.float32, device="cuda")
    g = torch.zeros(1, dtype=torch.float64, device="cuda")
    plans[1].epoch_delta_t(dP, g, 0.005, 0.02)
    torch.cuda.synchronize()
    plans[1].apply_delta_t(dP, g, 1.0 / len(r))
    torch.cuda.synchronize()
    a, b = plans[0].download(), plans[1].download()
    cu, ci, cr = _csr(u, i, r, nu)
    pos, off = plans[0].tile_order()
    smooth = O.svd_fit_works(cu[pos], ci[pos], cr[pos], off, P0, Q0, np.zeros(nu), np.zeros(ni), 3.5, compose=2)
    mean = O.svd_fit_works(cu[pos], ci[pos], cr[pos], off, P0, Q0, np.zeros(nu), np.zeros(ni), 3.5, compose=0)
    for pl in plans:
        pl.close()
    assert _maxdiff(a[:4], b[:4]) <= TOL
    assert abs(a[4] - smooth[4]) <= TOL and abs(b[4] - mean[4]) <= TOL


def test_heavy_user_cut_into_pieces_trains(ctx):
    """A user with more ratings than one tile's LDS holds (12,000 at k = 100) is cut into pieces over
    several tiles and merged by count-weighted average: the model stays finite and fits."""
    rng = np.random.default_rng(3)
    nu, ni = 400, 20000
    heavy = rng.choice(ni, 12000, replace=False)
    users = [np.zeros(12000, np.int64)]
    items = [heavy]
    for x in range(1, nu):
        d = int(rng.integers(5, 60))
        users.append(np.full(d, x))
        items.append(rng.choice(ni, d, replace=False))
    u, i = np.concatenate(users), np.concatenate(items)
    p_u, q_i = rng.normal(0, 0.5, (nu, 4)), rng.normal(0, 0.5, (ni, 4))
    r = np.clip(np.rint(3.5 + np.sum(p_u[u] * q_i[i], 1)), 1, 5)
    k = 100
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), float(np.mean(r)))
    e0 = plan.evaluate(u, i, r)[0]
    plan.epochs(10)
    P, Q, bu, bi, gb = plan.download()
    e1 = plan.evaluate(u, i, r)[0]
    plan.close()
    assert all(np.all(np.isfinite(x)) for x in (P, Q, bu, bi)) and np.isfinite(gb)
    assert e1 < e0 - 0.05, (e0, e1)


@pytest.mark.parametrize("wg,waves,run_cap", [(0, 16, 0), (64, 16, 0), (0, 8, 16)])
def test_rmse_parity_ml100k_configs(ctx, ml100k, wg, waves, run_cap):
    """P2 for tile configurations other than the default: 5-fold ML-100K (k=100, 20 epochs) within
    0.003 of the reference visit order (core/base_test.go:34-36 data)."""
    k = 100
    ref_r, gpu_r = [], []
    for f in folds(*ml100k):
        rng = np.random.default_rng(7)
        P0, Q0 = rng.normal(0, 0.1, (f.nu, k)), rng.normal(0, 0.1, (f.ni, k))
        ref_r.append(rmse(O.svd_predict(f.tu, f.ti, *O.svd_fit(f.iu, f.ii, f.r, P0, Q0)), f.te_r))
        rowptr, items, rr = O.csr_by(f.iu, f.nu, f.ii, f.r)
        gb0 = O.gb_warm_start(rowptr, items, rr, np.zeros(f.nu), np.zeros(f.ni))
        plan = ctx.svd_plan(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), k)
        plan.set_tiles(workgroups=wg, waves=waves, run_cap=run_cap)
        plan.upload(P0, Q0, np.zeros(f.nu), np.zeros(f.ni), gb0)
        plan.epochs(20)
        ou = np.where(f.tu >= 0, f.tu, -1)
        gpu_r.append(rmse(O.svd_predict(ou, f.ti, *plan.download()), f.te_r))
        plan.close()
    assert abs(np.mean(gpu_r) - np.mean(ref_r)) <= 0.003, (np.mean(gpu_r), np.mean(ref_r))


def test_mode_switch_keeps_model(ctx):
    """Tile epochs, then the hybrid schedule, then tiles again on the same plan: the item rows (and
    the hybrid's hot-item copies) follow, and the model keeps training."""
    u, i, r, nu, ni = synth.small_like(600, 300, 30000, seed=8)
    k = 64
    rng = np.random.default_rng(1)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    plan.upload(rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k)), np.zeros(nu), np.zeros(ni),
                float(np.mean(r)))
    errs = [plan.evaluate(u, i, r)[0]]
    for mode in (rsgpu.WB_TILE, rsgpu.WB_ATOMIC, rsgpu.WB_TILE):
        plan.set_mode(mode)
        before = plan.download()
        plan.epochs(3)
        errs.append(plan.evaluate(u, i, r)[0])
        assert np.isfinite(errs[-1])
        assert not np.array_equal(before[1], plan.download()[1])
    plan.close()
    assert errs[-1] < errs[0] - 0.1 and all(b < a for a, b in zip(errs, errs[1:])), errs


@pytest.mark.parametrize("mode", ["tile", "hybrid"])
def test_out_of_range_q_is_reported(ctx, mode):
    """Q is int32 fixed point (2^-24) during a call and integer atomics wrap: an item factor at or
    beyond 128 (or non-finite) is flagged and download reports RS_ERR_NUMERIC once (values returned)."""
    u, i, r, nu, ni = synth.small_like(200, 100, 4000, seed=3)
    k = 16
    rng = np.random.default_rng(0)
    Q0 = rng.normal(0, 0.1, (ni, k))
    Q0[7, 3] = 300.0
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    if mode == "hybrid":
        plan.set_mode(rsgpu.WB_ATOMIC)
    plan.upload(rng.normal(0, 0.1, (nu, k)), Q0, np.zeros(nu), np.zeros(ni), 3.0)
    plan.epochs(1)
    with pytest.raises(rsgpu.RsError) as e:
        plan.download()
    assert e.value.code == rsgpu.RS_ERR_NUMERIC
    plan.download()  # reported once
    plan.close()
