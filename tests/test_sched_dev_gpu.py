"""The tile schedule built on the device (RS_TILE_RULE_FILL_DEVICE, csrc/sched_dev.hip) -- one-shot Fit's
schedule -- against the host build of the same rule (RS_TILE_RULE_FILL, build_tile_host):
byte-identical schedules (rs_svd_plan_schedule_digest over every array the kernel reads), on real ML-100K
data, hot-item sets whose runs are cut into pieces, repeated (user, item) ratings, empty users, several
workgroup / wave counts and k; the kernel on a device-built schedule is the sequential SGD of
core/svd.go:93-129 in the host's visit order with one wave (1e-5); where the rule does not apply (a user
above the LDS bound) the device build falls back to the LPT host build."""
import numpy as np
import pytest

import oracle as O
import rsgpu
from helpers import folds
from rsgpu import synth

pytestmark = pytest.mark.gpu


def _digests(ctx, R, k, wg=0, waves=16, run_cap=0, cold=None):
    plan = ctx.svd_plan(R, k)
    if wg or waves != 16 or run_cap:
        plan.set_tiles(workgroups=wg, waves=waves, run_cap=run_cap)
    if cold is not None:
        plan.set_cold_store(cold)
    plan.set_tile_rule(rsgpu.TILE_RULE_FILL)
    host = plan.schedule_digest()
    plan.set_tile_rule(rsgpu.TILE_RULE_FILL_DEVICE)
    assert plan.tile_rule() == rsgpu.TILE_RULE_FILL_DEVICE
    dev = plan.schedule_digest()
    plan.set_tile_rule(rsgpu.TILE_RULE_LPT)
    lpt = plan.schedule_digest()
    plan.close()
    return host, dev, lpt


def _hot_set(nu=3000, ni=500, n=120000, seed=5, dup=True, empty=True):
    rng = np.random.default_rng(seed)
    u = rng.integers(0, nu, n)
    if empty:
        u = u[u % 97 != 3]  # users with no ratings
    i = np.minimum(rng.zipf(1.3, len(u)) - 1, ni - 1)  # a Zipf head: runs cut into pieces
    r = rng.integers(1, 6, len(u)).astype(np.float64)
    if dup:  # repeated (user, item) pairs keep their COO order inside a run
        j = rng.integers(0, len(u), 2000)
        u, i, r = np.concatenate([u, u[j]]), np.concatenate([i, i[j]]), np.concatenate([r, r[j] + 0.5])
    p = rng.permutation(len(u))
    return rsgpu.Ratings(u[p].astype(np.int32), i[p].astype(np.int32), r[p], nu, ni)


@pytest.mark.parametrize("k,wg,waves,run_cap", [(100, 0, 16, 0), (20, 64, 16, 0), (256, 7, 8, 3), (64, 0, 4, 5)])
def test_device_schedule_equals_host_ml100k(ctx, ml100k, k, wg, waves, run_cap):
    f = folds(*ml100k)[0]
    host, dev, lpt = _digests(ctx, rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni), k, wg, waves, run_cap)
    assert host == dev
    assert lpt != dev  # (the default build is a different rule)


@pytest.mark.parametrize("cold", [0.0, 0.05, 1e9])
def test_device_schedule_equals_host_cold_runs(ctx, ml100k, cold):
    """The cold-run header bit (sgd_plan.hpp kRunCold: items below cold_degree's ratings, marked only where the mean
    item is that cold -- cold_degree_used) is set identically by the host and the device builds; the library's 0.05
    leaves ML-100K unmarked (its mean item is far from cold, as ML-1M's), 1e9 marks every run."""
    f = folds(*ml100k)[1]
    R = rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni)
    host, dev, _ = _digests(ctx, R, 64, cold=cold)
    base, _, _ = _digests(ctx, R, 64, cold=0.0)
    assert host == dev
    assert (host == base) == (cold != 1e9)


@pytest.mark.parametrize("k,wg,waves", [(100, 0, 16), (100, 33, 16), (256, 0, 2), (8, 5, 1)])
def test_device_schedule_equals_host_hot_dups_empty(ctx, k, wg, waves):
    host, dev, _ = _digests(ctx, _hot_set(seed=k + wg), k, wg, waves)
    assert host == dev


def test_device_schedule_equals_host_ml1m_shape(ctx):
    u, i, r, nu, ni = synth.ml1m_like(seed=11)
    host, dev, _ = _digests(ctx, rsgpu.Ratings(u, i, r, nu, ni), 100)
    assert host == dev


def test_one_shot_fit_builds_on_device(ctx):
    """rs_svd_fit (the Go Fit) on a shuffled COO: its cached schedule is the device rule and equals the host
    fill build of a plan over the same ratings; the fit trains (held-out RMSE falls, finite)."""
    u, i, r, nu, ni = synth.ml1m_like(seed=12)
    p = np.random.default_rng(0).permutation(len(r))
    hold = p[:20000]
    keep = np.sort(p[20000:])  # COO order inside each user kept, users interleaved
    R = rsgpu.Ratings(u[keep], i[keep], r[keep], nu, ni)
    rng = np.random.default_rng(1)
    P0, Q0 = rng.normal(0, 0.1, (nu, 100)), rng.normal(0, 0.1, (ni, 100))
    P, Q, bu, bi, gb = ctx.svd_fit(R, P0, Q0, n_epochs=10)
    digest, rule = ctx.fit_schedule_digest()
    assert rule == rsgpu.TILE_RULE_FILL_DEVICE
    plan = ctx.svd_plan(R, 100)
    plan.set_tile_rule(rsgpu.TILE_RULE_FILL)
    assert plan.schedule_digest() == digest
    plan.close()
    pred = O.svd_predict(u[hold], i[hold], P, Q, bu, bi, gb)
    e = float(np.sqrt(np.mean((pred - r[hold]) ** 2)))
    assert np.isfinite(P).all() and np.isfinite(Q).all() and e < 0.80, e


@pytest.mark.parametrize("epochs,target,run_cap", [(1, 3000, 0), (2, 2000, 3)])
def test_one_wave_on_device_schedule_is_sequential_sgd(ctx, ml100k, epochs, target, run_cap):
    """One workgroup of one wave on the device-built schedule: svd.go:93-129 in the visit order the host's
    fill build exports (rs_svd_plan_tile_order), to 1e-5."""
    f = folds(*ml100k)[0]
    n, k = 20000, 64
    u, i, r, nu, ni = f.iu[:n], f.ii[:n], f.r[:n], f.nu, f.ni
    rng = np.random.default_rng(epochs)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    bu0, bi0 = rng.normal(0, 0.1, nu), rng.normal(0, 0.1, ni)
    plan = ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k)
    plan.set_tiles(workgroups=1, waves=1, target=target, run_cap=run_cap)
    plan.set_tile_rule(rsgpu.TILE_RULE_FILL_DEVICE)
    assert plan.tile_rule() == rsgpu.TILE_RULE_FILL_DEVICE
    plan.upload(P0, Q0, bu0, bi0, 3.2)
    plan.epochs(epochs)
    got = plan.download()
    rowptr, items, rr = O.csr_by(u, nu, i, r)
    cu = np.repeat(np.arange(nu, dtype=np.int32), np.diff(rowptr))
    pos, off = plan.tile_order()
    ref = O.svd_fit_works(cu[pos], np.asarray(items, np.int32)[pos], np.asarray(rr, np.float64)[pos], off,
                          P0, Q0, bu0, bi0, 3.2, epochs=epochs, compose=2)
    plan.close()
    d = max(float(np.max(np.abs(np.asarray(a) - np.asarray(b)))) for a, b in zip(ref[:4], got[:4]))
    assert d <= 1e-5 and abs(ref[4] - got[4]) <= 1e-5


def test_device_build_falls_back_above_lds_bound(ctx):
    """k = 256: a user of 12000 ratings exceeds one tile's LDS (pieces needed): the device rule does not
    apply -- the build falls back to LPT and the host fill rule is RS_ERR_UNSUPPORTED."""
    rng = np.random.default_rng(3)
    u = np.concatenate([np.zeros(12000, np.int32), rng.integers(1, 500, 30000).astype(np.int32)])
    i = rng.integers(0, 20000, len(u)).astype(np.int32)
    R = rsgpu.Ratings(u, i, rng.integers(1, 6, len(u)).astype(np.float64), 500, 20000)
    plan = ctx.svd_plan(R, 256)
    plan.set_tile_rule(rsgpu.TILE_RULE_FILL_DEVICE)
    assert plan.tile_rule() == rsgpu.TILE_RULE_LPT
    with pytest.raises(rsgpu.RsError) as e:
        plan.set_tile_rule(rsgpu.TILE_RULE_FILL)
    assert e.value.code == -4
    plan.epochs(1)
    plan.download()
    plan.close()
