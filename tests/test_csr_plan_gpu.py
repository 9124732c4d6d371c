"""GPU tests of the CSR plan entry point (rs_svd_plan_create_csr), the device factor init
(rs_svd_plan_init_normal) and the synthetic-CSR -> plan path of BASELINE configs[4].

A plan built from rs_csr_build's CSR must behave exactly like one built from the COO TrainSet:
checked bit-for-bit on race-free input (every user rates private items, so the FAST epoch is
deterministic) and against the restatement of the FAST schedule (or_svd_fit_chunked)."""
import numpy as np
import pytest

import oracle as O
import rsgpu

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _disjoint_input(n_users=200, per_user=30, seed=3):
    rng = np.random.default_rng(seed)
    deg = rng.integers(1, 2 * per_user, n_users)
    users = np.repeat(np.arange(n_users), deg)
    items = np.arange(len(users))
    perm = rng.permutation(len(users))
    users, items = users[perm], items[perm]
    r = rng.integers(1, 6, len(users)).astype(float)
    return users, items, r, n_users, len(users)


@pytest.mark.parametrize("k", [20, 100, 256])
def test_csr_plan_equals_coo_plan_race_free(ctx, k):
    u, i, r, nu, ni = _disjoint_input()
    rng = np.random.default_rng(k)
    P0, Q0 = rng.normal(0, 0.1, (nu, k)), rng.normal(0, 0.1, (ni, k))
    rowptr, cols, vals = rsgpu.csr_build(u, i, r, nu)
    outs = []
    for plan in (ctx.svd_plan(rsgpu.Ratings(u, i, r, nu, ni), k),
                 ctx.svd_plan_csr(nu, ni, rowptr, cols, vals, k)):
        plan.set_mode(rsgpu.WB_ATOMIC)  # the restatement's work items are user rows
        plan.upload(P0, Q0, np.zeros(nu), np.zeros(ni), 3.0)
        plan.epochs(3)
        outs.append(plan.download())
        plan.close()
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    rp, it, rr = O.csr_by(u, nu, i, r)
    ref = O.svd_fit_chunked(rp, it, rr, P0, Q0, 1 << 30, gb=3.0, epochs=3, warm=False)
    assert max(float(np.max(np.abs(x - y))) for x, y in zip(ref[:4], outs[1][:4])) <= TOL


def test_csr_plan_rejects_bad_csr(ctx):
    rowptr = np.array([0, 2, 1], np.int64)  # not monotone
    with pytest.raises(rsgpu.RsError):
        ctx.svd_plan_csr(2, 3, rowptr, np.zeros(2, np.int32), np.ones(2, np.float32), 8)
    with pytest.raises(rsgpu.RsError):  # item id out of range
        ctx.svd_plan_csr(1, 3, np.array([0, 2], np.int64), np.array([0, 3], np.int32),
                         np.ones(2, np.float32), 8)


def test_init_normal_distribution_and_warm_start(ctx):
    s = rsgpu.Synth(4000, 1500, mean_deg=30.0, seed=5, n_threads=4)
    k = 50
    plan = ctx.svd_plan_csr(4000, 1500, s.rowptr, s.cols, s.vals, k)
    plan.init_normal(0.0, 0.1, seed=9)
    P, Q, bu, bi, gb = plan.download()
    assert np.all(bu == 0) and np.all(bi == 0)
    assert abs(gb - float(np.mean(s.vals, dtype=np.float64))) <= 1e-9
    f = np.concatenate([P.ravel(), Q.ravel()])
    assert abs(f.mean()) < 2e-3 and abs(f.std() - 0.1) < 2e-3
    assert not np.array_equal(P[0], P[1]) and not np.array_equal(P[0], Q[0])
    plan.init_normal(0.0, 0.1, seed=9)  # deterministic in the seed
    assert np.array_equal(plan.download()[0], P)
    plan.close()
    s.close()


def test_synth_plan_trains_and_holds_out(ctx):
    """configs[4]-shaped path at small scale: generator CSR -> plan -> device init -> FAST epochs;
    the held-out RMSE (device evaluate) falls well below the init's and stays finite."""
    nu, ni, k = 20000, 4000, 64
    s = rsgpu.Synth(nu, ni, mean_deg=60.0, seed=20250826, n_threads=8)
    deg = np.diff(s.rowptr)
    users = np.repeat(np.arange(nu, dtype=np.int32), deg)
    hold = np.zeros(s.nnz, bool)
    hold[np.random.default_rng(0).random(s.nnz) < 0.05] = True
    keep = ~hold
    tr_rowptr = np.concatenate([[0], np.cumsum(np.bincount(users[keep], minlength=nu))]).astype(np.int64)
    plan = ctx.svd_plan_csr(nu, ni, tr_rowptr, s.cols[keep], s.vals[keep], k)
    plan.init_normal(0.0, 0.1, seed=1)
    rmse0, _ = plan.evaluate(users[hold], s.cols[hold], s.vals[hold])
    plan.epochs(10, 0.005, 0.02)
    rmse, mae = plan.evaluate(users[hold], s.cols[hold], s.vals[hold])
    plan.close()
    s.close()
    assert np.isfinite(rmse) and rmse < rmse0 - 0.05 and mae < rmse
