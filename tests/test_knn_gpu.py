"""GPU parity tests of K4 (int8-MFMA Cosine/MSD) and K5 (merge-order Pearson) through the C-ABI.

P3: Sims bitwise equal to the oracle's restatement of core/knn.go:143-217 + core/sim.go (NaN
pattern included), and therefore identical top-K neighbour lists under (sim desc, index asc).
"""
import json
import math
import os

import numpy as np
import pytest

import oracle as O
import rsgpu

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
KINDS = {"Cosine": rsgpu.SIM_COSINE, "MSD": rsgpu.SIM_MSD, "Pearson": rsgpu.SIM_PEARSON}


def bitwise_equal(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64)) or \
        (np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)]))


def topk(S, k=40):
    out = []
    for row in S:
        idx = np.nonzero(~np.isnan(row))[0]
        order = np.lexsort((idx, -row[idx]))
        out.append(idx[order][:k])
    return out


def test_sim_pair_known_answers(ctx):
    """core/sim_test.go:10-59 on the device: the exact values, bit for bit."""
    kat = json.load(open(os.path.join(HERE, "golden", "sim_kat.json")))
    a, b = kat["a"], kat["b"]
    for case in kat["cases"]:
        v = ctx.sim_pair(KINDS[case["sim"]], a["ids"], a["ratings"], b["ids"], b["ratings"])
        assert v == case["exact"], (case["sim"], v)
        assert abs(v - case["expect"]) <= kat["epsilon"]
    assert math.isnan(ctx.sim_pair(rsgpu.SIM_COSINE, [1], [2.0], [2], [3.0]))


@pytest.fixture(scope="module")
def ml100k_lists(ml100k):
    U, I, R = ml100k
    iu, ii, nu, ni = O.trainset_ids(U, I)
    return iu, ii, R, nu, ni


@pytest.mark.parametrize("user_based", [False, True])
@pytest.mark.parametrize("kind", [rsgpu.SIM_COSINE, rsgpu.SIM_MSD, rsgpu.SIM_PEARSON])
def test_knn_sims_ml100k_bitwise(ctx, ml100k_lists, kind, user_based):
    """Full ML-100K (item- and user-based): every Sims entry bitwise equal, NaN pattern too."""
    iu, ii, R, nu, ni = ml100k_lists
    left, right, nl, nr = (iu, ii, nu, ni) if user_based else (ii, iu, ni, nu)
    rowptr, ids, rr = O.csr_by(left, nl, right, R)
    ref = O.knn_sims(kind, rowptr, ids, rr)
    got = ctx.knn_sims(kind, rowptr, ids, rr, nr)
    assert np.array_equal(np.isnan(ref), np.isnan(got))
    m = ~np.isnan(ref)
    assert np.array_equal(ref[m].view(np.uint64), got[m].view(np.uint64))
    for x, y in zip(topk(ref)[:200], topk(got)[:200]):
        assert np.array_equal(x, y)


def test_knn_merge_path_matches_mfma(ctx, ml100k_lists, monkeypatch):
    iu, ii, R, nu, ni = ml100k_lists
    rowptr, ids, rr = O.csr_by(ii, ni, iu, R)
    a = ctx.knn_sims(rsgpu.SIM_MSD, rowptr, ids, rr, nu)
    monkeypatch.setenv("RSGPU_KNN_NO_MFMA", "1")
    b = ctx.knn_sims(rsgpu.SIM_MSD, rowptr, ids, rr, nu)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    m = ~np.isnan(a)
    assert np.array_equal(a[m].view(np.uint64), b[m].view(np.uint64))


def _random_lists(L, Rn, density, values, seed):
    rng = np.random.default_rng(seed)
    mask = rng.random((L, Rn)) < density
    rows, cols = np.nonzero(mask)
    perm = rng.permutation(len(rows))  # data order inside a row is arbitrary (sorts() fixes it)
    rows, cols = rows[perm], cols[perm]
    r = rng.choice(values, len(rows))
    return O.csr_by(rows, L, cols, r)


@pytest.mark.parametrize("kind", [rsgpu.SIM_COSINE, rsgpu.SIM_MSD, rsgpu.SIM_PEARSON])
@pytest.mark.parametrize("L,Rn,values", [
    (300, 1000, np.arange(1, 11) / 2.0),          # half stars (ML-20M): scale 2 on the MFMA path
    (129, 70, np.arange(0, 6, dtype=float)),       # zero ratings: rated but x = 0 (M carries them)
    (1, 5, np.array([3.0])),                        # single row: only the NaN diagonal
    (257, 300, np.array([1.3, 2.7, 4.1])),          # not x/s representable: merge path
    (200, 64, np.arange(-5, 6, dtype=float)),       # negative ratings, |x| <= 11
])
def test_knn_sims_random_bitwise(ctx, kind, L, Rn, values):
    rowptr, ids, rr = _random_lists(L, Rn, 0.05, values, seed=L + Rn)
    ref = O.knn_sims(kind, rowptr, ids, rr)
    got = ctx.knn_sims(kind, rowptr, ids, rr, Rn)
    assert np.array_equal(np.isnan(ref), np.isnan(got))
    m = ~np.isnan(ref)
    assert np.array_equal(ref[m].view(np.uint64), got[m].view(np.uint64))


@pytest.mark.parametrize("n_parts", [2, 3, 8])
@pytest.mark.parametrize("kind,values", [(rsgpu.SIM_COSINE, np.arange(1, 11) / 2.0),
                                         (rsgpu.SIM_MSD, np.arange(1, 6, dtype=float)),
                                         (rsgpu.SIM_PEARSON, np.arange(1, 6, dtype=float))])
def test_knn_sims_parts_assemble_bitwise(ctx, n_parts, kind, values):
    """the parts of rs_knn_sims_part (one per GPU in production; run here one after the
    other on one device into one buffer) write disjoint entries whose union is rs_knn_sims, bitwise."""
    L, Rn = 700, 900  # 6 row blocks of 128 (last ragged): every part owns >= 0 blocks
    rowptr, ids, rr = _random_lists(L, Rn, 0.04, values, seed=n_parts + kind)
    full = ctx.knn_sims(kind, rowptr, ids, rr, Rn)
    out = np.full((L, L), 12345.0)
    written = np.zeros((L, L), np.int32)
    for part in range(n_parts):
        mark = np.full((L, L), 12345.0)
        ctx.knn_sims(kind, rowptr, ids, rr, Rn, part=part, n_parts=n_parts, out=mark)
        wrote = mark != 12345.0
        written += wrote
        out[wrote] = mark[wrote]
    assert written.max() == 1 and written.min() == 1  # disjoint and complete
    assert np.array_equal(np.isnan(full), np.isnan(out))
    m = ~np.isnan(full)
    assert np.array_equal(full[m].view(np.uint64), out[m].view(np.uint64))


def test_knn_empty_rows(ctx):
    rowptr = np.array([0, 0, 2, 2, 3], np.int64)
    ids = np.array([1, 0, 1], np.int32)
    rr = np.array([4.0, 5.0, 3.0])
    for kind in KINDS.values():
        ref = O.knn_sims(kind, rowptr, ids, rr)
        got = ctx.knn_sims(kind, rowptr, ids, rr, 2)
        assert np.array_equal(np.isnan(ref), np.isnan(got))
        m = ~np.isnan(ref)
        assert np.array_equal(ref[m], got[m])


def test_knn_bad_arguments(ctx):
    with pytest.raises(rsgpu.RsError):
        ctx.knn_sims(7, [0, 1], [0], [1.0], 1)
    with pytest.raises(rsgpu.RsError):
        ctx.knn_sims(rsgpu.SIM_COSINE, [0, 1], [5], [1.0], 2)


def test_baseline_fit_bitwise(ctx, ml100k):
    """core/base.go:135-163 BaseLine.Fit (used by KNNBaseLine, knn.go:179-187): float64 serial
    chain in the reference order -> bitwise equal to the restatement."""
    from helpers import folds
    f = folds(*ml100k)[0]
    ref = O.baseline_fit(f.iu, f.ii, f.r, f.nu, f.ni)
    got = ctx.baseline_fit(rsgpu.Ratings(f.iu, f.ii, f.r, f.nu, f.ni))
    assert np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1]) and ref[2] == got[2]


@pytest.mark.parametrize("kind", [rsgpu.SIM_COSINE, rsgpu.SIM_PEARSON])
@pytest.mark.parametrize("user_based", [True, False])
def test_knn_plan_predict_bitwise(ctx, ml100k, kind, user_based):
    """KNN.Predict (knn.go:75-141) on the device-resident Sims equals the
    restatement bit for bit for all four KNN types, on fold 0 of ML-100K (train -> test pairs,
    unknown ids included), with the reference defaults k=40, mink=1 and a tight k=3 / mink=5."""
    from helpers import folds
    f = folds(*ml100k)[0]
    u, i, r = f.iu, f.ii, f.r
    left_key, right_key = (u, i) if user_based else (i, u)
    nl, nr = (f.nu, f.ni) if user_based else (f.ni, f.nu)
    lrp, lids, lr = O.csr_by(left_key, nl, right_key, r)
    rrp, rids, rr = O.csr_by(right_key, nr, left_key, r)
    plan = ctx.knn_plan(kind, lrp, lids, lr, nr)
    S = plan.sims()
    deg = np.diff(lrp).astype(float)
    means = np.add.reduceat(lr, lrp[:-1]) / np.maximum(deg, 1)      # data.go:222-235
    dev = (lr - np.repeat(means, np.diff(lrp))) ** 2
    stds = np.sqrt(np.add.reduceat(dev, lrp[:-1]) / np.maximum(deg, 1)) + 1e-5  # knn.go:167-177
    bu, bi, _ = O.baseline_fit(u, i, r, f.nu, f.ni)
    bias = bu if user_based else bi
    ql, qr = (f.tu, f.ti) if user_based else (f.ti, f.tu)
    gm = float(np.mean(r))
    differ = 0
    for stable in (False, True):  # knn.go:107-108's sort.Sort order (default), then RS_TIE_STABLE
        plan.set_tie_order(rsgpu.TIE_STABLE if stable else rsgpu.TIE_GO_SORT)
        for t, name in enumerate(["basic", "centered", "zscore", "baseline"]):
            for k, mink in [(40, 1), (3, 5)]:
                got = plan.predict(name, rrp, rids, rr, ql, qr, gm, means, stds, bias, k=k, min_k=mink)
                ref = O.knn_predict(t, S, rrp, rids, rr, means, stds, bias, gm, k, mink, ql, qr, stable=stable)
                assert bitwise_equal(got, ref), (name, k, mink, stable)
                if not stable:
                    alt = O.knn_predict(t, S, rrp, rids, rr, means, stds, bias, gm, k, mink, ql, qr, stable=True)
                    differ += int(np.count_nonzero(~np.isclose(alt, ref, rtol=0, atol=0)))
    plan.close()
    print(f"predictions whose value depends on the tie order: {differ}")


def test_knn_predict_go_order_long_rows(ctx):
    """Candidate rows longer than the kernel's LDS arrays (5000 > 4096: the per-block global scratch) and
    rows of exact ties (integer ratings, one co-rated item: Cosine 1.0 everywhere) through the Go-order
    kernel: bitwise the restatement of sort.Sort's order, for every KNN type."""
    rng = np.random.default_rng(21)
    nl, nr = 6000, 12  # user-based: left = users, right = items; item 0 rated by 5000 users
    users = [rng.choice(nl, 5000, replace=False)] + [rng.choice(nl, 300, replace=False) for _ in range(1, nr)]
    u = np.concatenate(users).astype(np.int32)
    i = np.concatenate([np.full(len(x), j) for j, x in enumerate(users)]).astype(np.int32)
    r = rng.integers(1, 6, len(u)).astype(float)
    lrp, lids, lr = O.csr_by(u, nl, i, r)
    rrp, rids, rr = O.csr_by(i, nr, u, r)
    plan = ctx.knn_plan(rsgpu.SIM_COSINE, lrp, lids, lr, nr)
    S = plan.sims()
    deg = np.diff(lrp).astype(float)
    means = np.add.reduceat(lr, lrp[:-1]) / np.maximum(deg, 1)
    stds = np.full(nl, 0.5)
    bias = rng.normal(0, 0.1, nl)
    ql = rng.integers(0, nl, 400).astype(np.int32)
    qr = rng.integers(0, nr, 400).astype(np.int32)
    qr[:100] = 0  # the 5000-candidate row
    for t, name in enumerate(["basic", "centered", "zscore", "baseline"]):
        got = plan.predict(name, rrp, rids, rr, ql, qr, 3.0, means, stds, bias, k=40, min_k=1)
        ref = O.knn_predict(t, S, rrp, rids, rr, means, stds, bias, 3.0, 40, 1, ql, qr)
        assert bitwise_equal(got, ref), name
    plan.close()


@pytest.mark.parametrize("kind", [rsgpu.SIM_COSINE, rsgpu.SIM_MSD, rsgpu.DEV_SLOPE_ONE])
def test_knn_streamed_download_multi_group(ctx, kind, monkeypatch):
    """rs_knn_sims streams the Sims to the host while later column groups still compute (one launch
    per 2048-row super-tile column group, rows copied as their groups complete).  With L = 4700
    (3 groups, a ragged last block) the streamed result equals, bit for bit: the device plan's
    one-launch Sims, the eight-wave tilings (RSGPU_KNN_PIPE=3, 4, 5 and 6: the default with and without
    the LEAN operand forms), the same call with the round-1 K loop (RSGPU_KNN_PIPE=0) and without streaming
    (RSGPU_KNN_NO_STREAM=1), and the oracle's restatement (knn.go:190-216) on rows from every group."""
    rng = np.random.default_rng(11)
    L, R, nnz = 4700, 900, 120_000
    left = rng.integers(0, L, nnz)
    right = rng.integers(0, R, nnz)
    key = np.unique(left.astype(np.int64) * R + right)  # no repeated (left, right) pair
    left, right = (key // R).astype(np.int32), (key % R).astype(np.int32)
    perm = rng.permutation(len(key))                     # rows arrive unsorted by id
    left, right = left[perm], right[perm]
    r = rng.integers(1, 11, len(key)) / 2.0              # half stars: the s = 2 int8 path
    rowptr, ids, rr = O.csr_by(left, L, right, r)
    S = ctx.knn_sims(kind, rowptr, ids, rr, R)
    plan = ctx.knn_plan(kind, rowptr, ids, rr, R)
    assert bitwise_equal(S, plan.sims())
    plan.close()
    for pipe in ("3", "4", "5", "6"):  # eight waves of 64 x 32 (two per SIMD): M in registers / staged / rotated loads (LEAN / not)
        monkeypatch.setenv("RSGPU_KNN_PIPE", pipe)
        assert bitwise_equal(S, ctx.knn_sims(kind, rowptr, ids, rr, R)), pipe
    monkeypatch.setenv("RSGPU_KNN_NO_STREAM", "1")
    monkeypatch.setenv("RSGPU_KNN_PIPE", "0")
    assert bitwise_equal(S, ctx.knn_sims(kind, rowptr, ids, rr, R))
    if kind == rsgpu.DEV_SLOPE_ONE:
        return  # the dev matrix is pinned against slope_one.go in test_slope_one_gpu.py
    srt = np.lexsort((ids, np.repeat(np.arange(L), np.diff(rowptr))))
    for a0 in (0, 2040, 4090, 4690):
        ref = O.knn_sims_rows(kind, rowptr, ids[srt], rr[srt], a0, min(L, a0 + 10))
        assert bitwise_equal(S[a0:a0 + 10], ref), a0
