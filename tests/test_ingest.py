"""TrainSet construction on the host (rs_trainset_ids / rs_csr_build / rs_global_mean)
against the oracle's sequential restatement of core/data.go:131-216, and the synthetic CSR generator
(rs_synth_*) used for BASELINE configs[4].  No GPU: these entry points are host C++."""
import numpy as np
import pytest

import oracle as O
import rsgpu


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_trainset_ids_match_first_appearance_ml100k(ml100k, threads):
    U, I, R = ml100k
    perm = np.random.default_rng(5).permutation(len(R))  # a shuffled TrainSet order
    iu_ref, ii_ref, nu, ni = O.trainset_ids(U[perm], I[perm])
    iu, inv_u = rsgpu.trainset_ids(U[perm], threads)
    ii, inv_i = rsgpu.trainset_ids(I[perm], threads)
    assert np.array_equal(iu, iu_ref) and np.array_equal(ii, ii_ref)
    assert len(inv_u) == nu and len(inv_i) == ni
    assert np.array_equal(inv_u[iu], U[perm]) and np.array_equal(inv_i[ii], I[perm])


def test_trainset_ids_edge_cases():
    for outer in ([], [7], [5, 5, 5], [-3, 2**62, -3, 0, 2**62, 1], list(range(1000, 0, -1))):
        o = np.array(outer, np.int64)
        inner, inv = rsgpu.trainset_ids(o, 4)
        if len(o):
            ref, _, n, _ = O.trainset_ids(o, o)
            assert np.array_equal(inner, ref) and len(inv) == n
        else:
            assert len(inner) == 0 and len(inv) == 0


def test_trainset_ids_many_collisions_random():
    rng = np.random.default_rng(2)
    o = rng.integers(-50_000, 50_000, 400_000).astype(np.int64) * 1_000_003
    inner, inv = rsgpu.trainset_ids(o, 8)
    ref, _, n, _ = O.trainset_ids(o, o)
    assert np.array_equal(inner, ref) and len(inv) == n


@pytest.mark.parametrize("threads", [1, 5, 16])
def test_csr_build_is_stable_grouping(ml100k, threads):
    U, I, R = ml100k
    iu, ii, nu, ni = O.trainset_ids(U, I)
    rowptr, cols, vals = rsgpu.csr_build(iu, ii, R, nu, threads)
    rp_ref, c_ref, v_ref = O.csr_by(iu, nu, ii, R)
    assert np.array_equal(rowptr, rp_ref) and np.array_equal(cols, c_ref)
    assert np.array_equal(vals, v_ref.astype(np.float32))
    # item-major lists (ItemRatings, data.go:202-216) with the same routine
    rowptr, cols, _ = rsgpu.csr_build(ii, iu, R, ni, threads)
    rp_ref, c_ref = O.csr_by(ii, ni, iu)
    assert np.array_equal(rowptr, rp_ref) and np.array_equal(cols, c_ref)


def test_csr_build_empty_rows_and_bad_ids():
    rows = np.array([3, 0, 3, 3], np.int32)
    cols = np.array([1, 2, 0, 1], np.int32)
    rowptr, c, v = rsgpu.csr_build(rows, cols, np.arange(4.0), 6, 2)
    assert rowptr.tolist() == [0, 1, 1, 1, 4, 4, 4]
    assert c.tolist() == [2, 1, 0, 1] and v.tolist() == [1.0, 0.0, 2.0, 3.0]
    with pytest.raises(rsgpu.RsError):
        rsgpu.csr_build(np.array([0, 6], np.int32), np.array([0, 0], np.int32), np.zeros(2), 6, 1)


def test_global_mean(ml100k):
    R = ml100k[2]
    assert rsgpu.global_mean(R, 1) == rsgpu.global_mean(R, 8)
    assert abs(rsgpu.global_mean(R, 4) - np.mean(R)) <= 1e-14
    big = np.random.default_rng(0).random(3_000_001) * 5
    assert abs(rsgpu.global_mean(big, 7) - np.mean(big)) <= 1e-12


def test_synth_deterministic_and_shards_are_filters():
    kw = dict(mean_deg=40.0, sigma=1.0, zipf_s=0.9, seed=11)
    a = rsgpu.Synth(3000, 2000, n_threads=1, **kw)
    b = rsgpu.Synth(3000, 2000, n_threads=7, **kw)
    assert np.array_equal(a.rowptr, b.rowptr) and np.array_equal(a.cols, b.cols)
    assert np.array_equal(a.vals, b.vals)
    assert a.nnz == a.rowptr[-1] and 0.7 * 40 * 3000 < a.nnz < 1.3 * 40 * 3000
    assert set(np.unique(a.vals)) <= {1.0, 2.0, 3.0, 4.0, 5.0}
    # no repeated (u, i) within a user
    for u in range(0, 3000, 97):
        row = a.cols[a.rowptr[u]:a.rowptr[u + 1]]
        assert len(np.unique(row)) == len(row)
    # Zipf head: the most popular item holds far more than the uniform share
    cnt = np.bincount(a.cols, minlength=2000)
    assert cnt.max() > 20 * a.nnz / 2000
    # shard [500, 1200) = the full set's ratings of those items in the same order
    s = rsgpu.Synth(3000, 2000, item_lo=500, item_hi=1200, n_threads=3, **kw)
    users = np.repeat(np.arange(3000), np.diff(a.rowptr))
    keep = (a.cols >= 500) & (a.cols < 1200)
    assert np.array_equal(s.cols, a.cols[keep]) and np.array_equal(s.vals, a.vals[keep])
    assert np.array_equal(np.diff(s.rowptr), np.bincount(users[keep], minlength=3000))
    for x in (a, b, s):
        x.close()


def test_csr_build_concurrent_callers_share_the_worker_pool():
    """The host passes run on a pool of persistent threads (ingest.cpp) that serves one job at a time; a
    caller that finds it busy (another host thread -- CrossValidate's goroutines, the shards of a
    multi-GPU fit) spawns its own threads.  Six Python threads (ctypes releases the GIL) building CSRs
    at once, several times over, each equal to the single-threaded build; an out-of-range id raises in
    its own caller only."""
    import threading

    rng = np.random.default_rng(5)
    sets = []
    for s in range(6):
        n, nr = 200000 + 1000 * s, 3000 + s
        rows, cols = rng.integers(0, nr, n), rng.integers(0, 5000, n)
        vals = rng.integers(1, 6, n).astype(float)
        sets.append((rows, cols, vals, nr, rsgpu.csr_build(rows, cols, vals, nr, n_threads=1)))
    errors = []

    def work(x):
        rows, cols, vals, nr, ref = sets[x]
        try:
            for _ in range(4):
                got = rsgpu.csr_build(rows, cols, vals, nr, n_threads=8)
                for a, b in zip(got, ref):
                    assert np.array_equal(a, b)
            bad = rows.copy()
            bad[len(bad) // 2] = nr  # out of range
            with pytest.raises(rsgpu.RsError):
                rsgpu.csr_build(bad, cols, vals, nr, n_threads=8)
        except BaseException as e:  # noqa: BLE001 -- reported below
            errors.append(e)

    th = [threading.Thread(target=work, args=(x,)) for x in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
