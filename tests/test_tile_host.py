"""Host side of the tile schedule (rs_tile_schedule_host: no device needed): every rating is visited
exactly once for any waves / workgroups / user blocks, including Zipf-hot items whose runs are cut
over all waves (the case that once dealt a run to no stream), item shards with few ratings per user,
and k up to 510 (LDS-bound tiles)."""
import numpy as np
import pytest

import rsgpu


def _csr(users, items, vals, nu):
    order = np.lexsort((items, users))
    rowptr = np.concatenate([[0], np.cumsum(np.bincount(users, minlength=nu))]).astype(np.int64)
    return rowptr, items[order].astype(np.int32), vals[order].astype(np.float32)


@pytest.mark.parametrize("k,waves,wg,blocks", [(100, 16, 256, 1), (100, 16, 64, 3), (256, 8, 256, 1),
                                               (20, 1, 1, 1), (510, 16, 256, 2), (64, 4, 7, 5)])
def test_schedule_visits_every_rating_once(k, waves, wg, blocks):
    rng = np.random.default_rng(k + waves)
    nu, ni = 3000, 800
    deg = rng.integers(1, 120, nu)
    users = np.repeat(np.arange(nu), deg)
    items = (rng.zipf(1.4, len(users)) - 1) % ni  # a very hot head: runs cut over all waves
    keep = np.unique(users.astype(np.int64) * ni + items, return_index=True)[1]
    users, items = users[keep], items[keep]
    rowptr, cols, vals = _csr(users, items, rng.integers(1, 6, len(users)).astype(float), nu)
    ms, nt, pos = rsgpu.tile_schedule_host(nu, ni, rowptr, cols, vals, k, workgroups=wg, waves=waves,
                                           n_blocks=blocks, want_pos=True)
    assert nt >= 1 and np.array_equal(np.sort(pos), np.arange(len(cols)))


def test_item_shard_shape():
    """configs[4]'s shape at small scale: the 1/8 item shard of the generator (about 13 ratings per
    user over many items), k = 256."""
    s = rsgpu.Synth(200_000, 20_000, mean_deg=100.0, seed=20250826, item_lo=0, item_hi=2_500, n_threads=4)
    ms, nt, pos = rsgpu.tile_schedule_host(200_000, 20_000, s.rowptr, s.cols, s.vals, 256, want_pos=True)
    n = s.nnz
    s.close()
    assert np.array_equal(np.sort(pos), np.arange(n))


def test_svdpp_variant_is_rejected():
    """svdpp != 0 selected the SVD++ tile schedule, removed in round 3 (it diverged across
    workgroups): the call fails loudly instead of building a schedule nothing runs."""
    rowptr = np.array([0, 2], np.int64)
    cols = np.array([0, 1], np.int32)
    vals = np.array([3.0, 4.0], np.float32)
    nt, ms = rsgpu._i32(0), rsgpu._dbl(0)
    rc = rsgpu.lib().rs_tile_schedule_host(1, 2, rsgpu._ptr(rowptr), rsgpu._ptr(cols), rsgpu._ptr(vals), 8,
                                           1, 1, 1, 1, None, None, None, rsgpu.C.byref(nt), rsgpu.C.byref(ms))
    assert rc == rsgpu.RS_ERR_UNSUPPORTED
