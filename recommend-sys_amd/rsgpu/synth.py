"""Deterministic synthetic rating sets of the BASELINE.json shapes.

The MovieLens-1M/20M files are not in the reference snapshot (they are downloaded at run time by
core/data.go:270-284, which must never run here), so the bench and the large parity tests use
synthetic sets of the same shape:

  ml1m_like()  U=6,040, I=3,706, nnz=1,000,209; >=20 ratings per user; user degree lognormal with
               mean 165.6 (capped at ML-1M's 2,314); item popularity Zipf(s=1.0) over permuted ids;
               no duplicate (u, i); integer ratings 1-5 from a planted biased rank-16 model,
               quantile-mapped to the published ML-1M histogram; emitted in shuffled order.
  ml20m_like() U=138,493, I=26,744, nnz=20,000,263; half-star ratings 0.5-5.0.

Everything is a pure function of the seed (numpy PCG64).
"""
from __future__ import annotations

import numpy as np

ML1M_HIST = (56174, 107557, 261197, 348971, 226310)  # ratings 1..5, sum = 1,000,209


def _degrees(rng, n_users, nnz, min_deg, max_deg, sigma=1.0):
    mean_extra = nnz / n_users - min_deg
    mu = np.log(mean_extra) - sigma * sigma / 2
    d = min_deg + rng.lognormal(mu, sigma, n_users)
    d = np.minimum(d, max_deg)
    # rescale the excess over min_deg so the total is exactly nnz, respecting the cap
    for _ in range(50):
        excess = d - min_deg
        target = nnz - min_deg * n_users
        d = np.minimum(min_deg + excess * (target / excess.sum()), max_deg)
        if abs(d.sum() - nnz) < 1:
            break
    deg = np.floor(d).astype(np.int64)
    short = nnz - deg.sum()
    order = np.argsort(-(d - deg), kind="stable")
    i = 0
    while short > 0:
        if deg[order[i % n_users]] < max_deg:
            deg[order[i % n_users]] += 1
            short -= 1
        i += 1
    return deg


def _sample_items(rng, deg, n_items, s=1.0, chunk=256):
    """Per user, deg distinct items drawn with Zipf(s) popularity over permuted ids (Gumbel top-k)."""
    ranks = np.arange(1, n_items + 1, dtype=np.float64)
    logp = -s * np.log(ranks)
    item_of_rank = rng.permutation(n_items)
    users, items = [], []
    n_users = len(deg)
    for b in range(0, n_users, chunk):
        e = min(n_users, b + chunk)
        keys = logp[None, :] + rng.gumbel(size=(e - b, n_items))
        order = np.argsort(-keys, axis=1)
        for x in range(b, e):
            sel = order[x - b, :deg[x]]
            users.append(np.full(deg[x], x, np.int64))
            items.append(item_of_rank[sel])
    return np.concatenate(users), np.concatenate(items)


def _planted_ratings(rng, users, items, n_users, n_items, hist, rank=16):
    xu = rng.normal(0, 1, (n_users, rank)) / np.sqrt(rank)
    yi = rng.normal(0, 1, (n_items, rank))
    bu = rng.normal(0, 0.5, n_users)
    bi = rng.normal(0, 0.5, n_items)
    score = bu[users] + bi[items] + np.einsum("nk,nk->n", xu[users], yi[items])
    score += rng.normal(0, 0.5, len(users))
    order = np.argsort(score, kind="stable")
    r = np.empty(len(users), np.float64)
    cut = np.cumsum((0,) + tuple(hist))
    for lvl in range(len(hist)):
        r[order[cut[lvl]:cut[lvl + 1]]] = lvl + 1
    return r


def ml1m_like(seed: int = 20250824):
    """Returns (users, items, ratings) in shuffled order; ids are already 0-based inner ids."""
    rng = np.random.default_rng(seed)
    n_users, n_items, nnz = 6040, 3706, sum(ML1M_HIST)
    deg = _degrees(rng, n_users, nnz, 20, 2314)
    users, items = _sample_items(rng, deg, n_items)
    ratings = _planted_ratings(rng, users, items, n_users, n_items, ML1M_HIST)
    perm = rng.permutation(nnz)
    return users[perm].astype(np.int32), items[perm].astype(np.int32), ratings[perm], n_users, n_items


def small_like(n_users, n_items, nnz, seed=1, min_deg=5, hist=None):
    """Scaled-down ML-1M-like set for parity tests."""
    rng = np.random.default_rng(seed)
    max_deg = min(n_items, max(min_deg + 1, nnz // 4))
    deg = _degrees(rng, n_users, nnz, min_deg, max_deg)
    users, items = _sample_items(rng, deg, n_items)
    if hist is None:
        frac = np.array(ML1M_HIST, np.float64) / sum(ML1M_HIST)
        h = np.floor(frac * nnz).astype(np.int64)
        h[-2] += nnz - h.sum()
        hist = tuple(int(x) for x in h)
    ratings = _planted_ratings(rng, users, items, n_users, n_items, hist)
    perm = rng.permutation(nnz)
    return users[perm].astype(np.int32), items[perm].astype(np.int32), ratings[perm], n_users, n_items


# Published ML-20M half-star histogram (0.5 .. 5.0), recalled from the MovieLens-20M README era
# statistics -- the file is not in the reference snapshot, so treat these counts as approximate.
ML20M_HIST = (239125, 680732, 279252, 1430997, 883398, 4291193, 2200156, 5561926, 1534824, 2898660)


def _zipf_items(rng, n, n_items, s, item_of_rank):
    ranks = np.arange(1, n_items + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** -s)
    cdf /= cdf[-1]
    return item_of_rank[np.searchsorted(cdf, rng.random(n), side="right").clip(0, n_items - 1)]


def ml20m_like(seed: int = 20250825, scale: float = 1.0):
    """U=138,493, I=26,744, nnz=20,000,263 (x scale on users and nnz); >=20 ratings per user;
    Zipf(1.0) item popularity over permuted ids; no duplicate (u, i); half-star ratings from user and
    item biases plus noise, quantile-mapped to ML20M_HIST.  Returns (users, items, ratings, U, I)."""
    rng = np.random.default_rng(seed)
    n_users = int(round(138493 * scale))
    n_items = 26744
    nnz = int(round(sum(ML20M_HIST) * scale))
    deg = _degrees(rng, n_users, nnz, 20, 9254)
    item_of_rank = rng.permutation(n_items)
    users = np.repeat(np.arange(n_users, dtype=np.int64), deg)
    items = _zipf_items(rng, nnz, n_items, 1.0, item_of_rank).astype(np.int64)
    for _ in range(30):  # resolve duplicate (u, i): redraw the later copies (uniformly after 10 rounds)
        key = users * n_items + items
        order = np.argsort(key, kind="stable")
        dup = np.zeros(nnz, bool)
        dup[order[1:]] = key[order[1:]] == key[order[:-1]]
        nd = int(dup.sum())
        if nd == 0:
            break
        items[dup] = (_zipf_items(rng, nd, n_items, 1.0, item_of_rank) if _ < 10
                      else rng.integers(0, n_items, nd))
    hist = np.array(ML20M_HIST, np.float64)
    hist = np.floor(hist / hist.sum() * nnz).astype(np.int64)
    hist[-4] += nnz - hist.sum()
    score = rng.normal(0, 0.5, n_users)[users] + rng.normal(0, 0.5, n_items)[items] + rng.normal(0, 0.7, nnz)
    order = np.argsort(score, kind="stable")
    r = np.empty(nnz)
    cut = np.concatenate([[0], np.cumsum(hist)])
    for lvl in range(len(hist)):
        r[order[cut[lvl]:cut[lvl + 1]]] = 0.5 * (lvl + 1)
    perm = rng.permutation(nnz)
    return users[perm].astype(np.int32), items[perm].astype(np.int32), r[perm], n_users, n_items
