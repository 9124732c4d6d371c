"""Host model of the RS_EXCHANGE_QDELTA merge rules (csrc/multi.hip epochs_qdelta) -- test infrastructure,
restating the library's rules in numpy for tests/test_multi.py (gloo ranks) and tests/test_multi_gpu.py
(the in-process group, one wave per shard).

Per rank, the items' rows are [q_i | b_i] (k + 1 columns).  After every block a rank merges a set X of rows --
every item at a full merge (after every cold_every-th block), the hot items otherwise: its own weighted moves
w_i (row - Q0) replace the raw ones at once, together with the correction still pending from the row's
previous merge (that merge's sum over the ranks minus the rank's own moves); Q0 = the row afterwards.  The
merge's own moves are summed over the ranks (the all-reduce), and each rank's pending correction for X becomes
sum - own.  After the call's last merge (a full one) every rank adds its pending corrections, and all ranks
hold the same rows.  GlobalBias folds merge m's partials after block m + 1 (or at the end).
"""
import numpy as np

HOT_RATINGS = 4.0  # sgd_plan.hpp qdelta_hot default: ratings per rank and block that make an item hot
COLD_EVERY = 2     # sgd_plan.hpp qdelta_cold_every default
CURVATURE = 0.25   # sgd_plan.hpp qdelta_curv default: the factor columns' contraction a = 1 - lr x this


def cold_every(merges):
    """multi.hip qdelta_cold_every: the largest divisor of merges up to COLD_EVERY."""
    for f in range(min(COLD_EVERY, max(1, merges)), 1, -1):
        if merges % f == 0:
            return f
    return 1


def hot_items(cnt, c, merges):
    """Items rated on several ranks with at least HOT_RATINGS ratings per rank and block (none when every merge
    is a full one)."""
    return (c > 1) & (cnt / (np.maximum(c, 1) * merges) >= HOT_RATINGS) & (cold_every(merges) > 1)


def weights(cnt, c, lr, merges, hot, curv=None, k=None):
    """kappa / c per item (rsgpu.h RS_EXCHANGE_QDELTA), n_i over a hot item's block or a cold item's cold_every
    blocks.  With k: an (items, k + 1) array, the factor columns' weights at a = 1 - lr x curv (default CURVATURE)
    and the bias column's at a = 1 - lr (multi.hip epochs_qdelta); without: one weight per item at a = 1 - lr."""
    per = np.where(hot, merges, max(1, merges // cold_every(merges))).astype(np.float64)
    m = (c > 1) & (cnt > 0)
    n = cnt[m] / c[m] / per[m]

    def kc(a):
        w = np.ones(len(cnt))
        w[m] = (1.0 - a ** (c[m] * n)) / (1.0 - a ** n) / c[m]
        return w
    lr32 = float(np.float32(lr))
    wb = kc(1.0 - lr32)
    if k is None:
        return wb
    wf = kc(max(1e-12, 1.0 - lr32 * (CURVATURE if curv is None else curv)))
    return np.concatenate([np.repeat(wf[:, None], k, 1), wb[:, None]], 1)


def merge_set(m, merges, hot):
    """(rows merged at merge m, full?)"""
    full = (m % merges) % cold_every(merges) == cold_every(merges) - 1
    return (np.ones_like(hot) if full else hot), full


class Rank:
    """One rank's merge state: the rows at their last merge (Q0) and the pending corrections."""

    def __init__(self, rows):
        self.q0 = rows.copy()
        self.pend = np.zeros_like(rows)
        self.own = np.zeros_like(rows)

    def merge(self, rows, X, w):
        """rows: the rank's [Q | b] after its block; returns them after the merge of the rows X (own moves)."""
        own = (w[:, None] if w.ndim == 1 else w) * (rows - self.q0)
        out = rows.copy()
        out[X] = self.q0[X] + own[X] + self.pend[X]
        self.pend[X] = 0.0
        self.q0[X] = out[X]
        self.own = np.where(X[:, None], own, 0.0)
        return out

    def settle(self, total, X):
        """The merge's all-reduced own moves came in: the rows X owe total - own at their next merge."""
        self.pend[X] = (total - self.own)[X]

    def flush(self, rows):
        out = rows + self.pend
        self.pend[:] = 0.0
        return out
