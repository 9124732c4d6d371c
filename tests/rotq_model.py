"""Host model of the ROTATE_Q exchange (csrc/multi.hip epochs_rotate with RS_EXCHANGE_ROTATE_Q, the one
rs_svd_fit_multi picks at configs[4]) -- test infrastructure, restating the library's rules in numpy:

* ranks hold user ranges; the items are cut into nb = N x pieces blocks of near-equal ratings
  (user_block_bounds over the item counts of all ranks);
* hot items (multi.hip shard_setup): share = count x nb / total above hot_share (when a stratum holds
  at least min_stratum ratings) -> copies = min(nb, ceil(share / hot_share)), natural block = the
  block holding the item; rating (u, item) of a hot item goes to block (nat + j (nb // copies)) % nb with
  j = mix32(u x 0x9E3779B97F4A7C15) % copies (sgd_tile.hip build_tile_strata), and trains that block's
  copy row n_items + b H + h of Q, seeded from the item's row at the call start;
* an epoch is N sub-epochs; in sub-epoch s rank g trains the strata (its users x item blocks of rank-block
  (g + s) mod N) and sends those Q rows, plus their copies, to rank g - 1 (rs_rotation_step);
* after the N sub-epochs the copies' moves since the last merge (copy - the item row, which holds the last
  merged value) are summed (each rank over the blocks it holds again, then over the ranks) and the item row
  and every copy take last + w x sum, with RS_HOT_SCALED's w = kappa / c (multi.hip: n = count / c,
  kappa = (1 - (1 - lr)^(c n)) / (1 - (1 - lr)^n));
* GlobalBias: a work-local copy per stratum, the partials n (gb_w - gb) summed over every stratum and rank
  and folded once per epoch (gb += sum / total);
* after the call the item rank-blocks and the ranks' P ranges are broadcast.

A stratum's epoch is the oracle's sequential SGD (svd.go:93-129, or_svd_fit_works) over its ratings in an
order the caller supplies (user-CSR order in the CPU tests; a GPU plan's exported tile order in
tests/test_multi_gpu.py).
"""
import numpy as np

import oracle as O

M64 = (1 << 64) - 1


def mix32(x):
    """sgd_tile.hip mix32 (splitmix64's finaliser, bits 16..47)."""
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return ((x ^ (x >> 31)) >> 16) & 0xFFFFFFFF


def block_bounds(keys, n, blocks):
    """user_block_bounds over rows counted by `keys`: bound b = first row whose ratings start at or past
    b / blocks of them."""
    cum = np.concatenate([[0], np.cumsum(np.bincount(keys, minlength=n))])
    return np.array([np.searchsorted(cum, cum[-1] * b // blocks, side="left") for b in range(blocks)] + [n])


class Layout:
    """Item blocks, hot items and every rating's stratum / Q row (identical on every rank: global counts)."""

    def __init__(self, u, i, n_items, n_ranks, pieces, hot_share=0.02, min_stratum=1 << 17, lr=0.005):
        self.ni, self.N, self.h = n_items, n_ranks, pieces
        self.nb = n_ranks * pieces
        self.ib = block_bounds(i, n_items, self.nb)
        tot = np.bincount(i, minlength=n_items).astype(np.float64)
        total = float(len(i))
        self.hot, self.meta, self.count = [], [], []
        if hot_share > 0 and total / (n_ranks * self.nb) >= min_stratum and total > 0:
            for x in range(n_items):
                share = tot[x] * self.nb / total
                if share <= hot_share:
                    continue
                copies = int(min(self.nb, np.ceil(share / hot_share)))
                nat = int(np.searchsorted(self.ib, x, side="right") - 1)
                self.hot.append(x)
                self.meta.append((nat, copies))
                self.count.append(tot[x])
        self.H = len(self.hot)
        self.hidx = {x: h for h, x in enumerate(self.hot)}
        self.w = np.array([self._weight(h, lr) for h in range(self.H)])

    def _weight(self, h, lr):  # RS_HOT_SCALED
        cp = self.meta[h][1]
        n = self.count[h] / cp
        a = max(1e-12, 1.0 - float(np.float32(lr)))
        kappa = (1.0 - a ** (cp * n)) / max(1e-300, 1.0 - a ** n)
        return float(np.float32(kappa / cp))

    def block_of(self, u, item):
        h = self.hidx.get(int(item), -1)
        if h < 0:
            return int(np.searchsorted(self.ib, item, side="right") - 1)
        nat, copies = self.meta[h]
        j = mix32((int(u) * 0x9E3779B97F4A7C15) & M64) % copies
        return (nat + j * (self.nb // copies)) % self.nb

    def row_of(self, b, item):
        h = self.hidx.get(int(item), -1)
        return int(item) if h < 0 else self.ni + b * self.H + h

    def rows(self):
        return self.ni + self.nb * self.H

    def copy_used(self, b, h):  # multi.hip hot_copy_used
        nat, copies = self.meta[h]
        stride = self.nb // copies
        off = (b - nat + self.nb) % self.nb
        return off % stride == 0 and off // stride < copies

    def copy_row(self, b, h):
        return self.ni + b * self.H + h

    def seed(self, Q, bi):
        """Every copy takes its item's row (hot_seed_kernel)."""
        for b in range(self.nb):
            for h, x in enumerate(self.hot):
                Q[self.copy_row(b, h)] = Q[x]
                bi[self.copy_row(b, h)] = bi[x]

    def partial(self, Q, bi, b0, b1):
        """Summed moves of the copies of blocks [b0, b1) (hot_partial_kernel), columns k factors + bias."""
        out = np.zeros((self.H, Q.shape[1] + 1))
        for h, x in enumerate(self.hot):
            base = np.concatenate([Q[x], [bi[x]]])
            for b in range(b0, b1):
                if self.copy_used(b, h):
                    out[h] += np.concatenate([Q[self.copy_row(b, h)], [bi[self.copy_row(b, h)]]]) - base
        return out

    def write(self, Q, bi, moves, b0, b1):
        """Item row and the copies of blocks [b0, b1) take last + w x moves (hot_write_kernel)."""
        k = Q.shape[1]
        for h, x in enumerate(self.hot):
            v = np.concatenate([Q[x], [bi[x]]]) + self.w[h] * moves[h]
            Q[x], bi[x] = v[:k], v[k]
            for b in range(b0, b1):
                Q[self.copy_row(b, h)], bi[self.copy_row(b, h)] = v[:k], v[k]


def stratum_csr(layout, u, i, r, b):
    """Ratings of (these users, item block b) in user-CSR order (data order per user), Q rows as trained."""
    blk = np.array([layout.block_of(a, x) for a, x in zip(u, i)], np.int64)
    m = blk == b
    order = np.argsort(u[m], kind="stable")
    su, si, sr = u[m][order], i[m][order], r[m][order]
    rows = np.array([layout.row_of(b, x) for x in si], np.int32)
    return su.astype(np.int32), rows, sr


def train_works(P, Q, bu, bi, gb, works):
    """Sequential SGD over works [(users, Q rows, ratings), ...] with a work-local GlobalBias each;
    returns the state and the works' GlobalBias partial sum n (gb_w - gb)."""
    works = [w for w in works if len(w[2])]
    if not works:
        return P, Q, bu, bi, 0.0
    U = np.concatenate([w[0] for w in works]).astype(np.int32)
    I = np.concatenate([w[1] for w in works]).astype(np.int32)
    R = np.concatenate([w[2] for w in works])
    off = np.concatenate([[0], np.cumsum([len(w[2]) for w in works])]).astype(np.int64)
    # svd_fit_works folds the works' partials into its gb (gb + sum / len): recover the raw sum
    P, Q, bu, bi, g = O.svd_fit_works(U, I, R, off, P, Q, bu, bi, gb, epochs=1)
    return P, Q, bu, bi, (g - gb) * len(R)


def sequential(layout, u, i, r, nu, P0, Q0, gb0, epochs, user_ranges, stratum_works):
    """Single process: per epoch the strata in rotation order (sub-epoch, then rank), the hot merge, the
    GlobalBias fold.  stratum_works(rank, b) -> [(users, Q rows, ratings), ...] in visit order."""
    N, h = layout.N, layout.h
    P, bu = P0.copy(), np.zeros(nu)
    Q = np.zeros((layout.rows(), Q0.shape[1]))
    Q[:layout.ni] = Q0
    bi = np.zeros(layout.rows())
    layout.seed(Q, bi)
    gb = gb0
    for _ in range(epochs):
        part = 0.0
        for st in range(N):
            for g in range(N):
                rb = (g + st) % N
                for j in range(h):
                    P, Q, bu, bi, p = train_works(P, Q, bu, bi, gb, stratum_works(g, rb * h + j))
                    part += p
        if layout.H:
            moves = sum(layout.partial(Q, bi, g * h, g * h + h) for g in range(N))
            layout.write(Q, bi, moves, 0, layout.nb)  # (every rank writes the same value: one write here)
        gb += part / len(r)
    return P, Q[:layout.ni], bu, bi[:layout.ni], gb
