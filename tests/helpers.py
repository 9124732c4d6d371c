"""Shared test helpers: TrainSet/KFold host logic restated with the oracle's id mapping."""
import numpy as np

import oracle as O


class Fold:
    """One KFold split (data.go:49-70) turned into a TrainSet (data.go:131-154)."""

    def __init__(self, U, I, R, tr, te):
        self.iu, self.ii, self.nu, self.ni = O.trainset_ids(U[tr], I[tr])
        self.r = R[tr]
        umap = dict(zip(U[tr].tolist(), self.iu.tolist()))
        imap = dict(zip(I[tr].tolist(), self.ii.tolist()))
        self.tu = np.array([umap.get(x, -1) for x in U[te].tolist()], np.int32)
        self.ti = np.array([imap.get(x, -1) for x in I[te].tolist()], np.int32)
        self.te_r = R[te]


def folds(U, I, R, k=5, seed=0):
    perm = np.random.default_rng(seed).permutation(len(R))
    return [Fold(U, I, R, tr, te) for tr, te in O.kfold_indices(len(R), k, perm)]


def rmse(pred, r):
    return float(np.sqrt(np.mean((pred - r) ** 2)))


def mae(pred, r):
    return float(np.mean(np.abs(pred - r)))
