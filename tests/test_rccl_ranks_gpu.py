"""The multi-GPU exchanges with real RCCL collectives between processes, on the one-GPU box
(tests/rccl_ranks.py: one NCCL_HOSTID per rank process, RCCL's network transport over loopback).

Every case runs its shards twice from the same start -- as N rank processes joined through
rs_svd_plan_join (RCCL all-reduce / send / recv / broadcast on the library's comm stream, overlapped with the
next block's kernel) and through the in-process exchange of one process (rs_svd_group on plans of one device,
the path the other multi-GPU tests pin against the oracle and the host models) -- with one wave per shard, so
both are deterministic.  Where the collective's arithmetic is order-free the two must agree bit for bit:
- every exchange at N = 2 (a sum of two terms is one rounding, whatever the order: the fp16 QDELTA wire, the
  AVERAGE float deltas and the GlobalBias partials included);
- the int32 QDELTA wire and the ROTATE_Q transfers at N = 3 (integer sums; rows moved, not summed) -- up to
  the GlobalBias partials' fp64 sum, whose order RCCL picks: within 1e-9 there.
Every rank must also end with the same replicated state as rank 0 (P, Q, b_u, b_i, GlobalBias).
Reference loop: core/svd.go:92-130 (north_star: item sharding with an RCCL all-reduce).
"""
import numpy as np
import pytest

import rccl_ranks as RR

pytestmark = pytest.mark.gpu


def _maxdiff(a, b):
    return max(float(np.max(np.abs(np.asarray(x) - np.asarray(y)))) if np.size(x) else 0.0 for x, y in zip(a, b))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case,n", [("qdelta32", 2), ("qdelta16", 2), ("rotate_q", 2), ("rotate", 2),
                                    ("average", 2), ("qdelta32", 3), ("rotate_q", 3), ("qdelta16", 3)])
def test_rccl_ranks_equal_in_process_exchange(ctx, tmp_path, case, n):
    """Real RCCL ranks (one process each, one GPU, tests/rccl_ranks.py) against the in-process group of the same
    shards: bitwise at 2 ranks for every exchange. At 3 ranks the exact wires agree to 1e-6 (the f64 GlobalBias
    partials are summed in RCCL's order); the fp16 QDELTA wire agrees to 2e-4 (7.6e-5 measured after 2 epochs;
    GlobalBias 2.2e-7,
    profiles/r06/): the in-process sum rounds to fp16 at every hop in ring order, but which rank starts each element's
    chain follows RCCL's run-time channel and chunk sizes, which the emulation does not know (at 2 ranks the order
    does not matter: fp16 addition commutes). Every rank still holds the same bits (the replica check)."""
    got, log = RR.launch(case, n, str(tmp_path))
    ref = RR.group(ctx, case, n)
    mode = RR.CASES[case][0]
    replicated = (0, 1, 2, 3) if mode in (RR.rsgpu.EXCHANGE_QDELTA, RR.rsgpu.EXCHANGE_ROTATE_Q) else (0, 2)
    for r in range(1, n):  # every rank holds the same replicated state
        assert all(np.array_equal(got[0][x], got[r][x]) for x in replicated), (case, n, r)
        assert got[0][4] == got[r][4]
    for r in range(n):  # and each rank's model is the in-process group's shard r
        if n == 2:
            bad = [x for x in range(4) if not np.array_equal(got[r][x], ref[r][x])]
            assert not bad and got[r][4] == ref[r][4], (case, r, bad, _maxdiff(got[r][:4], ref[r][:4]), got[r][4] - ref[r][4], log)
        else:  # (the GlobalBias partials are f64 sums in RCCL's order; the fp16 wire: see below)
            tol, tol_gb = (2e-4, 2e-6) if case == "qdelta16" else (1e-6, 1e-9)
            assert _maxdiff(got[r][:4], ref[r][:4]) <= tol and abs(got[r][4] - ref[r][4]) <= tol_gb, \
                (case, r, _maxdiff(got[r][:4], ref[r][:4]), got[r][4] - ref[r][4])


@pytest.mark.timeout(300)
def test_rccl_ranks_consistency_check_fails_everywhere(tmp_path):
    """One rank's replica perturbed by a word before the check (RS_FAULT_DIVERGE on rank 1 of 3): the RCCL max /
    min comparison makes the sharded call return RS_ERR_NUMERIC on every rank."""
    got, log = RR.launch("qdelta_diverge", 3, str(tmp_path))
    assert got == [RR.rsgpu.RS_ERR_NUMERIC] * 3, (got, log)
