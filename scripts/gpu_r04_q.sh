#!/bin/bash
# Round 4: claim-queue order inside a tile (0 key order, 1 single-rating runs last, 2 longest runs first,
# 3 shortest first) on the bench shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export REF=0
for q in 0 1 2 3; do
  RSGPU_X_QORDER=$q bash scripts/gpu_step.sh q_$q.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
done
RSGPU_FIT_TRACE=1 RSGPU_TILE_TRACE=1 bash scripts/gpu_step.sh q_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
