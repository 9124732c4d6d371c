#!/bin/bash
# Round 4: tile refinement cost-model sweep (run cost per distinct item, iteration cap) on the bench shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export REF=0
for rc in 3 2 4 6 1; do
  RSGPU_X_RUNCOST=$rc bash scripts/gpu_step.sh p_rc$rc.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
done
RSGPU_X_REFIT=16 bash scripts/gpu_step.sh p_it16.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
RSGPU_X_RUNCOST=4 RSGPU_X_REFIT=16 bash scripts/gpu_step.sh p_rc4_it16.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
