#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export REF=0
bash scripts/gpu_step.sh o_ref.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
RSGPU_TILE_NO_REFINE=1 bash scripts/gpu_step.sh o_noref.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
bash scripts/gpu_step.sh o_ref2.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
RSGPU_TILE_NO_REFINE=1 bash scripts/gpu_step.sh o_noref2.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
