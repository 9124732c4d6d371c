#!/bin/bash
# Round 4, session b: claimed-run variants (ring 3, chunk 8), diagnostics of the claim kernel, bench line,
# FAST stability sweep at library defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export REF=0
bash scripts/gpu_step.sh claim_b.log 300 python -u scripts/experiments/exp_claim.py 4,2 4,3 8,3 4,2 4,3 8,3 || exit $?
RSGPU_TILE_DIAG=1 bash scripts/gpu_step.sh claim_diag1.log 200 python -u scripts/experiments/exp_claim.py 4 || exit $?
RSGPU_TILE_DIAG=3 bash scripts/gpu_step.sh claim_diag3.log 200 python -u scripts/experiments/exp_claim.py 4 || exit $?
RSGPU_TILE_DIAG=16 bash scripts/gpu_step.sh claim_diag16.log 200 python -u scripts/experiments/tile_epochs.py || exit $?
bash scripts/gpu_step.sh bench_b.log 300 python -u bench.py --steps 20 --warmup 3 || exit $?
bash scripts/gpu_step.sh stability.log 600 python -u scripts/experiments/exp_stability.py || exit $?
