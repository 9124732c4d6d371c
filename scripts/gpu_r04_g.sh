#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C=scripts/config4_sharded.py
bash scripts/gpu_step.sh g_small.log 300 python -u $C --users 200000 --items 20000 --epochs 4 --k 64 --hot-min 0 || exit $?
bash scripts/gpu_step.sh g_mid.log 400 python -u $C --users 1000000 --items 100000 --epochs 4 || exit $?
bash scripts/gpu_step.sh g_full.log 900 python -u $C --epochs 5 --strata || exit $?
