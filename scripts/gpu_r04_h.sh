#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C=scripts/config4_sharded.py
bash scripts/gpu_step.sh h_small_avg.log 200 python -u $C --users 200000 --items 20000 --epochs 8 --k 64 --hot-min 0 || exit $?
bash scripts/gpu_step.sh h_small_sum.log 200 python -u $C --users 200000 --items 20000 --epochs 8 --k 64 --hot-min 0 --hot-sum --no-whole || exit $?
bash scripts/gpu_step.sh h_mid_avg.log 300 python -u $C --users 1000000 --items 100000 --epochs 5 || exit $?
bash scripts/gpu_step.sh h_mid_sum.log 300 python -u $C --users 1000000 --items 100000 --epochs 5 --hot-sum --no-whole || exit $?
bash scripts/gpu_step.sh h_multi.log 400 python -u -m pytest tests/test_multi_gpu.py -x -v --timeout 200 --timeout-method thread || exit $?
