#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C=scripts/config4_sharded.py
bash scripts/gpu_step.sh i_small.log 200 python -u $C --users 200000 --items 20000 --epochs 8 --k 64 --hot-min 0 --no-whole || exit $?
bash scripts/gpu_step.sh i_small4.log 200 python -u $C --users 200000 --items 20000 --epochs 8 --k 64 --hot-min 0 --hot-share 0.04 --no-whole || exit $?
bash scripts/gpu_step.sh i_mid.log 300 python -u $C --users 1000000 --items 100000 --epochs 5 --no-whole || exit $?
bash scripts/gpu_step.sh i_mid4.log 300 python -u $C --users 1000000 --items 100000 --epochs 5 --no-whole --hot-share 0.04 || exit $?
