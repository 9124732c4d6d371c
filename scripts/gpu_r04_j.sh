#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C=scripts/config4_sharded.py
bash scripts/gpu_step.sh j_uniform.log 200 python -u $C --users 200000 --items 20000 --epochs 8 --k 64 --zipf 0 || exit $?
bash scripts/gpu_step.sh j_uniform_p.log 200 python -u $C --users 200000 --items 20000 --epochs 8 --k 64 --zipf 0 --blocks 8 --no-whole || exit $?
bash scripts/gpu_step.sh j_small.log 200 python -u $C --users 200000 --items 20000 --epochs 8 --k 64 --hot-min 0 --no-whole || exit $?
