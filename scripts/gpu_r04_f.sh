#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
C=scripts/config4_sharded.py
bash scripts/gpu_step.sh c4_small.log 300 python -u $C --users 200000 --items 20000 --epochs 3 --shards 8 || exit $?
bash scripts/gpu_step.sh c4_small_k64.log 300 python -u $C --users 200000 --items 20000 --epochs 3 --shards 8 --k 64 || exit $?
bash scripts/gpu_step.sh c4_mid.log 400 python -u $C --users 1000000 --items 100000 --epochs 3 --shards 8 || exit $?
