#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh config4_e.log 600 python -u scripts/config4_sharded.py --no-whole --epochs 3 || exit $?
bash scripts/gpu_step.sh config4_e2.log 600 python -u scripts/config4_sharded.py --no-whole --epochs 3 --blocks 8 || exit $?
