#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh config4_full.log 1000 python -u scripts/config4_sharded.py --epochs 10 --strata || exit $?
