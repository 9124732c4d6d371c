#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh config4_full.log 1000 python -u scripts/config4_sharded.py --epochs 10 --strata || exit $?
bash scripts/gpu_step.sh stab_k.log 300 python -u scripts/experiments/exp_stability.py 128m_k256 8m_k256_hot || exit $?
