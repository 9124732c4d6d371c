#!/bin/bash
# Round 4: what moved the 8-shard ML-1M fit (run key A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh y_new.log 300 python -u scripts/experiments/exp_multi_key.py 8 4 || exit $?
RSGPU_X_OLDKEY=1 bash scripts/gpu_step.sh y_old.log 300 python -u scripts/experiments/exp_multi_key.py 8 4 || exit $?
