#!/bin/bash
# Round 4: stability sweep with the 0.3 % and 3 % hottest-item sets.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh s2_stab.log 900 python -u -m pytest tests/test_stability_gpu.py -v -s --timeout 600 --timeout-method thread || exit $?
