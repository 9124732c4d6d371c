#!/bin/bash
# Round 4: stability sweep twice after the guard's tighter signals; fit and svd suites.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh s3_stab1.log 900 python -u -m pytest tests/test_stability_gpu.py -v -s --timeout 600 --timeout-method thread || exit $?
bash scripts/gpu_step.sh s3_stab2.log 900 python -u -m pytest tests/test_stability_gpu.py -v -s --timeout 600 --timeout-method thread || exit $?
bash scripts/gpu_step.sh s3_svd.log 900 python -u -m pytest tests/test_sched_dev_gpu.py tests/test_fit_cache_gpu.py tests/test_svd_gpu.py tests/test_tile_gpu.py -x -q --timeout 200 --timeout-method thread || exit $?
bash scripts/gpu_step.sh s3_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
