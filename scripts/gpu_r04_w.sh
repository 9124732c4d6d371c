#!/bin/bash
# Round 4: divergence guard in plan_epochs; stability sweep; fit share; the SVD GPU suites.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh w_stab.log 900 python -u -m pytest tests/test_stability_gpu.py -v -s --timeout 600 --timeout-method thread || exit $?
bash scripts/gpu_step.sh w_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh w_svd.log 900 python -u -m pytest tests/test_sched_dev_gpu.py tests/test_fit_cache_gpu.py tests/test_svd_gpu.py tests/test_tile_gpu.py tests/test_concurrent_gpu.py -x -q --timeout 200 --timeout-method thread || exit $?
bash scripts/gpu_step.sh w_bench.log 600 python -u bench.py --no-strong || exit $?
bash scripts/gpu_step.sh w_c4.log 900 python -u -m pytest tests/test_config4_gpu.py -x -v -s --timeout 800 --timeout-method thread || exit $?
