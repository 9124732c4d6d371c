#!/bin/bash
# Round 4: one-shot Fit share with the download folded into the guard's wait.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh x_tests.log 600 python -u -m pytest tests/test_sched_dev_gpu.py tests/test_fit_cache_gpu.py tests/test_stability_gpu.py tests/test_concurrent_gpu.py -x -q --timeout 300 --timeout-method thread || exit $?
bash scripts/gpu_step.sh x_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh x_fit2.log 300 python -u scripts/bench_fit_e2e.py || exit $?
RSGPU_FIT_TRACE=1 bash scripts/gpu_step.sh x_fit_trace.log 300 python -u scripts/bench_fit_e2e.py || exit $?
