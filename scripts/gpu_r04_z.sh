#!/bin/bash
# Round 4: fill-rule device schedule (digest equality, fit share), multi-GPU exchange choice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh z_tests.log 600 python -u -m pytest tests/test_sched_dev_gpu.py tests/test_fit_cache_gpu.py tests/test_multi_gpu.py tests/test_stability_gpu.py -x -q --timeout 300 --timeout-method thread || exit $?
bash scripts/gpu_step.sh z_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh z_fit2.log 300 python -u scripts/bench_fit_e2e.py || exit $?
