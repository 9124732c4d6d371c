#!/bin/bash
# Round 4: one-shot Fit phases after folding the divergence check into the download; C-ABI call timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh u_sched.log 300 python -u -m pytest tests/test_sched_dev_gpu.py tests/test_fit_cache_gpu.py -x -q --timeout 120 --timeout-method thread || exit $?
RSGPU_FIT_TRACE=1 bash scripts/gpu_step.sh u_fit_trace.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh u_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh u_fit2.log 300 python -u scripts/bench_fit_e2e.py || exit $?
