#!/bin/bash
# Round 4: fit share after recycling the guard buffers; stability once more.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh s4_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh s4_fit2.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh s4_stab.log 900 python -u -m pytest tests/test_stability_gpu.py tests/test_sched_dev_gpu.py tests/test_fit_cache_gpu.py -q --timeout 600 --timeout-method thread || exit $?
