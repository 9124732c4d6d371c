#!/bin/bash
# Round 4: one-shot Fit phases (device schedule, recycled buffers, overlapped host work); stability sweep test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh t_sched.log 300 python -u -m pytest tests/test_sched_dev_gpu.py -x -q --timeout 120 --timeout-method thread || exit $?
RSGPU_FIT_TRACE=1 bash scripts/gpu_step.sh t_fit_trace.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh t_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh t_stab.log 900 python -u -m pytest tests/test_stability_gpu.py -v -s --timeout 600 --timeout-method thread || exit $?
