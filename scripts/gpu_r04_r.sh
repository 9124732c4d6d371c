#!/bin/bash
# Round 4: device-built tile schedule (tests, one-shot Fit phases), claim-queue order sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh r_sched.log 300 python -u -m pytest tests/test_sched_dev_gpu.py -x -v --timeout 120 --timeout-method thread || exit $?
RSGPU_FIT_TRACE=1 RSGPU_TILE_TRACE=1 bash scripts/gpu_step.sh r_fit_trace.log 300 python -u scripts/bench_fit_e2e.py || exit $?
bash scripts/gpu_step.sh r_fit.log 300 python -u scripts/bench_fit_e2e.py || exit $?
export REF=0
for q in 0 1 2 3; do
  RSGPU_X_QORDER=$q bash scripts/gpu_step.sh q_$q.log 200 python -u scripts/experiments/exp_claim.py 4 4 4 || exit $?
done
