#!/bin/bash
# Round-3 evidence session: GPU tests, smoke, bench (+ rocprofv3 kernel trace), one-shot Fit phases.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
RSGPU_FIT_TRACE=1 RSGPU_TILE_TRACE=1 timeout -k 10 300 python -u scripts/bench_fit_e2e.py > gpurun_out/fit_e2e.log 2> gpurun_out/fit_e2e_trace.log || exit 13
timeout -k 10 200 python -u scripts/bench_fit_e2e.py > gpurun_out/fit_e2e_notrace.log 2>&1 || exit 14
