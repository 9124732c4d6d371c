#!/bin/bash
# One-shot Fit host phases (RSGPU_FIT_TRACE / RSGPU_TILE_TRACE) and the SVD GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RSGPU_FIT_TRACE=1 RSGPU_TILE_TRACE=1 timeout -k 10 300 python -u scripts/bench_fit_e2e.py > gpurun_out/fit_e2e.log 2> gpurun_out/fit_e2e_trace.log || exit 13
timeout -k 10 200 python -u scripts/bench_fit_e2e.py > gpurun_out/fit_e2e_notrace.log 2>&1 || exit 14
if [ -n "${TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > gpurun_out/fit_tests.log 2>&1 || exit 15
fi
