#!/bin/bash
# ORDERED batched kernel: parity tests, then the ML-1M timing experiments
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 300 python -u -m pytest tests/test_svd_gpu.py -k "ordered" -x -v --timeout 120 --timeout-method thread > gpurun_out/ordered_tests.log 2>&1 || exit 11
fi
timeout -k 10 300 python -u scripts/experiments/exp_ordered_prof.py "$@" > gpurun_out/ordered_prof.log 2>&1 || exit 12
if [ "${FIT_TRACE:-0}" = "1" ]; then
RSGPU_FIT_TRACE=1 RSGPU_TILE_TRACE=1 timeout -k 10 300 python -u scripts/bench_fit_e2e.py > gpurun_out/fit_e2e.log 2> gpurun_out/fit_e2e_trace.log || exit 13
fi
