#!/bin/bash
# Round 4: kernel trace of the one-shot Fit bench (device schedule build kernels, transfers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_v
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_v -o fit -- python3 -u scripts/bench_fit_e2e.py > gpurun_out/v_fit.log 2>&1 || exit $?
