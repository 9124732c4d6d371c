#!/bin/bash
# Round 4, first session: tile + multi + concurrency + KNN tests (one-wave exactness now runs the claimed-run
# kernel; ROTATE_Q; Go sort order), the C++ mirror (threaded CrossValidate), the claim A/B on the ML-1M shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh tile_tests.log 500 python -u -m pytest tests/test_tile_gpu.py tests/test_multi_gpu.py tests/test_concurrent_gpu.py tests/test_host_cpp.py tests/test_knn_gpu.py -x -v --timeout 200 --timeout-method thread || exit $?
bash scripts/gpu_step.sh claim.log 400 python -u scripts/experiments/exp_claim.py || exit $?
