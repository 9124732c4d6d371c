#!/bin/bash
# headline check after the early prefill: tile exactness tests, claim timing, bench + rocprofv3 kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export REF=0
bash scripts/gpu_step.sh n_tile.log 300 python -u -m pytest tests/test_tile_gpu.py -x -q --timeout 200 --timeout-method thread || exit $?
bash scripts/gpu_step.sh n_claim.log 200 python -u scripts/experiments/exp_claim.py 4 4 || exit $?
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_n" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/n_bench_prof.log" 2>&1 || exit 14
