set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | head -30; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u scripts/bench_config5.py --epochs 3 --shard 0/8 --partition users --cpu-budget 0 > gpurun_out/c5_u8.json 2> gpurun_out/c5_u8.log || { echo "c5 users shard failed"; tail -20 gpurun_out/c5_u8.log; exit 3; }
cat gpurun_out/c5_u8.json
