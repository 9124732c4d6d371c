set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_csr_plan_gpu.py tests/test_ingest.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_csr.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_csr.log; exit 1; }
tail -3 gpurun_out/t_csr.log
timeout -k 10 300 python -u scripts/bench_config5.py --users 1000000 --items 100000 --k 256 --epochs 3 --cpu-budget 3 > gpurun_out/c5_small.json 2> gpurun_out/c5_small.log || { echo "c5 small failed"; tail -20 gpurun_out/c5_small.log; exit 2; }
cat gpurun_out/c5_small.json
timeout -k 10 300 python -u scripts/bench_config5.py --users 1000000 --items 100000 --k 256 --epochs 3 --shard 0/8 --cpu-budget 0 > gpurun_out/c5_small_s8.json 2> gpurun_out/c5_small_s8.log || { echo "c5 shard failed"; tail -20 gpurun_out/c5_small_s8.log; exit 3; }
cat gpurun_out/c5_small_s8.json
