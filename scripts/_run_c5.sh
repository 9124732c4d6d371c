set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/bench_config5.py --epochs 3 > gpurun_out/c5_full.json 2> gpurun_out/c5_full.log || { echo "c5 full failed"; tail -20 gpurun_out/c5_full.log; exit 2; }
cat gpurun_out/c5_full.json
timeout -k 10 400 python -u scripts/bench_config5.py --epochs 3 --shard 0/8 --cpu-budget 0 > gpurun_out/c5_s8.json 2> gpurun_out/c5_s8.log || { echo "c5 shard failed"; tail -20 gpurun_out/c5_s8.log; exit 3; }
cat gpurun_out/c5_s8.json
