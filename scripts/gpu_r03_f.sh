set -u
S=scripts/gpu_step.sh
ROOT=$(pwd)
bash $S pytest_gpu_r03.log 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_bench -o run -- \
    python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $ROOT/gpurun_out/prof_bench.log 2>&1 || exit 5
cd $ROOT
bash scripts/pmc_sgd.sh > gpurun_out/pmc_sgd.log 2>&1 || exit 6
bash scripts/gpu_round.sh > gpurun_out/gpu_round.log 2>&1 || exit 7
