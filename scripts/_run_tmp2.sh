set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_nmf_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_nmf.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_nmf.log; exit 1; }
tail -3 gpurun_out/t_nmf.log
timeout -k 10 300 python -u scripts/bench_configs.py --only nmf > gpurun_out/nmf.json 2> gpurun_out/nmf.err || { tail gpurun_out/nmf.err; exit 2; }
cat gpurun_out/nmf.json
