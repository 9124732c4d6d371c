set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_svdpp_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_pp.log 2>&1 || { tail -30 gpurun_out/t_pp.log; exit 1; }
tail -2 gpurun_out/t_pp.log
NB=default timeout -k 10 300 python -u scripts/exp_svdpp_blocks.py
