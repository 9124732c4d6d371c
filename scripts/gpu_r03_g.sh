set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_knn_gpu.py tests/test_slope_one_gpu.py > gpurun_out/g_tests.log 2>&1 || exit 3
for P in 5 6 5 6; do
  RSGPU_KNN_PIPE=$P timeout -k 10 300 python3 -u scripts/bench_configs.py --only 3 --out gpurun_out/g_cfg3_pipe$P.jsonl >> gpurun_out/g_cfg3.log 2>&1 || exit 4
done
