set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tile_gpu.py tests/test_svd_gpu.py "tests/test_configs_gpu.py::test_config4_item_shard_k256_defaults" -s > gpurun_out/h_tests.log 2>&1 || exit 3
timeout -k 10 400 python3 -u scripts/bench_configs.py --only 4 --out gpurun_out/h_cfg4.jsonl > gpurun_out/h_cfg4.log 2>&1 || exit 4
