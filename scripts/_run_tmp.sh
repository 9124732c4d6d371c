set -u
STEPS=20 bash scripts/gpu_check.sh; rc=$?
echo "gpu_check rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_configs.py --out gpurun_out/configs.jsonl > gpurun_out/configs.log 2>&1 || exit 30
bash scripts/pmc_sgd.sh || exit 31
echo done
