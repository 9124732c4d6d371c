set -u
S=scripts/gpu_step.sh
bash $S ordered_tests.log 500 python -u -m pytest tests/test_svd_gpu.py -v -k "ordered or tiny" --timeout 300 --timeout-method thread || exit $?
bash $S ordered_tput.log 300 python -u scripts/experiments/exp_ordered.py || exit $?
