set -u
S=scripts/gpu_step.sh
bash $S pytest_gpu_r03.log 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
bash $S ordered_tput.log 300 python -u scripts/experiments/exp_ordered.py || exit $?
bash $S smoke_r03.log 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash $S bench_r03.log 400 python -u bench.py --steps 20 --warmup 5 || exit $?
