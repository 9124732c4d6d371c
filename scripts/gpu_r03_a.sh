set -u
S=scripts/gpu_step.sh
bash $S multi_r03.log 700 python -u -m pytest tests/test_multi_gpu.py -v -s --timeout 300 --timeout-method thread || exit $?
RSGPU_TILE_DIAG=16 EPOCHS=3 bash $S tile_clocks_r03.log 120 python -u scripts/experiments/tile_epochs.py || exit $?
for d in 0 1 2 3 4 8; do
  RSGPU_TILE_DIAG=$d REF=0 bash $S tile_diag_$d.log 120 python -u scripts/experiments/exp_tile_sweep.py 0,16,0,0,4 0,16,0,0,2 || exit $?
done
