set -u
mkdir -p gpurun_out
for d in 0 1 2 3 4 12 15; do
  echo "== diag $d" >> gpurun_out/tile_diag.log
  RSGPU_TILE_DIAG=$d REF=0 timeout -k 10 120 python -u scripts/experiments/exp_tile_sweep.py 0,16,0,0,4 >> gpurun_out/tile_diag.log 2>&1 || exit 3
done
