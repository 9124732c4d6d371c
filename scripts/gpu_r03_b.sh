set -u
S=scripts/gpu_step.sh
REF=1 bash $S cold_ref.log 200 python -u scripts/experiments/exp_tile_sweep.py 0,16,0,0,2 || exit $?
for c in 1 2 4 8 16 32 64 128 256; do
  RSGPU_TILE_COLD=$c REF=0 bash $S cold_$c.log 120 python -u scripts/experiments/exp_tile_sweep.py 0,16,0,0,2 || exit $?
done
