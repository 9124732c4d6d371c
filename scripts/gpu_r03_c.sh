set -u
S=scripts/gpu_step.sh
RSGPU_TILE_DIAG=16 EPOCHS=3 CLOCKS_NPZ=gpurun_out/tile_clocks.npz bash $S tile_clocks_r03b.log 400 python -u scripts/experiments/tile_epochs.py || exit $?
