set -u
mkdir -p gpurun_out
for D in 8 16 32; do
  RSGPU_PP_DEPTH=$D CFGS="d:d" REPS=2 timeout -k 10 300 python -u scripts/experiments/exp_pp_accuracy.py > gpurun_out/pp_depth$D.log 2>&1 || exit 3
done
