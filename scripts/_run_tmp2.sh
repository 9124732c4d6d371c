set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for T in 0 100 300 1000; do
  echo "== merge ticks $T" >> gpurun_out/rep_sweep.log
  RSGPU_MERGE_TICKS=$T CFGS="256x8,384x8,512x8,256x4" timeout -k 10 300 python -u scripts/exp_replicas.py >> gpurun_out/rep_sweep.log 2>&1 || exit 1
done
cat gpurun_out/rep_sweep.log
