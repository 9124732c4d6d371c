#!/bin/bash
# configs[4] at 1/8 scale, item shard 0/8 (delta protocol): held-out RMSE per schedule toggle
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/c5_matrix.log
for opts in "" "--split 0" "--fixed-q 0" "--hot 0" "--split 0 --fixed-q 0 --hot 0" "--item-cap 0"; do
  timeout -k 10 120 python -u scripts/bench_config5.py --users 1250000 --items 125000 --epochs 2 --shard 0/8 \
      --cpu-budget 0 $opts > gpurun_out/c5m.json 2> gpurun_out/c5m.log || { echo "failed: $opts"; tail -5 gpurun_out/c5m.log; exit 2; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c5m.json')); h=d['holdout']
print('opts=[$opts]', 'epoch_ms=%.2f' % (d['epoch_s']*1e3), 'rmse0=%.4f rmse=%.4f' % (h['rmse_init'], h['rmse']))" >> gpurun_out/c5_matrix.log
done
cat gpurun_out/c5_matrix.log
