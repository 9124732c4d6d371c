#!/bin/bash
# HBM traffic of the SGD kernel from PMC counters: FETCH_SIZE and WRITE_SIZE in separate passes
# (MI355X_MICROARCH.md rocprofv3 PMC slots: FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2), kernel
# trace only (no sys/runtime trace with --pmc).  Summary -> profiles/sgd_traffic.json.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/$C.log" 2>&1 || exit 20
done
python3 "$ROOT/scripts/parse_pmc.py" "$OUT" svd_epoch_tile_kernel > "$ROOT/gpurun_out/sgd_traffic.json"
