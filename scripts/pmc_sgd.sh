#!/bin/bash
# HBM traffic of the SGD tile kernel from PMC counters: FETCH_SIZE and WRITE_SIZE in separate passes
# (MI355X_MICROARCH.md rocprofv3 PMC slots: FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2), kernel
# trace only (no sys/runtime trace with --pmc).  Driver: scripts/experiments/tile_epochs.py (the
# bench.py workload without torch; PMC passes under torch's runtime hung on this image).
# Also the access-width calibration (scripts/experiments/pmc_calib.hip, prebuilt in scripts/bin).
# Summaries -> gpurun_out/pmc/*.json (copied to profiles/ by hand).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$ROOT/gpurun_out/pmc
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/$C" -o run -- \
      python3 "$ROOT/scripts/experiments/tile_epochs.py" > "$OUT/$C.log" 2>&1 || { echo "pmc $C failed"; exit 20; }
done
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" svd_epoch_tile_kernel > "$OUT/sgd_traffic.json" || exit 21
if [ -x "$ROOT/scripts/bin/pmc_calib" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/calib/$C" -o run -- \
        "$ROOT/scripts/bin/pmc_calib" > "$OUT/calib_$C.log" 2>&1 || { echo "calib $C failed"; exit 22; }
  done
  python3 "$ROOT/scripts/pmc_summary.py" --all "$OUT/calib" > "$OUT/calib.json" || exit 23
fi
cat "$OUT"/*.json
