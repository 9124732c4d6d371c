#!/bin/bash
# Second GPU session of a round: the other BASELINE configs (bench_configs.py), their rocprofv3
# kernel trace, and FETCH/WRITE PMC passes of their kernels.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/cfg
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
ONLY=${ONLY:-0,2,nmf,3,4}
timeout -k 10 600 python3 -u scripts/bench_configs.py --only $ONLY --out "$OUT/configs.jsonl" > "$OUT/configs.log" 2>&1 \
  || { echo "bench_configs failed"; exit 31; }
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/scripts/bench_configs.py" --only ${PONLY:-2,nmf,3,4} > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; exit 32; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/pmc/$C" -o run -- \
      python3 "$ROOT/scripts/bench_configs.py" --only ${PONLY:-2,nmf,3,4} > "$OUT/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; exit 33; }
done
python3 "$ROOT/scripts/pmc_summary.py" --all "$OUT/pmc" > "$OUT/pmc.json"
cat "$OUT/pmc.json"
