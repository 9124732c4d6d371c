#!/bin/bash
# SQ / GRBM counters of the K4 kernel on configs[3] (ML-20M-shaped item Cosine, default K loop),
# two passes (<= 8 SQ counters each), then scripts/pmc_knn_summary.py.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/knn_pmc
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
P1="SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/pass$i" -o run -- \
      python3 "$ROOT/scripts/bench_configs.py" --only 3 > "$OUT/pass$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 41; }
done
python3 "$ROOT/scripts/pmc_knn_summary.py" "$OUT" > "$OUT/knn_pmc.json" && cat "$OUT/knn_pmc.json"
