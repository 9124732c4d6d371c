# PMC passes over the SGD epoch kernel of bench.py (ML-1M shape), one rocprofv3 run per counter group.
set -u
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/tile_pmc
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for G in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
         "SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_ANY" \
         "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" ; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $G --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/scripts/experiments/tile_epochs.py" > "$OUT/p$i.log" 2>&1) || { echo "pass $i failed"; grep -v "^W20" "$OUT/p$i.log" | tail -5; exit 3; }
done
python3 scripts/pmc_summary.py "$OUT" epoch
