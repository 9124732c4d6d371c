#!/bin/bash
# KNN (K4) session: parity tests of the similarity kernels, then configs[3] (ML-20M-shaped item
# Cosine) for each K-loop variant (RSGPU_KNN_PIPE 0, 3, 4, 5) and with / without the streamed download,
# then a rocprofv3 kernel trace of the default.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/knn
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_knn_gpu.py tests/test_slope_one_gpu.py -x -v --timeout 300 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "knn tests failed"; exit 21; }
for P in ${PIPES:-0 3 4 5}; do
  RSGPU_KNN_PIPE=$P timeout -k 10 300 python3 -u scripts/bench_configs.py --only 3 --out "$OUT/cfg3_pipe$P.jsonl" \
      > "$OUT/cfg3_pipe$P.log" 2>&1 || { echo "config 3 pipe $P failed"; exit 22; }
done
RSGPU_KNN_NO_STREAM=1 timeout -k 10 300 python3 -u scripts/bench_configs.py --only 3 --out "$OUT/cfg3_nostream.jsonl" \
    > "$OUT/cfg3_nostream.log" 2>&1 || { echo "config 3 no-stream failed"; exit 23; }
if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOT/scripts/bench_configs.py" --only 3 > "$OUT/prof.log" 2>&1 || { echo "rocprof failed"; exit 24; }
fi
echo done
