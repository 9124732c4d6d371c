#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel-trace summary.
# Stops at the first GPU fault / abort / timeout (exit codes other than 0 or a plain test failure 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-20}

ok() { local c=$1; [ "$c" -eq 0 ] || [ "$c" -eq 1 ]; }

# extensions are built in-tree on the CPU container before the call (they travel with the tree)
echo "== start" > "$OUT/session.log"

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu" >> "$OUT/session.log"
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  c=$?; echo "pytest exit $c" >> "$OUT/session.log"; ok $c || exit 11
fi

if [ "${SKIP_SMOKE:-0}" != "1" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  c=$?; echo "smoke exit $c" >> "$OUT/session.log"; [ $c -eq 0 ] || exit 12
fi

echo "== bench" >> "$OUT/session.log"
timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 > "$OUT/bench.log" 2>&1
c=$?; echo "bench exit $c" >> "$OUT/session.log"; [ $c -eq 0 ] || exit 13

if [ "${SKIP_PROF:-0}" != "1" ]; then
  echo "== rocprofv3 kernel trace" >> "$OUT/session.log"
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python3 "$ROOT/bench.py" --steps $STEPS --warmup 3 --no-cpu-baseline --no-strong > "$OUT/bench_prof.log" 2>&1
  c=$?; echo "rocprof exit $c" >> "$OUT/session.log"; [ $c -eq 0 ] || exit 14
fi
echo "== done" >> "$OUT/session.log"
