#!/bin/bash
# Round 4, session c: per-workgroup spans of the claim kernel, stability of the hot set (grid / claim / guard),
# configs[4] as a sharded fit at full size (ROTATE_Q, 8 shards on one GPU) with per-stratum times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_step.sh tile_span.log 200 python -u scripts/experiments/tile_span.py || exit $?
S=scripts/experiments/exp_stability.py
bash scripts/gpu_step.sh stab_hot.log 300 bash -c "python -u $S 1m_k100_hot --claim 0 && python -u $S 1m_k100_hot --wg 128 && python -u $S 1m_k100_hot --wg 64 && python -u $S 1m_k100_hot 1m_k64_hot --fit" || exit $?
bash scripts/gpu_step.sh config4.log 900 python -u scripts/config4_sharded.py --strata || exit $?
