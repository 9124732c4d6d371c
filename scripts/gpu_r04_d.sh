#!/bin/bash
# Round 4, session d: hot-set stability vs the placement of an item's pieces in the claim queue; configs[4]
# sharded with fewer workgroups per shard (staleness check).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=scripts/experiments/exp_stability.py
bash scripts/gpu_step.sh stab_d.log 300 bash -c "RSGPU_TILE_SPREAD=0 python -u $S 1m_k100_hot 1m_k64 && python -u $S 1m_k100_hot --claim 8 && RSGPU_TILE_SPREAD=0 python -u $S 1m_k100_hot --claim 8 && python -u $S 1m_k100_hot --claim 0 --wg 512" || exit $?
RSGPU_TILE_SPREAD=0 bash scripts/gpu_step.sh claim_d.log 200 python -u scripts/experiments/exp_claim.py 4 8 || exit $?
