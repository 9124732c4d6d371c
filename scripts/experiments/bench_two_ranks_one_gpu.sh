#!/bin/bash
# Rehearsal of the driver's `bench.py --gpus N` on ONE GPU (experiment; N = 2 by default, RANKS=4 at most here,
# never 8): N bench.py rank processes on device 0 (LOCAL_RANK=0 for all), each with its own NCCL_HOSTID so RCCL connects them through its socket transport
# (tests/rccl_ranks.py explains why), torch.distributed "nccl" and the library's communicator both.  Rank logs go to
# gpurun_out/bench2/; rank 0's JSON line is the result.  Usage: bash scripts/experiments/bench_two_ranks_one_gpu.sh [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/bench2
PORT=$(python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
N=${RANKS:-2}
[ "$N" -le 4 ] || { echo "at most 4 ranks on one GPU here"; exit 2; }
pids=()
for r in $(seq 0 $((N - 1))); do
  env RANK=$r LOCAL_RANK=0 WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
      HSA_ENABLE_IPC_MODE_LEGACY=0 NCCL_HOSTID=rsgpu-bench-$r NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 \
      timeout -k 10 900 python3 -u bench.py --gpus $N --no-cpu-baseline "$@" > gpurun_out/bench2/r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
tail -5 gpurun_out/bench2/r$((N - 1)).log
grep '^{' gpurun_out/bench2/r0.log | tail -1
exit $rc
