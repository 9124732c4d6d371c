# gpu_step.sh LOG SECONDS CMD... -- one GPU step under its own time limit; output to gpurun_out/LOG.
# Exit status 0 or 1 (a test failure) lets the caller go on; anything else (fault, abort, timeout) stops.
set -u
log=$1; lim=$2; shift 2
mkdir -p gpurun_out
echo "== $(date +%T) $*" >> gpurun_out/steps.log
timeout -k 10 "$lim" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "== rc=$rc $log" >> gpurun_out/steps.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
exit 0
