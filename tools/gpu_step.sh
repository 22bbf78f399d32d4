#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a fault / abort / segfault / timeout
# (exit codes 124, 134, 137, 139) so that nothing else touches the GPU after it. Ordinary failures
# (e.g. a failing test, exit 1) are reported and the next step may run.
#   tools/gpu_step.sh <seconds> <logname> <command...>
set -u
secs=$1; shift
log=$1; shift
mkdir -p gpurun_out
echo "=== $(date +%T) start: $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "=== $(date +%T) rc=$rc: $*" | tee -a gpurun_out/steps.log
tail -n 25 "gpurun_out/$log"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] || [ $rc -ge 128 ]; then
    echo "FATAL step (rc=$rc): stopping this call" | tee -a gpurun_out/steps.log
    exit 99
fi
exit 0
