#!/bin/bash
# Run one GPU step under its own time limit; stop the whole script on a
# fault / abort / segfault / timeout (exit >= 124 or signal), continue on
# ordinary failures (exit 1-2, e.g. a failing assertion).
#   usage: gpu_step.sh <seconds> <logfile> <cmd...>
secs=$1; log=$2; shift 2
echo "=== $(date +%T) $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "=== rc=$rc $*" | tee -a gpurun_out/steps.log
tail -5 "$log"
if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then
  echo "FATAL step (rc=$rc): stopping" | tee -a gpurun_out/steps.log
  exit 99
fi
exit 0
