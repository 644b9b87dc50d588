#!/bin/bash
# Runs GPU steps in order; each has its own time limit. Stops at the first step that fails
# in any way (a failed test may be a GPU fault: nothing more runs on the card after it).
# Usage: scripts/gpu_job.sh "name:secs:cmd" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] $(date +%T) $cmd" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc $(date +%T)" | tee -a gpurun_out/job.log
  tail -3 "gpurun_out/$name.log" | tee -a gpurun_out/job.log
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc" | tee -a gpurun_out/job.log; exit $rc; fi
done
exit 0
