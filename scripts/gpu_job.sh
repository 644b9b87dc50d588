#!/bin/bash
# Runs GPU steps in order; each has its own time limit. Stops at the first step that
# faults, aborts, segfaults or times out (exit 124/134/137/139 or >128); ordinary test
# failures (exit 1) do not stop later steps.  Usage: scripts/gpu_job.sh "name:secs:cmd" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] $(date +%T) $cmd" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc $(date +%T)" | tee -a gpurun_out/job.log
  tail -3 "gpurun_out/$name.log" | tee -a gpurun_out/job.log
  if [ $rc -ge 124 ]; then echo "stopping after fatal rc=$rc" | tee -a gpurun_out/job.log; exit $rc; fi
done
exit 0
