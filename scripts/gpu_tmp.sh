#!/bin/bash
# round-end benches for configs 1 and 5 (config 2/3 lines are in profiles/ already)
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "bench1:200:python bench.py --config 1 --steps 20 --warmup 3" \
  "bench5:300:python bench.py --config 5 --steps 10 --warmup 3"
