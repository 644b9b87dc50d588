#!/bin/bash
# round 5: GPU suite + bench lines of configs 2 (with the CPU baseline) and 1
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:900:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench2:300:python bench.py --steps 10 --warmup 3" \
  "c1:300:python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e"
