#!/bin/bash
# round-5 final: default bench line (config 2, with CPU baseline), configs 1/3/4, config-2 profile
export TMPDIR=/tmp
scripts/gpu_job.sh \
  "bench2:300:python bench.py --steps 20 --warmup 5" \
  "c1:300:python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e" \
  "c3:300:python bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e" \
  "c4:400:python bench.py --config 4 --steps 5 --warmup 2" && \
scripts/pmc_config.sh r05_c2 2
