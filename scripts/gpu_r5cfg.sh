#!/bin/bash
# round 5: bench lines of configs 1, 3, 4, 5 with the default (sampled) codebook + kernel stats
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "c3:300:python bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e" \
  "c1:300:python bench.py --config 1 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e" \
  "c5:300:python bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e" \
  "c4:400:python bench.py --config 4 --steps 5 --warmup 2" \
  "stats3:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats3 -o run --output-format csv -- python3 bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --profile-only" \
  "stats1:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats1 -o run --output-format csv -- python3 bench.py --config 1 --steps 5 --warmup 2 --no-cpu-baseline --profile-only"
