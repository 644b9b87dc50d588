#!/bin/bash
# bench lines for every single-GPU BASELINE config (config 2 is the metric's workload) and
# kernel-stats profiles of configs 3 and 5
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "c2:300:python bench.py --steps 10 --warmup 3" \
  "c5:300:python bench.py --config 5 --steps 10 --warmup 3" \
  "c3:300:python bench.py --config 3 --steps 10 --warmup 3" \
  "c1:300:python bench.py --config 1 --steps 20 --warmup 3" \
  "stats3:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats3 -o run --output-format csv -- python3 bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --profile-only" \
  "stats5:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats5 -o run --output-format csv -- python3 bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline --profile-only"
