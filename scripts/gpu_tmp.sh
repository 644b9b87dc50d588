#!/bin/bash
# scratch GPU check: config-2 bench with the sampled-codebook leg, kernel stats
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "bench:300:python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e" \
  "stats:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --profile-only"
