#!/bin/bash
# GPU suite + default config-2 bench (quick: no CPU baseline / e2e) + kernel stats
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench2:300:python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e" \
  "stats:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --profile-only"
