#!/bin/bash
# sampled/stream mode: parity + bench + kernel profile
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "sampled:300:python -u -m pytest tests/test_gpu_sampled.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "bench2:300:python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e" \
  "stats:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --profile-only"
