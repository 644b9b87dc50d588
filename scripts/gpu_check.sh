#!/bin/bash
# Standard GPU pass: every GPU test, the default bench line, the brick micro-benchmark, the
# decoder phase profile (instrumented build, cusz_amd/lib_prof) and a kernel-stats profile.
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
  "brick:120:python scripts/brick_bench.py --reps 20" \
  "bprof:120:python scripts/brick_profile.py" \
  "stats:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-only"
