#!/bin/bash
# Round check on the GPU box: GPU parity tests, smoke, bench line, brick micro-bench, kernel stats.
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:600:python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py --steps 10 --warmup 3" \
  "brick:120:python scripts/brick_bench.py --reps 10" \
  "stats:200:scripts/prof_stats.sh gpurun_out/prof_stats"
