#!/bin/bash
# GPU suite + config 1 / 5 benches after folding the finalize launches
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:400:python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "bench1:200:python bench.py --config 1 --steps 20 --warmup 3 --no-e2e" \
  "bench5:300:python bench.py --config 5 --steps 10 --warmup 3 --no-e2e"
