#!/bin/bash
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench2:300:python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e" \
  "bench4:400:python bench.py --config 4 --steps 5 --warmup 2"
