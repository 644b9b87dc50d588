#!/bin/bash
# Decoder iteration on the GPU box: brick parity tests, then the brick micro-benchmark.
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "brick_tests:300:python -u -m pytest tests/test_gpu_brick.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "brick:120:python scripts/brick_bench.py --reps 10 --dbg 0" \
  "tests:600:python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider"
