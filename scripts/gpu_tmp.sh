#!/bin/bash
# scratch GPU check: sampled-codebook parity, micro-bench
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "sampled:200:python -u -m pytest tests/test_gpu_sampled.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "single:60:python scripts/single_bench.py"
