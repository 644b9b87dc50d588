#!/bin/bash
# scratch GPU check: sampled-codebook mode tests, then the brick suite, then a timing line
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "sampled:200:python -u -m pytest tests/test_gpu_sampled.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "tests:400:python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider"
