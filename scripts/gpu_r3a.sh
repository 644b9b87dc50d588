#!/bin/bash
# round 3, first GPU pass: every GPU test, the default bench line, config 4 on one GPU
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:600:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench4:300:python bench.py --config 4 --steps 5 --warmup 2"
