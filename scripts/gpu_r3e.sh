#!/bin/bash
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "brick_tests:300:python -u -m pytest tests/test_gpu_brick.py tests/test_gpu_parity.py tests/test_gpu_wire.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "variants:300:bash scripts/dec_variants.sh" \
  "bprof2:200:python scripts/brick_profile2.py"
