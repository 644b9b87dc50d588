#!/bin/bash
# v2 decoder phase profile
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "bprof2:200:python scripts/brick_profile2.py" \
  "bprof1:200:env CUSZ_AMD_BRICK_DEC_V1=1 python scripts/brick_profile.py"
