#!/bin/bash
# fused decoder diagnosis: phase clocks (instrumented build) + SQ/LDS counters of k_brick3_decode
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "bprof:200:python scripts/brick_profile.py" \
  "bbench:200:python scripts/brick_bench.py --reps 10" \
  "pmc:400:bash scripts/pmc_brick.sh k_brick3_decode"
