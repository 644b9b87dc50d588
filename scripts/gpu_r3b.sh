#!/bin/bash
# round 3: GPU tests, default bench line, decoder diagnosis (phase clocks, ring variants, SQ counters)
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
  "bprof:200:python scripts/brick_profile.py" \
  "variants:300:bash scripts/dec_variants.sh" \
  "pmc:400:bash scripts/pmc_brick.sh k_brick3_decode"
