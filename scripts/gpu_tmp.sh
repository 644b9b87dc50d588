#!/bin/bash
# decoder tile-store change: full GPU suite, config-2 and config-3 benches
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:400:python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "bench:300:python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e" \
  "bench3:300:python bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e"
