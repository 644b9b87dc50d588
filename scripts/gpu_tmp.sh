#!/bin/bash
# round-end measurement: GPU suite, smoke, config-2 bench (CPU baseline, e2e), config-2 profile
# (stats + FETCH/WRITE), config-3 bench
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "tests:400:python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py --steps 20 --warmup 5" \
  "prof2:500:bash scripts/pmc_config.sh r03_c2 2" \
  "bench3:300:python bench.py --config 3 --steps 10 --warmup 3"
