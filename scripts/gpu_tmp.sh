#!/bin/bash
# round-end measurement after the decoder change: smoke, config-2 bench + profile, config-3 bench
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py --steps 20 --warmup 5" \
  "prof2:500:bash scripts/pmc_config.sh r03_c2 2" \
  "bench3:300:python bench.py --config 3 --steps 10 --warmup 3" \
  "prof3:500:bash scripts/pmc_config.sh r03_c3 3"
