#!/bin/bash
# round 5: decoder phase profile (instrumented build) + kernel-trace stats and FETCH/WRITE passes
# of configs 2, 1, 3, 5 (scripts/pmc_config.sh)
export TMPDIR=/tmp
true && \
scripts/pmc_config.sh r05_c2 2 && scripts/pmc_config.sh r05_c1 1 && \
  scripts/pmc_config.sh r05_c3 3 && scripts/pmc_config.sh r05_c5 5
