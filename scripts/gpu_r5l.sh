#!/bin/bash
# config 5 bench + its profile after the spline changes
export TMPDIR=/tmp
scripts/gpu_job.sh "c5:300:python bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e" && \
scripts/pmc_config.sh r05_c5 5
