#!/bin/bash
# SQ / LDS counters of the spline kernels (config 5) + the spline bench
export TMPDIR=/tmp
timeout -k 10 120 python scripts/spline_bench.py --reps 5 > gpurun_out/splb.log 2>&1 && cat gpurun_out/splb.log && \
scripts/pmc_kern.sh k_spline3_c splc cusz_amd/lib scripts/spline_bench.py && scripts/pmc_kern.sh k_spline3_x splx cusz_amd/lib scripts/spline_bench.py
