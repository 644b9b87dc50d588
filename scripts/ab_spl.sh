#!/bin/bash
# A/B timing of variant libraries on the spline path (config 5), interleaved 3 times
export TMPDIR=/tmp
for rep in 1 2 3; do
  for d in cusz_amd/lib cusz_amd/lib_v*; do
    CUSZ_AMD_LIB=$d/libcusz_amd.so timeout -k 10 90 python scripts/spline_bench.py --reps 5 $@ > gpurun_out/ab.tmp 2>&1 || { cat gpurun_out/ab.tmp; exit 1; }
    echo "$rep $d $(grep -E 'spline_c=' gpurun_out/ab.tmp)"
  done
done
