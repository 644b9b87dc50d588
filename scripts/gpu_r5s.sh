#!/bin/bash
export TMPDIR=/tmp
for rep in 1 2 3; do for d in cusz_amd/lib cusz_amd/lib_v1; do
  CUSZ_AMD_LIB=$d/libcusz_amd.so timeout -k 10 60 python scripts/brick_bench.py --reps 20 > gpurun_out/ab.tmp 2>&1 || { cat gpurun_out/ab.tmp; exit 1; }
  echo "$rep $d $(grep -E '^(layout|compress|decompress) ' gpurun_out/ab.tmp | grep -v dbg | tr '\n' ' ' | cut -c1-220)"
done; done
