#!/bin/bash
# A/B timing of in-tree variant libraries (cusz_amd/lib and cusz_amd/lib_v*), interleaved 3 times:
# prints compress / decompress us of scripts/brick_bench.py per library
export TMPDIR=/tmp
for rep in 1 2 3; do
  for d in cusz_amd/lib cusz_amd/lib_v*; do
    CUSZ_AMD_LIB=$d/libcusz_amd.so timeout -k 10 60 python scripts/brick_bench.py --reps 20 $@ > gpurun_out/ab.tmp 2>&1 || { cat gpurun_out/ab.tmp; exit 1; }
    echo "$rep $d $(grep -E '^(compress|decompress) [0-9]' gpurun_out/ab.tmp | awk '{print $1, $2}' | tr '\n' ' ')"
  done
done
