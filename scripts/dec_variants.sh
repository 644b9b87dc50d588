#!/bin/bash
# Time the brick decoder of each in-tree variant library (cusz_amd/lib_v*/): name -> decompress us
for d in cusz_amd/lib cusz_amd/lib_v*; do
  echo "== $d"
  CUSZ_AMD_LIB=$d/libcusz_amd.so timeout -k 10 60 python scripts/brick_bench.py --reps 10 --dbg 0 2>&1 | grep -E "^decompress dbg" || exit 1
done
