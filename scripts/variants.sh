#!/bin/bash
# Time compress/decompress of each in-tree variant library (cusz_amd/lib, cusz_amd/lib_v*/).
for d in cusz_amd/lib cusz_amd/lib_v*; do
  echo "== $d"
  CUSZ_AMD_LIB=$d/libcusz_amd.so timeout -k 10 60 python scripts/brick_bench.py --reps 10 --dbg 0 "$@" 2>&1 | grep -E "^decompress|^compress" || exit 1
done
