#!/bin/bash
for d in cusz_amd/lib cusz_amd/lib_s*; do
  echo "== $d"
  CUSZ_AMD_LIB=$d/libcusz_amd.so timeout -k 10 60 python scripts/scan_bench.py 2>&1 | grep -E "^scan|Error" || true
done
