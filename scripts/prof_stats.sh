#!/bin/bash
# Kernel-trace stats of a short bench run; prints our kernels' average durations (us).
# Usage (on the GPU box): scripts/prof_stats.sh <outdir> [bench args...]
out=$1; shift
export TMPDIR=/tmp
rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-only "$@" > "$out.log" 2>&1 || exit $?
f=$(find "$out" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'cusz' in r['Name']:
        print(f"{float(r['AverageNs'])/1000:9.1f} us  x{r['Calls']:>3}  {r['Name'][:110]}")
PY
