#!/bin/bash
# One rocprofv3 PMC pass over a short brick_bench run; prints per-kernel counter sums/averages.
# Usage (on the GPU box): scripts/pmc_pass.sh <outdir> "<counters>" [brick_bench args...]
out=$1; ctr=$2; shift 2
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$out" -o run --output-format csv -- python3 scripts/brick_bench.py --reps 2 "$@" > "$out.log" 2>&1 || exit $?
python3 scripts/pmc_summary.py "$(find "$out" -name "*counter_collection.csv" | head -1)" > "$out.summary" && cat "$out.summary" && rm -rf "$out"
