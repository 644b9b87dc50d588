#!/bin/bash
# A/B of variant libraries on config $1 (default 1) (bench.py lines), interleaved 3 times, then the kernel
# stats of the in-tree library
export TMPDIR=/tmp
CFG=${1:-1}
for rep in 1 2 3; do
  for d in cusz_amd/lib cusz_amd/lib_v*; do
    CUSZ_AMD_LIB=$d/libcusz_amd.so timeout -k 10 120 python bench.py --config $CFG --steps 30 --warmup 3 --no-other-modes > gpurun_out/abc$CFG.json 2> gpurun_out/abc$CFG.err || { tail gpurun_out/abc$CFG.err; exit 1; }
    echo "$rep $d $(python -c "import json; d=json.load(open('gpurun_out/abc$CFG.json')); print(d['ms_per_step'], d['stages_ms']['encode'], d['stages_ms']['compress'])")"
  done
done
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/abc$CFG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --steps 20 --warmup 3 --no-other-modes > /dev/null 2>&1 || exit 1
f=$(find $GRAFT_REPO_ROOT/gpurun_out/abc$CFG -name "*kernel_stats.csv" | head -1); cp $f $GRAFT_REPO_ROOT/gpurun_out/abc${CFG}_kernel_stats.csv
rm -rf $GRAFT_REPO_ROOT/gpurun_out/abc$CFG
