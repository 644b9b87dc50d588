#!/bin/bash
# per-kernel A/B on a bench config: rocprofv3 --kernel-trace --stats of bench.py --config $2 for
# each variant library; prints the averages of the kernels whose names match $1
export TMPDIR=/tmp
pat=$1; cfg=$2
for d in cusz_amd/lib cusz_amd/lib_v*; do
  o=$GRAFT_REPO_ROOT/gpurun_out/abpb_$(basename $d)
  rm -rf $o
  (cd /tmp && CUSZ_AMD_LIB=$GRAFT_REPO_ROOT/$d/libcusz_amd.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $o -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $cfg --steps 10 --warmup 2 --no-other-modes --profile-only > /dev/null 2>&1) || exit 1
  f=$(find $o -name "*kernel_stats.csv" | head -1)
  echo "$d"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if '$pat' in r['Name']: print('  %-40s %6s %8.1f us' % (r['Name'].split('(')[0][-40:], r['Calls'], float(r['AverageNs'])/1000))"
  rm -rf $o
done
