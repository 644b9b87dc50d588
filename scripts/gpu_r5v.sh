#!/bin/bash
# fused tile scan (reference-layout encoder): GPU suite, then config-1 bench and profile
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5v_tests.log 2>&1 || { tail -30 gpurun_out/r5v_tests.log; exit 1; }
tail -3 gpurun_out/r5v_tests.log
timeout -k 10 120 python bench.py --config 1 --steps 20 --warmup 3 > gpurun_out/r5v_c1.json 2> gpurun_out/r5v_c1.err || { tail gpurun_out/r5v_c1.err; exit 1; }
cat gpurun_out/r5v_c1.json | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['stages_ms'])"
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5v_prof -o c1 -- python3 $GRAFT_REPO_ROOT/bench.py --config 1 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r5v_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $GRAFT_REPO_ROOT/gpurun_out/r5v_c1_kernel_stats.csv
rm -rf $GRAFT_REPO_ROOT/gpurun_out/r5v_prof
