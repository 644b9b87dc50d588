#!/bin/bash
# summarise the last gpurun_out (job log, bench line, profile) ; arg1 = profile tag
grep -E "rc=|passed|failed|error" gpurun_out/job.log
grep '"value"' gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', d['value'], 'comp', d['compress_gbps'], 'decomp', d['decompress_gbps'], 'CR', d['compression_ratio']); print(d['stages_ms']); print(d['roofline']); print(d.get('cpu_baseline'))"
[ -n "$1" ] && [ -f gpurun_out/prof_stats/run_kernel_stats.csv ] && python3 scripts/prof_summary.py "$1" gpurun_out/prof_stats gpurun_out/prof_pmc1 gpurun_out/prof_pmc2
