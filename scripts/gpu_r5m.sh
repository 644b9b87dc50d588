#!/bin/bash
# kernel timeline of bench.py's timed steps (config 2) for gap analysis
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/tl/t -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-other-modes > gpurun_out/tl/t.log 2>&1
python3 - <<'PY'
import csv, glob, re
f = glob.glob('gpurun_out/tl/t/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'cusz_amd' in r['Kernel_Name']]
# find the longest run of brick kernels: print the 30 kernels before the last 60
sel = rows[-(8 + 80 + 80 + 80):-(8 + 80 + 80 + 56)]
prev = None
for r in sel:
    m = re.search(r'(k_\w+)', r['Kernel_Name']); name = m.group(1) if m else r['Kernel_Name'][:30]
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{name:28s} start+{gap:8.1f} us  dur {(e - s) / 1e3:8.1f} us")
    prev = e
PY
rm -rf gpurun_out/tl/t
