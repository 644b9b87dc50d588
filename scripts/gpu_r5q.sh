#!/bin/bash
# kernel timeline of a 64-plane slab's compress / decompress (brick_bench, back-to-back calls)
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tl/s -o run --output-format csv -- python3 scripts/brick_bench.py --dims 512x512x64 --reps 5 > gpurun_out/tl/s.log 2>&1
python3 - <<'PY'
import csv, glob, re
f = glob.glob('gpurun_out/tl/s/**/*kernel_trace.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'cusz_amd' in r['Kernel_Name']]
prev = None
for r in rows[-26:]:
    m = re.search(r'(k_\w+)', r['Kernel_Name']); name = m.group(1)
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{name:28s} start+{(s - prev) / 1e3 if prev else 0:8.1f} us  dur {(e - s) / 1e3:8.1f} us")
    prev = e
PY
rm -rf gpurun_out/tl/s
