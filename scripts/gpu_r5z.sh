#!/bin/bash
# end-of-round refresh, part 2: slab-step table, configs 3 and 4 lines, config-3 profile
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in 64 128 256 512; do
  timeout -k 10 120 python scripts/brick_bench.py --dims 512x512x$p --reps 20 > gpurun_out/r5z_slab$p.log 2>&1 || { tail gpurun_out/r5z_slab$p.log; exit 1; }
  echo "planes $p: $(grep -E '^(compress|decompress) [0-9]' gpurun_out/r5z_slab$p.log | awk '{print $1, $2}' | tr '\n' ' ')"
done
timeout -k 10 300 python bench.py --config 3 > gpurun_out/r5z_c3.json 2> gpurun_out/r5z_c3.err || { tail gpurun_out/r5z_c3.err; exit 1; }
bash scripts/pmc_config.sh r05_c3 3 > /dev/null || exit 1
timeout -k 10 400 python bench.py --config 4 > gpurun_out/r5z_c4.json 2> gpurun_out/r5z_c4.err || { tail gpurun_out/r5z_c4.err; exit 1; }
tail -c 400 gpurun_out/r5z_c4.json
