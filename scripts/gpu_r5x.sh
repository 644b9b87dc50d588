#!/bin/bash
# end-of-round refresh: default bench line (config 2) and its profile; config-1 and -5 lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r5x_c2.json 2> gpurun_out/r5x_c2.err || { tail gpurun_out/r5x_c2.err; exit 1; }
tail -c 600 gpurun_out/r5x_c2.json
bash scripts/pmc_config.sh r05_c2 2 || exit 1
timeout -k 10 200 python bench.py --config 1 > gpurun_out/r5x_c1.json 2> gpurun_out/r5x_c1.err || { tail gpurun_out/r5x_c1.err; exit 1; }
bash scripts/pmc_config.sh r05_c1 1 || exit 1
timeout -k 10 300 python bench.py --config 5 > gpurun_out/r5x_c5.json 2> gpurun_out/r5x_c5.err || { tail gpurun_out/r5x_c5.err; exit 1; }
bash scripts/pmc_config.sh r05_c5 5 || exit 1
