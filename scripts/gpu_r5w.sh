#!/bin/bash
# fused tile totals: GPU suite, config-1 A/B (+ stats), config-5 bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5w_tests.log 2>&1 || { tail -30 gpurun_out/r5w_tests.log; exit 1; }
tail -2 gpurun_out/r5w_tests.log
bash scripts/ab_c1.sh || exit 1
timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-other-modes > gpurun_out/r5w_c5.json 2> gpurun_out/r5w_c5.err || { tail gpurun_out/r5w_c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r5w_c5.json')); print('c5', d['value'], d['ms_per_step'], d['stages_ms'])"
