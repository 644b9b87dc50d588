#!/bin/bash
export TMPDIR=/tmp
scripts/gpu_job.sh "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" || exit 1
echo "== lib" >> gpurun_out/var.log
timeout -k 10 60 python scripts/brick_bench.py --reps 20 >> gpurun_out/var.log 2>&1 || exit 1
timeout -k 10 60 python scripts/brick_bench.py --dims 280953867x1x1 --reps 10 >> gpurun_out/var.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/kt -o kt --output-format csv -- python3 scripts/brick_bench.py --reps 3 > gpurun_out/kt.log 2>&1
