#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tall.log 2>&1; rc=$?; tail -3 gpurun_out/tall.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/b2.log 2>&1 && tail -1 gpurun_out/b2.log | cut -c1-300
