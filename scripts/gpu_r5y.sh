#!/bin/bash
# 1-D decoder cell ring: GPU suite, then config-3 A/B against lib_v0
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5y_tests.log 2>&1 || { tail -30 gpurun_out/r5y_tests.log; exit 1; }
tail -2 gpurun_out/r5y_tests.log
bash scripts/ab_cfg.sh 3
