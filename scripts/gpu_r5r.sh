#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tall.log 2>&1; rc=$?; tail -3 gpurun_out/tall.log; exit $rc
