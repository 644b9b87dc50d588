#!/bin/bash
# device codebook: parity test, then its kernel time under the kernel trace
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "book:300:python -u -m pytest tests/test_gpu_book.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "bookprof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_book -o run --output-format csv -- python3 -m pytest tests/test_gpu_book.py -x -q -p no:cacheprovider"
