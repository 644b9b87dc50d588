#!/bin/bash
# Single-pass (stream) mode: its parity tests, then brick_bench in stream and default modes.
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "stream_tests:300:python -u -m pytest tests/test_gpu_sampled.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "bb_stream:120:python scripts/brick_bench.py --reps 20 --codebook stream" \
  "bb_default:120:python scripts/brick_bench.py --reps 20" \
  "prof:200:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stream -o run --output-format csv -- python3 scripts/brick_bench.py --reps 10 --codebook stream"
