#!/bin/bash
# Standard GPU verification + measurement pass (run through gpurun from the repo root).
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "parity:400:python -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests -q -m gpu --timeout 250 -p no:cacheprovider -x" \
  "bench:300:python bench.py --steps 10 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline}" \
  "stats:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-only" \
  "pmc1:300:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_pmc1 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-only" \
  "pmc2:300:rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_pmc2 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --profile-only"
