#!/bin/bash
# round 3: decoder v2 -- brick parity, full GPU suite, A/B of the two fused decoders, bench
export TMPDIR=/tmp
exec scripts/gpu_job.sh \
  "brick_tests:300:python -u -m pytest tests/test_gpu_brick.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "ab_v2:120:python scripts/brick_bench.py --reps 20 --dbg 0" \
  "ab_v1:120:env CUSZ_AMD_BRICK_DEC_V1=1 python scripts/brick_bench.py --reps 20 --dbg 0" \
  "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
  "stats:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stats -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-only" \
  "pmc:400:bash scripts/pmc_brick.sh k_brick3_decode"
