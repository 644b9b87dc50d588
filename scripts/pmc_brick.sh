#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over the brick micro-benchmark.
# Usage (GPU box): scripts/pmc_brick.sh <kernel regex> [brick_bench args...]
export TMPDIR=/tmp
re=${1:-k_brick}; shift
mkdir -p gpurun_out/pmc
P=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-include-regex "$re" --pmc $p -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 scripts/brick_bench.py --reps 2 --dbg 0 "$@" > gpurun_out/pmc/p$i.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py "$(find gpurun_out/pmc/p$i -name "*counter_collection.csv" | head -1)" > gpurun_out/pmc/s$i.txt || exit 1
  rm -rf gpurun_out/pmc/p$i
done
cat gpurun_out/pmc/s*.txt
