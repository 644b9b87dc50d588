#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over the brick micro-benchmark.
# Usage (GPU box): scripts/pmc_brick.sh <kernel regex> [brick_bench args...]
# (CUSZ_AMD_LIB selects a variant library)
export TMPDIR=/tmp
re=${1:-k_brick}; shift
mkdir -p gpurun_out/pmc
P=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL"
 "SQ_IFETCH SQ_INSTS_VMEM_RD SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_WR"
 "SQC_ICACHE_MISSES SQC_ICACHE_HITS"
 "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
 "FETCH_SIZE"
 "WRITE_SIZE"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-include-regex "$re" --pmc $p -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 scripts/brick_bench.py --reps 2 --dbg 0 "$@" > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; continue; }
  python3 scripts/pmc_summary.py "$(find gpurun_out/pmc/p$i -name "*counter_collection.csv" | head -1)" > gpurun_out/pmc/s$i.txt || exit 1
  rm -rf gpurun_out/pmc/p$i
done
cat gpurun_out/pmc/s*.txt
