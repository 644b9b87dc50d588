#!/bin/bash
# SQ counter passes over the sampled-mode kernels (k_brick3_stream, k_brick3_sample) of the
# config-2 single_bench run (diagnostic):  scripts/pmc_stream.sh <kernel-regex> <tag>
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
re=$1; tag=$2
mkdir -p gpurun_out/$tag
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA TA_TA_BUSY TA_BUFFER_WAVEFRONTS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-include-regex "$re" --pmc $ctr -d gpurun_out/$tag/p$i -o run --output-format csv -- python3 scripts/single_bench.py > gpurun_out/$tag/p$i.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py "$(find gpurun_out/$tag/p$i -name '*counter_collection.csv' | head -1)" > gpurun_out/$tag/p$i.summary
  rm -rf gpurun_out/$tag/p$i
done
cat gpurun_out/$tag/p*.summary
