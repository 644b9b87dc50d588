#!/bin/bash
# SQ/LDS/TA counter passes over one kernel of the config-2 brick_bench run (diagnostic):
#   scripts/pmc_kern.sh <kernel-regex> <tag> [lib dir] [driver script, default scripts/brick_bench.py] [driver args]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export CUSZ_AMD_NO_GATE=1  # counter passes serialise dispatches (see pmc_config.sh)
re=$1; tag=$2; lib=${3:-cusz_amd/lib}; drv=${4:-scripts/brick_bench.py}; shift $(( $# < 4 ? $# : 4 )); extra="$@"
mkdir -p gpurun_out/$tag
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA TA_TA_BUSY TA_BUFFER_WAVEFRONTS GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  CUSZ_AMD_LIB=$lib/libcusz_amd.so timeout -s KILL 90 rocprofv3 --kernel-include-regex "$re" --pmc $ctr -d gpurun_out/$tag/p$i -o run --output-format csv -- python3 $drv --reps 2 $extra > gpurun_out/$tag/p$i.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py "$(find gpurun_out/$tag/p$i -name '*counter_collection.csv' | head -1)" > gpurun_out/$tag/p$i.summary
  rm -rf gpurun_out/$tag/p$i
done
cat gpurun_out/$tag/p*.summary
