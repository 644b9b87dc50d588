#!/bin/bash
# PMC passes over the decoder micro-benchmark: scripts/pmc_dec.sh KIND [SUBLEN]
export TMPDIR=/tmp
K=${1:-3}; S=${2:-1024}
mkdir -p gpurun_out/pmc
P=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"
 "TCP_PENDING_STALL_CYCLES TCP_TCC_WRITE_REQ TCP_TCC_READ_REQ TCP_TOTAL_CACHE_ACCESSES GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0
for p in "${P[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-include-regex "k_hf_decode" --pmc $p -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 scripts/dec_bench.py 512x512x512 1e-4 $S $K > gpurun_out/pmc/p$i.log 2>&1 || exit 1
done
python3 scripts/pmc_kernel.py k_hf_decode gpurun_out/pmc/p1 gpurun_out/pmc/p2 gpurun_out/pmc/p3; rm -rf gpurun_out/pmc
