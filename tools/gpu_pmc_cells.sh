#!/bin/bash
# PMC passes on the 4096-walker MFE score path (separate passes, kernel-trace only).
# usage: tools/gpu_pmc_cells.sh [tag]   (ADX_MFE_KERNEL from the environment)
set -e
tag=${1:-cells}
mkdir -p gpurun_out/pmc_$tag
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM_NORM"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp -d gpurun_out/pmc_$tag -o g$i --output-format csv -- python tools/pf_latency.py --W 4096 --reps 1 --fold mfe >> gpurun_out/pmc_$tag/log.txt 2>&1
done
