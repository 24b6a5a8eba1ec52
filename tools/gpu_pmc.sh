#!/bin/bash
# PMC passes on the 4096-walker score path (separate passes, kernel-trace only).
# usage: tools/gpu_pmc.sh [tag]   -> gpurun_out/pmc_<tag>/
set -e
tag=${1:-base}
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT"; do
  i=$((i+1))
  ADX_LIB=addapt_amd/_lib/ablate/lib_base.so timeout -k 10 200 rocprofv3 --pmc $grp -d gpurun_out/pmc_$tag -o g$i --output-format csv -- python tools/pf_latency.py --W 4096 --reps 1 >> gpurun_out/pmc_$tag.log 2>&1
done
