#!/bin/bash
# PMC passes on the 1-walker score path (separate passes, kernel-trace only).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base none; do
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE"; do
  tag=$(echo $grp | cut -c1-12 | tr ' ' '_')
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 rocprofv3 --pmc $grp -d gpurun_out/pmc_$v -o $tag --output-format csv -- python tools/pf_latency.py --W 1 --reps 2 >> gpurun_out/pmc.log 2>&1
done
done
