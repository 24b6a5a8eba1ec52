#!/bin/bash
# instruction-cache PMC passes on the 4096-walker MFE folds (one small pass each)
set -e
tag=${1:-ic}
mkdir -p gpurun_out/pmc_$tag
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
i=0
for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" "SQC_ICACHE_BUSY_CYCLES SQC_TC_INST_REQ" "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp -d gpurun_out/pmc_$tag -o g$i --output-format csv -- python tools/pf_latency.py --W 4096 --reps 1 --fold mfe >> gpurun_out/pmc_$tag/log.txt 2>&1
done
