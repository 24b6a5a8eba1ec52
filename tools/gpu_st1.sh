#!/bin/bash
# stamps of the given stamp variants at W=1 and W=4096
set -e
tag=${1:-st1}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
for v in ${SVARIANTS}; do
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/cells_stamps.py 100 1 > gpurun_out/$tag/st1_$v.txt 2>&1
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/cells_stamps.py 100 4096 > gpurun_out/$tag/st4096_$v.txt 2>&1
done
