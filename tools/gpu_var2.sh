#!/bin/bash
# timing of product-flag variants (tools/build_ablate.sh VARIANTS): full-fold
# latency per variant, then stamps of the stamp variants
set -e
tag=${1:-var}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
for v in ${VARIANTS}; do
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/$tag/lat_$v.txt 2>&1
done
for v in ${SVARIANTS}; do
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/cells_stamps.py 100 4096 > gpurun_out/$tag/st_$v.txt 2>&1
done
