#!/bin/bash
# timing-only ablations of the lanes = cells MFE kernel (tools/build_ablate.sh
# VARIANTS with -DMFE_ABL_*): kernel ms and per-wave phase cycles per variant
set -e
tag=${1:-abl}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
for v in ${VARIANTS:-stamp}; do
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/cells_stamps.py 100 4096 > gpurun_out/$tag/$v.txt 2>&1
done
