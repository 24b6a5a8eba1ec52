#!/bin/bash
# fold latency of build variants (tools/build_ablate.sh), each run twice
# usage: VARIANTS="b0 t1 ..." tools/gpu_lat_variants.sh <tag>
set -e
tag=${1:-lv}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
for v in $VARIANTS $VARIANTS; do ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/pf_latency.py --fold mfe >> gpurun_out/$tag/lat.txt 2>&1; done
