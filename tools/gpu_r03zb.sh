#!/bin/bash
# MFE 4-lane partition seeds / list-role wave (tools/build_mfe_roles.sh) vs the product (lib_et)
set -e
D=gpurun_out/${TAG:-r03zb}
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
for v in ${VARS:-et mfe_x2 mfe_x3 mfe_lw2}; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-sub-records > $D/mfe_${v}_$k.json 2> $D/mfe_${v}_$k.err
done
done
