#!/bin/bash
# MFE timing-only ablations (tools/build_mfe_abl.sh) against the product build
set -e
D=gpurun_out/r03x
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
for v in base mfe_nomask mfe_nosel mfe_noct; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-sub-records > $D/mfe_${v}_$k.json 2> $D/mfe_${v}_$k.err
done
done
