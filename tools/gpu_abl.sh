#!/bin/bash
# Ablation sweep: for each ADX_LIB variant in $VARIANTS, MFE stamps + MFE bench
set -e
D=gpurun_out/${1:-abl}
mkdir -p $D
export TMPDIR=/tmp
for v in ${VARIANTS:-sbase}; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python tools/mfe_mc_stamps.py > $D/stamps_$v.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline --no-sub-records > $D/bench_$v.json 2> $D/bench_$v.err
done
