#!/bin/bash
# PF: the U column helper on the Q wave (pb, product) or on qm waves 12 / 13
set -e
D=gpurun_out/r03zg
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
for v in pb u12 u13; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --fold pf --steps 100 --no-cpu-baseline --no-sub-records > $D/pf_${v}_$k.json 2> $D/pf_${v}_$k.err
done
done
