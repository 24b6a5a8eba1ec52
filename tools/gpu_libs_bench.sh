#!/bin/bash
# A/B of engine library variants: the default (MFE) bench, interleaved, twice
# usage: VARIANTS="va vb" tools/gpu_libs_bench.sh <tag> [bench args]
set -e
D=gpurun_out/${1:-libs}
shift || true
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
for v in $VARIANTS; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-sub-records "$@" > $D/bench_${v}_$k.json 2> $D/bench_${v}_$k.err
done
done
