#!/bin/bash
# A/B of two library variants ($A, $B) on the PF, config-3 and config-4 benches
set -e
D=gpurun_out/${1:-ab3}
mkdir -p $D
export TMPDIR=/tmp
for v in $A $B; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --fold pf --steps 100 --no-cpu-baseline --no-sub-records > $D/bench_${v}pf_1.json 2> $D/${v}pf.err
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --bppm --steps 100 --no-cpu-baseline --no-sub-records > $D/bench_${v}c3_1.json 2> $D/${v}c3.err
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --bppm --length 150 --steps 40 --warmup 3 --no-cpu-baseline --no-sub-records > $D/bench_${v}c4_1.json 2> $D/${v}c4.err
done
