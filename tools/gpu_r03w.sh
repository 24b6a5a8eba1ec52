#!/bin/bash
# PF qm-item variants: qm waves (4 / 6) x unpaired part by column recursion; then
# the parity tests on the m6u library
set -e
D=gpurun_out/r03w
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
for v in base urec m6 m6u; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --fold pf --steps 100 --no-cpu-baseline --no-sub-records > $D/pf_${v}_$k.json 2> $D/pf_${v}_$k.err
done
done
for v in base m6u; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --bppm --steps 100 --no-cpu-baseline --no-sub-records > $D/c3_${v}.json 2> $D/c3_${v}.err
done
ADX_LIB=addapt_amd/_lib/ablate/lib_m6u.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bppm.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest_m6u.log 2>&1
