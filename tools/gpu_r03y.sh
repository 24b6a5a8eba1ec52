#!/bin/bash
# MFE per-slice energy table (lib_et) against the committed blocks (lib_base), then its parity
set -e
D=gpurun_out/r03y
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
for v in base et; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-sub-records > $D/mfe_${v}_$k.json 2> $D/mfe_${v}_$k.err
done
done
ADX_LIB=addapt_amd/_lib/ablate/lib_et.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mfe.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest_et.log 2>&1
