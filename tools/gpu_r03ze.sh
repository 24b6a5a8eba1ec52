#!/bin/bash
# MFE: count + speculative record in one LDS round trip (lib_spec) vs the product (lib_et)
set -e
D=gpurun_out/r03ze
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
for v in et spec mfe_lw7 mfe_lw7s; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-sub-records > $D/mfe_${v}_$k.json 2> $D/mfe_${v}_$k.err
done
done
ADX_LIB=addapt_amd/_lib/ablate/lib_spec.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mfe.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest_spec.log 2>&1
