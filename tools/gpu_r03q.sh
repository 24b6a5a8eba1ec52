#!/bin/bash
# MFE: parity tests + bench of the product lib, then stamps + bench of the
# list-wave placement variants (stamp = wave 7, lw2, lw0)
set -e
D=gpurun_out/${1:-r03q}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfe.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-sub-records > $D/mfe.json 2> $D/mfe.err
for v in stamp lw2 lw0; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python tools/mfe_mc_stamps.py > $D/stamps_$v.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --steps 60 --no-cpu-baseline --no-sub-records > $D/bench_$v.json 2> $D/bench_$v.err
done
