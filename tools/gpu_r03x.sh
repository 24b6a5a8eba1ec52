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
# product build: PF / config 4 with the qm column recursion, ring + PF parity
timeout -k 10 200 python bench.py --fold pf --steps 100 --no-cpu-baseline --no-sub-records > $D/pf_product.json 2> $D/pf_product.err
timeout -k 10 200 python bench.py --bppm --length 150 --steps 40 --warmup 3 --no-cpu-baseline --no-sub-records > $D/c4_product.json 2> $D/c4_product.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest_ring.log 2>&1
