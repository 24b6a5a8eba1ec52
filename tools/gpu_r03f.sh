#!/bin/bash
# config-4 kernels after the outside M pipelining: ring tests, config-4 bench,
# kernel stats, pf_ring stamps
set -e
D=gpurun_out/${1:-r03f}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_bppm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest_ring.log 2>&1
timeout -k 10 300 python bench.py --bppm --length 150 --steps 60 --warmup 3 --no-cpu-baseline --no-sub-records > $D/c4.json 2> $D/c4.err
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 200 python tools/ring_stamps.py 150 4096 3 > $D/ring_stamps.txt 2>&1
