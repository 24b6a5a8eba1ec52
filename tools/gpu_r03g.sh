#!/bin/bash
# PF-side changes (M items round-robin, ring prep on an M wave): PF + ring
# parity tests, PF and config-4 benches, ring stamps
set -e
D=gpurun_out/${1:-r03g}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_bppm.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 300 python bench.py --fold pf --steps 100 --no-cpu-baseline --no-sub-records > $D/pf.json 2> $D/pf.err
timeout -k 10 300 python bench.py --bppm --length 150 --steps 60 --warmup 3 --no-cpu-baseline --no-sub-records > $D/c4.json 2> $D/c4.err
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 200 python tools/ring_stamps.py 150 4096 3 > $D/ring_stamps.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 200 python tools/outside_stamps.py 150 4096 3 > $D/outside_ring_stamps.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 200 python tools/pf_cells_stamps.py > $D/pf_cells_stamps.txt 2>&1
