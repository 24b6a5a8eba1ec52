#!/bin/bash
# PF-side parity (pf_cells, pf_ring, bppm, full-size) + PF and config-4 benches
set -e
D=gpurun_out/${1:-r03s}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_bppm.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 300 python bench.py --fold pf --steps 100 --no-cpu-baseline --no-sub-records > $D/pf.json 2> $D/pf.err
timeout -k 10 300 python bench.py --bppm --steps 100 --no-cpu-baseline --no-sub-records > $D/c3.json 2> $D/c3.err
timeout -k 10 300 python bench.py --bppm --length 150 --steps 60 --warmup 3 --no-cpu-baseline --no-sub-records > $D/c4.json 2> $D/c4.err
