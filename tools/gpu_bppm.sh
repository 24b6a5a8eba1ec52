#!/bin/bash
# BASELINE configs 3/4 (pf + bppm score) on one MI355X: the outside-pass GPU
# tests, bench lines and a rocprofv3 kernel-trace summary of config 3.
# usage: tools/gpu_bppm.sh <tag>
set -e
tag=${1:-bppm}
D=gpurun_out/$tag
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bppm.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 300 python bench.py --bppm --steps 30 --no-cpu-baseline > $D/bench_c3.json 2> $D/bench_c3.err
timeout -k 10 300 python bench.py --bppm --length 150 --steps 10 --no-cpu-baseline > $D/bench_c4.json 2> $D/bench_c4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o c3 -- python bench.py --bppm --steps 5 --warmup 1 --no-cpu-baseline > $D/trace_c3.json 2> $D/trace_c3.err
