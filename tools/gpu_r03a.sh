#!/bin/bash
# Round-3 start: GPU suite, default bench, PMC passes of mfe_cells_kernel.
set -e
D=gpurun_out/r03a
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err
BENCH_ARGS="--fold mfe" bash tools/gpu_pmc.sh r03a/pmc_mfe
