#!/bin/bash
# cells MFE kernel: parity tests, fold latency, stamps (stamp build), short bench.
# usage: tools/gpu_cells_check.sh <tag>   (build lib_s1.so first: VARIANTS="s1:-DADX_STAMP" tools/build_ablate.sh)
set -e
tag=${1:-cc}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_mfe.log 2>&1
timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/$tag/lat.txt 2>&1
ADX_NWV=8 ADX_LIB=addapt_amd/_lib/ablate/lib_s1.so timeout -k 10 120 python tools/cells_stamps.py 100 4096 > gpurun_out/$tag/st4096.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
