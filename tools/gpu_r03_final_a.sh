#!/bin/bash
# Round-3 evidence, part A: the GPU suite, then HBM traffic (FETCH_SIZE /
# WRITE_SIZE passes) of the four bench workloads
set -e
D=gpurun_out/${1:-r03fa}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest_gpu.txt 2>&1
bash tools/gpu_traffic.sh ${1:-r03fa}/tr
