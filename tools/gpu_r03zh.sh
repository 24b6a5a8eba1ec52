#!/bin/bash
# Final tree: GPU suite, smoke, default bench line
set -e
D=gpurun_out/r03zh
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest_gpu.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.txt 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err
