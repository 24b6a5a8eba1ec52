#!/bin/bash
# GPU suite (incl. the multi-rank and full-size tests) + the default bench line
# with its sub-records; logs under gpurun_out/$1
set -e
D=gpurun_out/${1:-r03b}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err
