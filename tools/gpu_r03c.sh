#!/bin/bash
# ring-kernel tests first (new kernel), then the whole GPU suite and the default bench
set -e
D=gpurun_out/${1:-r03c}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ring.py tests/test_gpu_bppm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest_ring.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 600 python bench.py > $D/bench.json 2> $D/bench.err
