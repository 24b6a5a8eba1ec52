#!/bin/bash
# MFE B-block changes: MFE parity + full-size tests, MFE bench, MFE stamps
set -e
D=gpurun_out/${1:-r03o}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfe.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-sub-records > $D/mfe.json 2> $D/mfe.err
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 200 python tools/mfe_mc_stamps.py > $D/mfe_stamps.txt 2>&1
