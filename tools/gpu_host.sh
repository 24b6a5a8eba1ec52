set -e
mkdir -p gpurun_out/h
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_host_gpu.py -q -x -p no:cacheprovider > gpurun_out/h/pytest.log 2>&1
