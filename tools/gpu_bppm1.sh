set -e
mkdir -p gpurun_out/bppm1
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_bppm.py -q -x -p no:cacheprovider > gpurun_out/bppm1/pytest_bppm.log 2>&1
timeout -k 10 600 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/bppm1/pytest_gpu.log 2>&1
