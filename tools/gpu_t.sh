set -e
mkdir -p gpurun_out/t
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider -k incremental > gpurun_out/t/pytest.log 2>&1
