set -e
mkdir -p gpurun_out/c29
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/c29/pytest_mfe.log 2>&1
ADX_MFE_KERNEL=quad timeout -k 10 300 python -u -m pytest tests/test_gpu_mfe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k mlbase > gpurun_out/c29/pytest_mfe_quad.log 2>&1
ADX_MFE_KERNEL=rows timeout -k 10 300 python -u -m pytest tests/test_gpu_mfe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k mlbase > gpurun_out/c29/pytest_mfe_rows.log 2>&1
