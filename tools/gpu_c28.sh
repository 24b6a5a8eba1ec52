set -e
mkdir -p gpurun_out/c28
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
ADX_LIB=addapt_amd/_lib/ablate/lib_r1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mfe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/c28/pytest_mfe_r1.log 2>&1
bash tools/gpu_c21.sh
