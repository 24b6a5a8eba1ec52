# four-fold MFE kernel: MFE parity tests, latency of quad vs cells, bench
set -e
tag=${1:-q}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
ADX_MFE_KERNEL=quad timeout -k 10 300 python -u -m pytest tests/test_gpu_mfe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_mfe.log 2>&1
ADX_MFE_KERNEL=quad timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/$tag/lat.txt 2>&1
ADX_MFE_KERNEL=cells timeout -k 10 120 python tools/pf_latency.py --fold mfe >> gpurun_out/$tag/lat.txt 2>&1
ADX_MFE_KERNEL=quad timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
