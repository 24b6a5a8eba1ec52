# lanes = cells MFE kernel: parity tests (MFE files first), then both kernels' latency and the bench
set -e
tag=${1:-m2}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mfe.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_mfe.log 2>&1
timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/$tag/lat_cells.txt 2>&1
ADX_MFE_KERNEL=rows timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/$tag/lat_rows.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_all.log 2>&1
