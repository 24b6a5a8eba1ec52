# full GPU suite with each MFE kernel, then the default bench
set -e
tag=${1:-all}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_cells.log 2>&1
ADX_MFE_KERNEL=quad timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_quad.log 2>&1
ADX_MFE_KERNEL=rows timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_rows.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
