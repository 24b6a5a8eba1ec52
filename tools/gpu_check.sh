# quick GPU validation: parity tests + default bench (no CPU baseline)
set -e
tag=${1:-chk}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --fold pf > gpurun_out/$tag/bench_pf.json 2> gpurun_out/$tag/bench_pf.err
