# full GPU test suite + MFE/PF/bppm benches
set -e
mkdir -p gpurun_out/f
export TMPDIR=/tmp
rm -f gpurun_out/f/*
timeout -k 10 600 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/f/pytest.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/f/bench.json 2> gpurun_out/f/bench.err
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --fold pf > gpurun_out/f/bench_pf.json 2> gpurun_out/f/bench_pf.err
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --bppm > gpurun_out/f/bench_bppm.json 2> gpurun_out/f/bench_bppm.err
