set -e
mkdir -p gpurun_out/bppm2
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_bppm.py -q -x -p no:cacheprovider > gpurun_out/bppm2/pytest_bppm.log 2>&1
timeout -k 10 300 python bench.py --bppm --no-cpu-baseline > gpurun_out/bppm2/bench_bppm100.json 2> gpurun_out/bppm2/bench_bppm100.err
timeout -k 10 400 python bench.py --bppm --length 150 --no-cpu-baseline --steps 10 > gpurun_out/bppm2/bench_bppm150.json 2> gpurun_out/bppm2/bench_bppm150.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bppm2/trace -o bppm -- python bench.py --bppm --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bppm2/trace.json 2> gpurun_out/bppm2/trace.err
