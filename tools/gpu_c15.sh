set -e
mkdir -p gpurun_out/c15
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/c15/bench.json 2> gpurun_out/c15/bench.err
ADX_NO_INCR=1 timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/c15/bench_noincr.json 2> gpurun_out/c15/bench_noincr.err
