set -e
mkdir -p gpurun_out/i
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/i/b_on.json 2> gpurun_out/i/b_on.err
ADX_NO_INCR=1 timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/i/b_off.json 2> gpurun_out/i/b_off.err
