#!/bin/bash
# Round evidence on one MI355X: parity tests, smoke, the default bench line
# (MFE, BASELINE configs[1], with the CPU baseline) and the PF bench line, a
# rocprofv3 kernel-trace summary of the default bench and the two PMC traffic
# passes.   usage: tools/gpu_profile.sh <round-tag>
set -e
tag=${1:-r01}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/$tag/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
timeout -k 10 600 python bench.py --fold pf > gpurun_out/$tag/bench_pf.json 2> gpurun_out/$tag/bench_pf.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/trace -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$tag/trace_bench.json 2> gpurun_out/$tag/trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$tag/pmc_fetch -o fetch --output-format csv -- python bench.py --steps 3 --warmup 0 --no-cpu-baseline > gpurun_out/$tag/pmc_fetch.out 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$tag/pmc_write -o write --output-format csv -- python bench.py --steps 3 --warmup 0 --no-cpu-baseline > gpurun_out/$tag/pmc_write.out 2>&1
python tools/pmc_traffic.py $(find gpurun_out/$tag/pmc_fetch -name "*counter_collection.csv") $(find gpurun_out/$tag/pmc_write -name "*counter_collection.csv") > gpurun_out/$tag/traffic.json
python tools/trace_summary.py $(find gpurun_out/$tag/trace -name "*kernel_trace.csv") --last 10 > gpurun_out/$tag/score_kernel_summary.json
