#!/bin/bash
# GPU probe: parity tests, ablation latencies, bench (gpurun helper).
mkdir -p gpurun_out
set -e
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu --timeout=300 -p no:cacheprovider -x > gpurun_out/t.log 2>&1; echo rc=$? >> gpurun_out/t.log
for v in base nogen noml nospec none; do
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/pf_latency.py >> gpurun_out/abl.txt 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err
