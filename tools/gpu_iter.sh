#!/bin/bash
# one GPU iteration: parity tests -> latency of every diagnostic variant -> stamps -> bench
set -e
mkdir -p gpurun_out
rm -f gpurun_out/abl.txt gpurun_out/stamp.txt gpurun_out/b.json
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -q -m gpu --timeout=300 -p no:cacheprovider -x > gpurun_out/t.log 2>&1
for f in addapt_amd/_lib/ablate/lib_*.so; do
  ADX_LIB=$f timeout -k 10 120 python tools/pf_latency.py >> gpurun_out/abl.txt 2>&1 || true
done
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/pf_stamps.py > gpurun_out/stamp.txt 2>&1 || true
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err
