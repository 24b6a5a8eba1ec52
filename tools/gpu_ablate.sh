#!/bin/bash
# latency / throughput of every diagnostic variant in addapt_amd/_lib/ablate

mkdir -p gpurun_out
rm -f gpurun_out/abl.txt
for f in addapt_amd/_lib/ablate/lib_*.so; do
  ADX_LIB=$f timeout -k 10 120 python tools/pf_latency.py >> gpurun_out/abl.txt 2>&1
done
