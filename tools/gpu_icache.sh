#!/bin/bash
# List the PMC counters, then one pass of instruction-cache counters on the MFE bench
set -e
D=gpurun_out/${1:-icache}
mkdir -p $D
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $D/counters.txt 2>&1 || true
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*" $D/counters.txt | sort -u > $D/sqc.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d $D/p1 -o g1 --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub-records > $D/log1.txt 2>&1
