#!/bin/bash
# LDS PMC (bank conflicts, LDS-active cycles, instructions) of library variants ($VARIANTS) on one bench workload ($BENCH_ARGS)
set -e
D=gpurun_out/${1:-pmcab}
mkdir -p $D
export TMPDIR=/tmp
for v in $VARIANTS; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d $D/$v -o p --output-format csv -- python bench.py $BENCH_ARGS --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records > $D/$v.log 2>&1
done
