#!/bin/bash
# One LDS-counter pass (bank conflicts, LDS-active cycles, LDS / VALU
# instructions) of the default bench for each ablate build lib_<v>.so.
# usage: tools/lds_pmc.sh <tag> <variant>...
set -e
tag=$1; shift
D=gpurun_out/$tag
mkdir -p $D
export TMPDIR=/tmp
for v in "$@"; do
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace \
    --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU -d $D/lds_$v -o c --output-format csv \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub-records > $D/lds_$v.log 2>&1
done
