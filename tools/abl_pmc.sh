#!/bin/bash
# LDS counters of ablation builds (addapt_amd/_lib/ablate/lib_<v>.so): one
# rocprofv3 pass per build with the LDS counters only, plus a short bench
# (results of ablation builds are wrong by design: timing / counters only).
# usage: tools/abl_pmc.sh <tag> <variant>...
set -e
tag=$1; shift
D=gpurun_out/$tag
mkdir -p $D
export TMPDIR=/tmp
for v in "$@"; do
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace \
    --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU -d $D/abl_$v -o c --output-format csv \
    -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-sub-records > $D/abl_$v.log 2>&1
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --steps 60 --warmup 5 \
    --no-cpu-baseline --no-sub-records > $D/abl_$v.json 2> $D/abl_$v.err
done
