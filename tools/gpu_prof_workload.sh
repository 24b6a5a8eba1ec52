#!/bin/bash
# One workload on one MI355X: rocprofv3 kernel-trace summary, PMC passes (one
# counter group per run), HBM traffic (FETCH_SIZE / WRITE_SIZE passes).
# usage: tools/gpu_prof_workload.sh <tag> <traffic-name> <bench args...>
set -e
tag=$1; tname=$2; shift 2
D=gpurun_out/$tag
mkdir -p $D
export TMPDIR=/tmp
B="--steps 3 --warmup 1 --no-cpu-baseline --no-sub-records"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o k -- python bench.py "$@" --steps 10 --warmup 2 --no-cpu-baseline --no-sub-records > $D/trace.json 2> $D/trace.err
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $D/p$i -o g$i --output-format csv -- python bench.py "$@" $B > $D/log$i.txt 2>&1
done
python tools/pmc_traffic.py $(find $D/p4 -name "*counter_collection.csv") $(find $D/p5 -name "*counter_collection.csv") > $D/traffic_latest_$tname.json
