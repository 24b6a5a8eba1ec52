#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on a bench
# workload (BENCH_ARGS, default the config-3 bppm bench): per-dispatch counters.
# usage: tools/gpu_pmc_outside.sh <tag>
set -e
tag=${1:-pmco}
BENCH_ARGS=${BENCH_ARGS:---bppm}
D=gpurun_out/$tag
mkdir -p $D
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d $D/p$i -o g$i --output-format csv -- python bench.py $BENCH_ARGS --steps 2 --warmup 1 --no-cpu-baseline > $D/log$i.txt 2>&1
done
