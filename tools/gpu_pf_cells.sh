#!/bin/bash
# pf_cells_kernel on one MI355X: PF bench (cells vs rows kernel), config 3
# (pf + bppm), a rocprofv3 kernel-trace summary of the PF bench and the
# per-wave stamps (tools/build_ablate.sh stamp build).
# usage: tools/gpu_pf_cells.sh <tag>
set -e
D=gpurun_out/${1:-pfc}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --fold pf --steps 100 --no-cpu-baseline > $D/pf_cells.json 2> $D/pf_cells.err
ADX_PF_KERNEL=rows timeout -k 10 200 python bench.py --fold pf --steps 60 --no-cpu-baseline > $D/pf_rows.json 2> $D/pf_rows.err
timeout -k 10 200 python bench.py --bppm --steps 60 --no-cpu-baseline > $D/c3.json 2> $D/c3.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o pf -- python bench.py --fold pf --steps 10 --warmup 1 --no-cpu-baseline > $D/trace_pf.json 2> $D/trace_pf.err
if [ -f addapt_amd/_lib/ablate/lib_stamp.so ]; then
  ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 200 python tools/pf_cells_stamps.py > $D/stamps.txt 2>&1
fi
