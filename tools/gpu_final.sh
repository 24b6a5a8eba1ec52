#!/bin/bash
# Round-end evidence on one MI355X: bench lines of the four workloads (MFE
# default, PF, config 3 pf + bppm, config 4 pf + bppm at N = 150) with a
# rocprofv3 kernel-trace summary each.
# usage: tools/gpu_final.sh <tag>
set -e
D=gpurun_out/${1:-final}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --fold pf > $D/bench_pf.json 2> $D/bench_pf.err
timeout -k 10 300 python bench.py --bppm > $D/bench_c3.json 2> $D/bench_c3.err
timeout -k 10 300 python bench.py --bppm --length 150 --steps 10 --warmup 2 --no-cpu-baseline > $D/bench_c4.json 2> $D/bench_c4.err
for w in "mfe:" "pf:--fold pf" "c3:--bppm" "c4:--bppm --length 150"; do
  n=${w%%:*}; args=${w#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace_$n -o $n -- python bench.py $args --steps 20 --warmup 2 --no-cpu-baseline > $D/trace_$n.json 2> $D/trace_$n.err
done
