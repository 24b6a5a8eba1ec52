#!/bin/bash
# Round-3 evidence, part B: bench lines of the four workloads (traffic from
# profiles/traffic_latest_*.json) and a rocprofv3 kernel-trace summary each
set -e
D=gpurun_out/${1:-r03fb}
mkdir -p $D
export TMPDIR=/tmp
WORKLOADS=mfe bash tools/gpu_traffic.sh ${1:-r03fb}/tr
cp $D/tr/traffic_latest_mfe.json profiles/traffic_latest_mfe.json
timeout -k 10 300 python bench.py > $D/bench_mfe.json 2> $D/bench_mfe.err
timeout -k 10 300 python bench.py --fold pf --no-sub-records > $D/bench_pf.json 2> $D/bench_pf.err
timeout -k 10 300 python bench.py --bppm --no-sub-records > $D/bench_c3.json 2> $D/bench_c3.err
timeout -k 10 300 python bench.py --bppm --length 150 --steps 60 --warmup 3 --no-cpu-baseline --no-sub-records > $D/bench_c4.json 2> $D/bench_c4.err
for w in "mfe:" "pf:--fold pf" "c3:--bppm" "c4:--bppm --length 150"; do
  n=${w%%:*}; args=${w#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace_$n -o $n -- python bench.py $args --steps 20 --warmup 2 --no-cpu-baseline --no-sub-records > $D/trace_$n.json 2> $D/trace_$n.err
done
