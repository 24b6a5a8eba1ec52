#!/bin/bash
# Round-3 evidence (late): bench lines of the four workloads (default line with
# sub-records; traffic from profiles/traffic_latest_*.json) and a rocprofv3
# kernel-trace summary each, plus smoke()
set -e
D=gpurun_out/${1:-r03zd}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $D/bench_mfe.json 2> $D/bench_mfe.err
timeout -k 10 300 python bench.py --fold pf --no-sub-records > $D/bench_pf.json 2> $D/bench_pf.err
timeout -k 10 300 python bench.py --bppm --no-sub-records > $D/bench_c3.json 2> $D/bench_c3.err
timeout -k 10 300 python bench.py --bppm --length 150 --steps 60 --warmup 3 --no-cpu-baseline --no-sub-records > $D/bench_c4.json 2> $D/bench_c4.err
for w in "mfe:" "pf:--fold pf" "c3:--bppm" "c4:--bppm --length 150"; do
  n=${w%%:*}; args=${w#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace_$n -o $n -- python bench.py $args --steps 20 --warmup 2 --no-cpu-baseline --no-sub-records > $D/trace_$n.json 2> $D/trace_$n.err
done
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.txt 2>&1
