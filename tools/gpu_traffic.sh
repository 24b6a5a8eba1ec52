#!/bin/bash
# HBM traffic per step (FETCH_SIZE / WRITE_SIZE, one counter per rocprofv3
# pass, MI355X_MICROARCH.md HBM corrections in tools/pmc_traffic.py) of the
# bench workloads: mfe, pf, pf + bppm at N = 100 and 150.
# usage: [WORKLOADS="pf pf_bppm"] tools/gpu_traffic.sh <tag>   -> gpurun_out/<tag>/traffic_latest_*.json
set -e
tag=${1:-traffic}
D=gpurun_out/$tag
mkdir -p $D
export TMPDIR=/tmp
run() {   # name, dominant kernel (roofline.traffic; "" = the most bytes), bench args
  local n=$1; local dk=$2; shift 2
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $D/$n/f -o f --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records "$@" > $D/$n.fetch.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $D/$n/w -o w --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records "$@" > $D/$n.write.log 2>&1
  python tools/pmc_traffic.py $(find $D/$n/f -name "*counter_collection.csv") $(find $D/$n/w -name "*counter_collection.csv") $dk > $D/traffic_latest_$n.json
}
W=${WORKLOADS:-"mfe pf pf_bppm pf_bppm_n150"}
for n in $W; do
  case $n in
    mfe) run mfe mfe_cells_kernel ;;
    pf) run pf pf_cells_kernel --fold pf ;;
    pf_bppm) run pf_bppm outside_cells_kernel --bppm ;;
    pf_bppm_n150) run pf_bppm_n150 outside_ring_kernel --bppm --length 150 ;;
  esac
done
