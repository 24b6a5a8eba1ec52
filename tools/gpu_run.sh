#!/bin/bash
# One parameterised GPU run (the command gpurun executes on the MI355X box).
# Every step runs under its own time limit; the first failure ends the script.
#
# usage: tools/gpu_run.sh <tag> <step> [<step> ...]     -> gpurun_out/<tag>/
#   pytest:<name>:<pytest args>     e.g. 'pytest:mfe:tests/test_gpu_mfe.py -k auto'
#   suite                           the whole -m gpu suite (pytest_gpu.txt)
#   smoke                           __graft_entry__.smoke()
#   bench:<name>:<bench.py args>    one bench line -> <name>.json
#   prof:<name>:<bench.py args>     rocprofv3 --kernel-trace --stats of a bench run
#   pmc:<name>:<bench.py args>      three PMC passes (SQ occupancy / instruction
#                                   mix / LDS), kernel trace only, per dispatch
#   pmcx:<name>:<counters,...>:<bench.py args>   one PMC pass of the listed counters
#   traffic:<name>:<kernel>:<bench.py args>   FETCH_SIZE + WRITE_SIZE passes ->
#                                   traffic_latest_<name>.json (tools/pmc_traffic.py)
#   py:<name>:<script args>         a tools/ script (e.g. 'py:stamp_mfe:tools/pf_stamps.py 100 mfe';
#                                   ADX_LIB=<.so> in the environment selects an ablate build)
#   libs:<name>:<variants>:<bench.py args>    interleaved A/B of engine builds in
#                                   addapt_amd/_lib/ablate/lib_<variant>.so (tools/build_ablate.sh)
set -e
tag=${1:?tag}
shift
D=gpurun_out/$tag
mkdir -p $D
export TMPDIR=/tmp
T=${STEP_TIMEOUT:-300}
for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  name=${rest%%:*}
  args=${rest#*:}
  [ "$rest" = "$step" ] && { name=$kind; args=; }
  echo "[$(date +%T)] $step"
  case $kind in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $D/pytest_gpu.txt 2>&1 ;;
    pytest)
      timeout -k 10 $T python -u -m pytest -x -v --timeout 240 --timeout-method thread \
        -p no:cacheprovider $args > $D/pytest_$name.txt 2>&1 ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.txt 2>&1 ;;
    bench)
      timeout -k 10 $T python bench.py $args > $D/$name.json 2> $D/$name.err ;;
    prof)
      timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$name -o $name \
        -- python bench.py $args > $D/prof_$name.json 2> $D/prof_$name.err ;;
    pmc)
      i=0
      for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                 "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
                 "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC"; do
        i=$((i+1))
        timeout -k 10 120 rocprofv3 --pmc $grp -d $D/pmc_$name/p$i -o g$i --output-format csv \
          -- python bench.py $args --steps 2 --warmup 1 --no-cpu-baseline --no-sub-records > $D/pmc_${name}_$i.txt 2>&1
      done ;;
    pmcx)   # one PMC pass of the given counters: pmcx:<name>:<counters, comma-separated>:<bench.py args>
      ctrs=${args%%:*}
      bargs=${args#*:}
      [ "$ctrs" = "$args" ] && bargs=
      timeout -k 10 120 rocprofv3 --pmc ${ctrs//,/ } -d $D/pmcx_$name -o x --output-format csv \
        -- python bench.py $bargs --steps 2 --warmup 1 --no-cpu-baseline --no-sub-records > $D/pmcx_$name.txt 2>&1 ;;
    traffic)
      kern=${args%%:*}
      bargs=${args#*:}
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 200 rocprofv3 --pmc $c -d $D/traffic_$name/$c -o $c --output-format csv \
          -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sub-records $bargs > $D/traffic_${name}_$c.log 2>&1
      done
      python tools/pmc_traffic.py $(find $D/traffic_$name/FETCH_SIZE -name "*counter_collection.csv") \
        $(find $D/traffic_$name/WRITE_SIZE -name "*counter_collection.csv") $kern > $D/traffic_latest_$name.json ;;
    py)
      timeout -k 10 $T python $args > $D/$name.txt 2>&1 ;;
    libs)
      variants=${args%%:*}
      bargs=${args#*:}
      [ "$variants" = "$args" ] && bargs=
      for k in $(seq ${REPS:-2}); do
        for v in $variants; do
          ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline \
            --no-sub-records $bargs > $D/${name}_${v}_$k.json 2> $D/${name}_${v}_$k.err
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$(date +%T)] done"
