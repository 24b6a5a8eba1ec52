#!/bin/bash
# A/B builds of the engine into addapt_amd/_lib/ablate/lib_<name>.so: each spec
# name=<git rev or "tree">:<kernel files, comma-separated>:<flags> replaces those
# kernel sources by their version at that revision (the rest is the working
# tree; host code and headers always from the tree) and adds the flags
# ("__" for spaces); generated includes (*.inc) in the list are replaced too.  Select one with ADX_LIB=addapt_amd/_lib/ablate/lib_<name>.so
# (tools/gpu_run.sh "libs" step).
#   tools/build_ab.sh new=tree:mfe_cells.hip: old=HEAD:mfe_cells.hip: stamp=tree:mfe_cells.hip:-DADX_STAMP
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/addapt_amd/csrc
OUT=$ROOT/addapt_amd/_lib/ablate
mkdir -p $OUT
T=$(mktemp -d)
H="hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC"
$H -c $SRC/adx_api.cpp -o $OUT/api.o &
$H -c $SRC/energy.cpp -o $OUT/energy.o &
for f in kernels.hip mfe_cells.hip mfe_pair.hip outside_cells.hip pf_cells.hip pf_ring.hip outside_ring.hip; do
  $H -c $SRC/$f -o $OUT/tree_${f%.hip}.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}; rest=${spec#*=}
  IFS=: read -r rev file flags <<< "$rest"
  flags=${flags//__/ }
  mkdir -p $T/$name
  cp $SRC/* $T/$name/
  files=${file//,/ }
  if [ "$rev" != "tree" ]; then
    for f in $files; do git -C $ROOT show $rev:addapt_amd/csrc/$f > $T/$name/$f; done
  fi
  (
  for f in $files; do case $f in *.hip) $H $flags -c $T/$name/$f -o $OUT/${name}_${f%.hip}.o ;; esac; done
  objs=""
  for f in kernels mfe_cells mfe_pair outside_cells pf_cells pf_ring outside_ring; do
    if [[ " $files " == *" $f.hip "* ]]; then objs="$objs $OUT/${name}_$f.o"; else objs="$objs $OUT/tree_$f.o"; fi
  done
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$name.so $objs $OUT/api.o $OUT/energy.o
  ) &
done
wait
rm -rf $T
