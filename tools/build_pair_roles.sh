#!/bin/bash
# mfe_pair_kernel role-cost variants: the 4-lanes-per-cell block partition seeded
# with other role costs (ADX_GEN_PAIR_ROLES4, "wave:cost,...") and mfe_pair.hip
# built with extra flags ("__" for spaces); every other source from the tree.
# usage: tools/build_pair_roles.sh name/PAIR_ROLES4/FLAGS ...  -> addapt_amd/_lib/ablate/lib_<name>.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/addapt_amd/csrc
OUT=$ROOT/addapt_amd/_lib/ablate
mkdir -p $OUT
T=$(mktemp -d)
H="hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC"
$H -c $SRC/adx_api.cpp -o $OUT/api.o &
$H -c $SRC/energy.cpp -o $OUT/energy.o &
for f in kernels.hip mfe_cells.hip outside_cells.hip pf_cells.hip pf_ring.hip outside_ring.hip; do
  $H -c $SRC/$f -o $OUT/tree_${f%.hip}.o &
done
wait
for spec in "$@"; do
  IFS=/ read -r name roles flags <<< "$spec"
  flags=${flags//__/ }
  (
  mkdir -p $T/$name; cp $SRC/* $T/$name/
  ADX_GEN_OUT=$T/$name ADX_GEN_ONLY=pair ADX_GEN_PAIR_ROLES4="$roles" python3 $ROOT/tools/gen_mfe_blocks.py > /dev/null
  $H $flags -c $T/$name/mfe_pair.hip -o $OUT/${name}_mfe_pair.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$name.so $OUT/tree_kernels.o $OUT/tree_mfe_cells.o \
    $OUT/${name}_mfe_pair.o $OUT/tree_outside_cells.o $OUT/tree_pf_cells.o $OUT/tree_pf_ring.o \
    $OUT/tree_outside_ring.o $OUT/api.o $OUT/energy.o
  ) &
done
wait
rm -rf $T
