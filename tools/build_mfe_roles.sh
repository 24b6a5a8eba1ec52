#!/bin/bash
# MFE block-partition variants: the 4-lanes-per-cell partition seeded with other
# role costs (ADX_GEN_ROLES4) and/or the list role on another wave (MFE_LW).
# usage: tools/build_mfe_roles.sh name/ROLES4/LW ...  -> addapt_amd/_lib/ablate/lib_mfe_<name>.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/addapt_amd/_lib/ablate
mkdir -p $OUT
T=$(mktemp -d)
for spec in "$@"; do
  IFS=/ read -r name roles lw <<< "$spec"
  (
  mkdir -p $T/$name; cp $ROOT/addapt_amd/csrc/* $T/$name/
  ADX_GEN_OUT=$T/$name ADX_GEN_ROLES4="$roles" python3 $ROOT/tools/gen_mfe_blocks.py 2>/dev/null
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC ${lw:+-DMFE_LW=$lw} -c $T/$name/mfe_cells.hip -o $OUT/c_mfe_$name.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_mfe_$name.so $OUT/k_et.o $OUT/c_mfe_$name.o $OUT/o_et.o $OUT/p_et.o $OUT/r_et.o $OUT/q_et.o $OUT/api.o $OUT/energy.o
  ) &
done
wait
rm -rf $T
