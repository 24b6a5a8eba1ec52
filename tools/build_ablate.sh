#!/bin/bash
# Build diagnostic variants of the engine (timing only; ablated results are wrong):
# base (= product flags), stamp (per-wave phase cycle counters, tools/pf_stamps.py,
# tools/cells_stamps.py), and ablations that drop one part of the per-diagonal work.
set -e
cd "$(dirname "$0")/../addapt_amd/csrc"
OUT=../_lib/ablate
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c adx_api.cpp -o $OUT/api.o &
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c energy.cpp -o $OUT/energy.o &
VARIANTS=${VARIANTS:-"base: stamp:-DADX_STAMP noqbt:-DADX_ABL_QBT nored:-DADX_ABL_RED noqm:-DADX_ABL_QM noq5:-DADX_ABL_Q5"}
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//__/ }
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c kernels.hip -o $OUT/k_$name.o &
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c mfe_cells.hip -o $OUT/c_$name.o &
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c mfe_quad.hip -o $OUT/q_$name.o &
done
wait
for v in $VARIANTS; do
  name=${v%%:*}
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$name.so $OUT/k_$name.o $OUT/c_$name.o $OUT/q_$name.o $OUT/api.o $OUT/energy.o
done
