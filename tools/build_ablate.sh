#!/bin/bash
# Build diagnostic variants of the engine into addapt_amd/_lib/ablate/:
# base (= product flags) and stamp (-DADX_STAMP: per-wave phase cycle
# counters, read by tools/pf_stamps.py and tools/cells_stamps.py).
# Select one with ADX_LIB=addapt_amd/_lib/ablate/lib_<name>.so.
set -e
cd "$(dirname "$0")/../addapt_amd/csrc"
OUT=../_lib/ablate
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c adx_api.cpp -o $OUT/api.o &
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c energy.cpp -o $OUT/energy.o &
VARIANTS=${VARIANTS:-"base: stamp:-DADX_STAMP"}
for v in $VARIANTS; do
  name=${v%%:*}; flags=${v#*:}; flags=${flags//__/ }
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c kernels.hip -o $OUT/k_$name.o &
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c mfe_cells.hip -o $OUT/c_$name.o &
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c mfe_pair.hip -o $OUT/m_$name.o &
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c outside_cells.hip -o $OUT/o_$name.o &
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c pf_cells.hip -o $OUT/p_$name.o &
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c pf_ring.hip -o $OUT/r_$name.o &
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c outside_ring.hip -o $OUT/q_$name.o &
done
wait
for v in $VARIANTS; do
  name=${v%%:*}
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$name.so $OUT/k_$name.o $OUT/c_$name.o $OUT/m_$name.o $OUT/o_$name.o $OUT/p_$name.o $OUT/r_$name.o $OUT/q_$name.o $OUT/api.o $OUT/energy.o
done
