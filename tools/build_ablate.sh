#!/bin/bash
# Build the diagnostic variants of the engine: base (= product flags) and stamp
# (per-wave phase cycle counters, tools/pf_stamps.py).
set -e
cd "$(dirname "$0")/../addapt_amd/csrc"
OUT=../_lib/ablate
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c adx_api.cpp -o $OUT/api.o &
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c energy.cpp -o $OUT/energy.o &
for v in "base:" "stamp:-DADX_STAMP"; do
  name=${v%%:*}; flags=${v#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c kernels.hip -o $OUT/k_$name.o &
done
wait
for name in base stamp; do
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$name.so $OUT/k_$name.o $OUT/api.o $OUT/energy.o
done
