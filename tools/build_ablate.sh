#!/bin/bash
# Build timing-only ablation variants of the engine (results are wrong by design).
set -e
cd "$(dirname "$0")/../addapt_amd/csrc"
OUT=../_lib/ablate
mkdir -p $OUT
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c adx_api.cpp -o $OUT/api.o &
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c energy.cpp -o $OUT/energy.o &
for v in "base:" "nogen:-DADX_ABL_GENERIC" "noml:-DADX_ABL_ML" "nospec:-DADX_ABL_SPECIAL" "none:-DADX_ABL_GENERIC -DADX_ABL_ML -DADX_ABL_SPECIAL" "stamp:-DADX_STAMP"; do
  name=${v%%:*}; flags=${v#*:}
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $flags -c kernels.hip -o $OUT/k_$name.o &
done
wait
for name in base nogen noml nospec none stamp; do
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_$name.so $OUT/k_$name.o $OUT/api.o $OUT/energy.o
done
