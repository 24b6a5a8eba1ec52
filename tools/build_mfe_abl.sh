#!/bin/bash
# Timing-only ablations of mfe_cells_kernel (results WRONG; never the product):
#   nomask  constrained-cell shape masks off (U.mk = false)
#   nosel   per-slice generic energies not selected (slice 0's value for every lane)
#   noct    loop-correction gathers at a uniform address (no dependent second read)
# Libraries: addapt_amd/_lib/ablate/lib_mfe_<name>.so (the other kernels from base).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/addapt_amd/_lib/ablate
mkdir -p $OUT
T=$(mktemp -d)
build() {   # name, python transform of (hip, inc)
  local name=$1; local code=$2
  mkdir -p $T/$name; cp $ROOT/addapt_amd/csrc/* $T/$name/ 2>/dev/null || true
  python3 - $T/$name "$code" <<'PY'
import re, sys
d, code = sys.argv[1], sys.argv[2]
hip = open(d + "/mfe_cells.hip").read(); inc = open(d + "/mfe_blocks.inc").read()
exec(code)
open(d + "/mfe_cells.hip", "w").write(hip); open(d + "/mfe_blocks.inc", "w").write(inc)
PY
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $T/$name/mfe_cells.hip -o $OUT/c_mfe_$name.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib_mfe_$name.so $OUT/k_base.o $OUT/c_mfe_$name.o $OUT/o_base.o $OUT/p_base.o $OUT/r_base.o $OUT/q_base.o $OUT/api.o $OUT/energy.o
}
build nomask 'hip = hip.replace("U.mk = mk;", "U.mk = false;")' &
build nosel 'inc = re.sub(r"\(C\.r2 \? \(C\.r1 \? (\w+(?:\[\d+\])?) : \w+(?:\[\d+\])?\) : \(C\.r1 \? \w+(?:\[\d+\])? : \w+(?:\[\d+\])?\)\)", r"\1", inc); inc = re.sub(r"\(C\.r1 \? (\w+(?:\[\d+\])?) : \w+(?:\[\d+\])?\)", r"\1", inc)' &
build noct 'inc = re.sub(r"U\.ct\[([A-Za-z_.0-9]+) \+ c\w+\]", r"U.ct[\1]", inc); inc = re.sub(r"U\.ct\[CT_STK \+ C\.ty8 \+ \(\(c\w+ \* 41\) >> 10\)\]", "U.ct[CT_STK + C.ty8]", inc)' &
wait
rm -rf $T
