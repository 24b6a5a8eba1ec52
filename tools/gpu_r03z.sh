#!/bin/bash
# per-wave phase stamps of mfe_cells_kernel and pf_cells_kernel (diagnostic build)
set -e
D=gpurun_out/r03z
mkdir -p $D
export TMPDIR=/tmp
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/mfe_mc_stamps.py 100 4096 3 > $D/mfe_stamps.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/pf_cells_stamps.py 100 4096 3 > $D/pf_stamps.txt 2>&1
