#!/bin/bash
# A/B of the PF record prefetch (lib_head = previous pf_cells) and the MFE
# per-wave stamps
set -e
D=gpurun_out/${1:-r03n}
mkdir -p $D
export TMPDIR=/tmp
for k in 1 2; do
ADX_LIB=addapt_amd/_lib/ablate/lib_head.so timeout -k 10 200 python bench.py --fold pf --steps 100 --no-cpu-baseline --no-sub-records > $D/pf_head$k.json 2> $D/pf_head$k.err
ADX_LIB=addapt_amd/_lib/ablate/lib_base.so timeout -k 10 200 python bench.py --fold pf --steps 100 --no-cpu-baseline --no-sub-records > $D/pf_new$k.json 2> $D/pf_new$k.err
done
timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline --no-sub-records > $D/mfe.json 2> $D/mfe.err
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 200 python tools/mfe_mc_stamps.py > $D/mfe_stamps.txt 2>&1
