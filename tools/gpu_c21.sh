set -e
mkdir -p gpurun_out/c30
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
for v in b0 t1 t2 t3 b0 t1 t2 t3; do ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/pf_latency.py --fold mfe >> gpurun_out/c30/lat.txt 2>&1; done
