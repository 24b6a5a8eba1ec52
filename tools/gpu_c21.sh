set -e
mkdir -p gpurun_out/c22
export TMPDIR=/tmp ADX_MFE_KERNEL=cells
for v in p0 p2 p4 p5 p6 p0 p2 p4 p5 p6; do ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/pf_latency.py --fold mfe >> gpurun_out/c22/lat.txt 2>&1; done
