set -e
mkdir -p gpurun_out/c25
export TMPDIR=/tmp
for v in q0 q2 q0 q2; do ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/pf_latency.py >> gpurun_out/c25/lat.txt 2>&1; done
