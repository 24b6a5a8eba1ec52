set -e
mkdir -p gpurun_out/a5
export TMPDIR=/tmp ADX_MFE_KERNEL=cells ADX_NWV=8
for v in s1; do
  ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 120 python tools/cells_stamps.py 100 4096 > gpurun_out/a5/$v.txt 2>&1
done
