set -e
mkdir -p gpurun_out/st1
for v in stamp 1wg; do
ADX_LIB=addapt_amd/_lib/ablate/lib_$v.so timeout -k 10 200 python tools/mfe_mc_stamps.py > gpurun_out/st1/stamps_$v.txt 2>&1
done
