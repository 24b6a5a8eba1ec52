# latency of every diagnostic library variant (MFE and PF, 4096 walkers)
set -e
mkdir -p gpurun_out/v
export TMPDIR=/tmp
rm -f gpurun_out/v/lat.txt
for f in addapt_amd/_lib/ablate/lib_*.so; do
  ADX_LIB=$f timeout -k 10 120 python tools/pf_latency.py --fold mfe >> gpurun_out/v/lat.txt 2>&1
  ADX_LIB=$f timeout -k 10 120 python tools/pf_latency.py --fold pf >> gpurun_out/v/lat.txt 2>&1
done
