# per-phase stamps + ablation latencies for MFE and PF (diagnostic builds in _lib/ablate)
set -e
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/pf_stamps.py 100 mfe > gpurun_out/diag/stamp_mfe.txt 2>&1
for f in addapt_amd/_lib/ablate/lib_*.so; do
  ADX_LIB=$f timeout -k 10 120 python tools/pf_latency.py --fold mfe >> gpurun_out/diag/abl_mfe.txt 2>&1
done
