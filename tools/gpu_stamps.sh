set -e
mkdir -p gpurun_out/st
export TMPDIR=/tmp
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/pf_stamps.py 100 mfe > gpurun_out/st/stamp_mfe.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/pf_stamps.py 100 pf > gpurun_out/st/stamp_pf.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_base.so timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/st/lat_mfe.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_base.so timeout -k 10 120 python tools/pf_latency.py --fold pf > gpurun_out/st/lat_pf.txt 2>&1
