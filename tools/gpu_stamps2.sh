set -e
mkdir -p gpurun_out/st2
export TMPDIR=/tmp
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/pf_stamps.py 100 mfe > gpurun_out/st2/stamp_mfe16.txt 2>&1
ADX_NO_MFE16=1 ADX_LIB=addapt_amd/_lib/ablate/lib_base.so timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/st2/lat_mfe32.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_base.so timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/st2/lat_mfe16.txt 2>&1
