set -e
tag=${1:-qst}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
export ADX_MFE_KERNEL=quad
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/quad_stamps.py 100 1 > gpurun_out/$tag/st1.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/quad_stamps.py 100 4096 > gpurun_out/$tag/st4096.txt 2>&1
