# latency of every variant in _lib/ablate (MFE, lanes = cells) + stamps
set -e
tag=${1:-var}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
export ADX_MFE_KERNEL=cells
for f in addapt_amd/_lib/ablate/lib_*.so; do
  case $f in *stamp*) continue;; esac
  ADX_LIB=$f timeout -k 10 120 python tools/pf_latency.py --fold mfe >> gpurun_out/$tag/lat.txt 2>&1
done
for f in addapt_amd/_lib/ablate/lib_stamp*.so; do
  ADX_LIB=$f timeout -k 10 120 python tools/cells_stamps.py 100 4096 > gpurun_out/$tag/st_$(basename $f .so).txt 2>&1
done
