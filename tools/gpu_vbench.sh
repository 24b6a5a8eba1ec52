# bench (MC steps, incremental folds) with every diagnostic library variant
set -e
mkdir -p gpurun_out/vb
export TMPDIR=/tmp
rm -f gpurun_out/vb/*
for f in addapt_amd/_lib/ablate/lib_*.so; do
  n=$(basename $f .so)
  ADX_LIB=$f timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/vb/$n.mfe.json 2>/dev/null
  ADX_LIB=$f timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --fold pf > gpurun_out/vb/$n.pf.json 2>/dev/null
done
