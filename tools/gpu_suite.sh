# GPU test suite + default bench (MFE) + PF bench; logs under gpurun_out/$1
set -e
D=gpurun_out/${1:-s}
mkdir -p $D
export TMPDIR=/tmp
rm -f $D/*
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err
timeout -k 10 300 python bench.py --fold pf --no-cpu-baseline > $D/bench_pf.json 2> $D/bench_pf.err
