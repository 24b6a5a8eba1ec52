set -e
mkdir -p gpurun_out/mfe1
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/mfe1/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/mfe1/smoke.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/mfe1/bench_mfe.json 2> gpurun_out/mfe1/bench_mfe.err
timeout -k 10 300 python bench.py --no-cpu-baseline --fold pf > gpurun_out/mfe1/bench_pf.json 2> gpurun_out/mfe1/bench_pf.err
cat gpurun_out/mfe1/bench_mfe.json gpurun_out/mfe1/bench_pf.json
