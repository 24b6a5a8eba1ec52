# parity (PF + MFE) -> latency (diagnostic base build) -> MFE and PF benches
set -e
mkdir -p gpurun_out/q
export TMPDIR=/tmp
rm -f gpurun_out/q/*
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_gpu_mfe.py -q -x -p no:cacheprovider > gpurun_out/q/pytest.log 2>&1
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline --fold pf > gpurun_out/q/bench_pf.json 2> gpurun_out/q/bench_pf.err
