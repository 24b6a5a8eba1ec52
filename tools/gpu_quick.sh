# parity (PF + MFE) -> latency + stamps (diagnostic builds) -> MFE bench
set -e
mkdir -p gpurun_out/q
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py tests/test_gpu_mfe.py -q -x -p no:cacheprovider > gpurun_out/q/pytest.log 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/pf_stamps.py 100 mfe > gpurun_out/q/stamp_mfe.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_base.so timeout -k 10 120 python tools/pf_latency.py --fold mfe > gpurun_out/q/lat_mfe.txt 2>&1
ADX_LIB=addapt_amd/_lib/ablate/lib_base.so timeout -k 10 120 python tools/pf_latency.py --fold pf > gpurun_out/q/lat_pf.txt 2>&1
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/q/bench.json 2> gpurun_out/q/bench.err
