timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bppm.py > gpurun_out/oc1.log 2>&1; tail -3 gpurun_out/oc1.log
timeout -k 10 200 python bench.py --bppm --steps 60 --no-cpu-baseline > gpurun_out/oc1_c3.json 2> gpurun_out/oc1_c3.err && head -c 200 gpurun_out/oc1_c3.json && echo
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 200 python tools/outside_stamps.py
