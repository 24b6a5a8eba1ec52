set -e
bash tools/gpu_suite.sh r02f
mkdir -p gpurun_out/r02f/tr
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r02f/tr/w -o w --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02f/tr/w.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02f/tr/f -o f --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02f/tr/f.log 2>&1
python tools/pmc_traffic.py $(find gpurun_out/r02f/tr/f -name "*counter_collection.csv") $(find gpurun_out/r02f/tr/w -name "*counter_collection.csv") > gpurun_out/r02f/traffic_latest_mfe.json
