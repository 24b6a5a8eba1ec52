#!/bin/bash
# Late round 3: PMC passes of the final mfe_cells_kernel and pf_cells_kernel
set -e
BENCH_ARGS="--fold mfe --no-sub-records" bash tools/gpu_pmc.sh r03zf/pmc_mfe
BENCH_ARGS="--fold pf --no-sub-records" bash tools/gpu_pmc.sh r03zf/pmc_pf
