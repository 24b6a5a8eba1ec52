#!/bin/bash
set -e
mkdir -p gpurun_out
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so timeout -k 10 120 python tools/pf_stamps.py > gpurun_out/stamp.txt 2>&1
