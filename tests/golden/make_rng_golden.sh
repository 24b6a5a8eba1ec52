#!/bin/bash
# Regenerate tests/golden/rng_mt19937.json with the host g++/libstdc++.
set -e
cd "$(dirname "$0")"
g++ -std=c++11 -O2 -o /tmp/adx_gen_rng gen_rng.cc
/tmp/adx_gen_rng > rng_mt19937.json
