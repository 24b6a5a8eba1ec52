#!/bin/bash
# Regenerate tests/golden/nth_element.json with the host g++/libstdc++.
set -e
cd "$(dirname "$0")"
g++ -std=c++11 -O2 -o /tmp/adx_gen_nth gen_nth_element.cc
/tmp/adx_gen_nth > nth_element.json
