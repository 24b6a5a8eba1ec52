#!/usr/bin/env python3
"""Summarise an interleaved A/B run (tools/gpu_run.sh "libs" step):
gpurun_out/<tag>/<name>_<variant>_<rep>.json -> per variant mean / min / max
MC steps/s and the ratio to the first variant listed.
usage: ab_summary.py <dir> <name> <variant> [<variant> ...]"""
import json
import os
import statistics
import sys

d, name, variants = sys.argv[1], sys.argv[2], sys.argv[3:]
base = None
for v in variants:
    vals = []
    k = 1
    while os.path.exists(os.path.join(d, "%s_%s_%d.json" % (name, v, k))):
        try:
            with open(os.path.join(d, "%s_%s_%d.json" % (name, v, k))) as f:
                vals.append(json.load(f)["value"])
        except (ValueError, KeyError):
            pass
        k += 1
    if not vals:
        print("%-10s no results" % v)
        continue
    m = statistics.mean(vals)
    base = base or m
    print("%-10s n=%d mean %.0f  min %.0f  max %.0f  x%.4f" % (v, len(vals), m, min(vals), max(vals), m / base))
