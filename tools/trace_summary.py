#!/usr/bin/env python3
"""Per-step duration of the score kernel(s) in a rocprofv3 kernel trace
(bench_kernel_trace.csv), comparable with bench.py's
roofline.kernel_ms_per_launch (HIP events around each step's score launch,
which for the MFE fold covers the packed 16-bit kernel and its FP32 fallback
launch).  For every score_kernel instantiation the LAST `--last K` launches
(K = the bench's --steps: calibration, walkers_init and warmup launches
excluded) are averaged; the per-step figure is the sum over instantiations.

usage: trace_summary.py bench_kernel_trace.csv [--last K]
"""
import collections
import csv
import json
import sys

# the fold kernels one score launch consists of (kernels.hip, mfe_cells.hip)
SCORE_KERNELS = ("score_kernel", "mfe_cells_kernel", "pf_cells_kernel")

path = sys.argv[1]
last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 10
by = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    if any(k in r["Kernel_Name"] for k in SCORE_KERNELS):
        by[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
out = {"selection": "last %d launches of each score_kernel instantiation (the timed steps)" % last,
       "kernels": {}}
per_step = 0.0
for name, rows in by.items():
    rows.sort()
    d = [(e - s) / 1e6 for s, e in rows][-last:]
    avg = sum(d) / len(d)
    per_step += avg
    out["kernels"][name] = {"launches": len(d), "avg_ms": avg, "min_ms": min(d), "max_ms": max(d)}
out["avg_ms_per_step"] = per_step
print(json.dumps(out, indent=1))
