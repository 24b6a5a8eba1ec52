#!/usr/bin/env python3
"""Average duration of the MC-step score_kernel launches in a rocprofv3
kernel trace (bench_kernel_trace.csv): skips the calibration and
walkers_init launches (the first two), so it is comparable with bench.py's
roofline.kernel_ms_per_launch (HIP events around the same launches)."""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "score_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
step = d[2:] if len(d) > 2 else d
print(json.dumps({"score_kernel_launches": len(step), "avg_ms": sum(step) / len(step),
                  "min_ms": min(step), "max_ms": max(step),
                  "skipped": "calibration + walkers_init launches"}, indent=1))
