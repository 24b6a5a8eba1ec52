#!/usr/bin/env python3
"""Average duration of the timed MC-step score_kernel launches in a rocprofv3
kernel trace (bench_kernel_trace.csv): the LAST `--last K` launches (K = the
bench's --steps), i.e. the launches bench.py's roofline.kernel_ms_per_launch
times with HIP events -- calibration, walkers_init and warmup launches are
excluded.

usage: trace_summary.py bench_kernel_trace.csv [--last K]
"""
import csv
import json
import sys

path = sys.argv[1]
last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 10
rows = [r for r in csv.DictReader(open(path)) if "score_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
step = d[-last:]
names = sorted({r["Kernel_Name"] for r in rows[-last:]})
print(json.dumps({"score_kernel_launches": len(step), "avg_ms": sum(step) / len(step),
                  "min_ms": min(step), "max_ms": max(step), "kernel_names": names,
                  "selection": "last %d launches (the timed steps)" % last}, indent=1))
