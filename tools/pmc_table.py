#!/usr/bin/env python3
"""Sum PMC counters per kernel from rocprofv3 counter_collection CSVs (largest dispatch kernel only).
usage: pmc_table.py <csv>... [--kernel substr]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
ksub = None
if "--kernel" in sys.argv:
    ksub = sys.argv[sys.argv.index("--kernel") + 1]
    args = [a for a in args if a != ksub]
tot = defaultdict(float)
for path in args:
    for r in csv.DictReader(open(path)):
        k = r.get("Kernel_Name", "")
        if ksub and ksub not in k:
            continue
        if not ksub and "score_kernel" not in k and "mfe_cells" not in k:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k in sorted(tot):
    print("%-28s %16.0f" % (k, tot[k]))
