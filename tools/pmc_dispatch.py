#!/usr/bin/env python3
"""Per-dispatch PMC counters of one kernel from rocprofv3 counter-collection CSVs
(one counter group per file, the same bench command each pass), with derived
ratios.  The first dispatch of the kernel (the walkers' initial full folds) is
reported apart from the MC-step dispatches, which are averaged.

usage: pmc_dispatch.py --kernel mfe_cells [--ops-per-launch X] <csv>...
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--ops-per-launch", type=float, default=None,
                    help="algorithmic lane-ops per MC launch (bench.py roofline flop_per_launch)")
    ap.add_argument("--lane-ops-per-inst", type=float, default=64.0,
                    help="useful ops one VALU instruction can do (64 lanes; x2 for packed 16-bit)")
    ap.add_argument("csv", nargs="+")
    a = ap.parse_args()
    # per counter: {per-file dispatch order: value}
    per = collections.defaultdict(dict)
    for path in a.csv:
        disp = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            disp[(r["Counter_Name"], int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
        for name in {k[0] for k in disp}:
            ids = sorted(d for (n, d) in disp if n == name)
            per[name] = [disp[(name, d)] for d in ids]
    rows = {}
    for name, vals in sorted(per.items()):
        first, rest = vals[0], vals[1:] or vals[:1]
        rows[name] = (first, sum(rest) / len(rest), len(rest))
        print("%-26s first %16.0f   MC avg %16.0f  (%d launches)" % (name, first, rows[name][1], rows[name][2]))

    def g(n):
        return rows[n][1] if n in rows else None

    print()
    if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
        print("waves waiting            %.1f %% of wave cycles" % (100 * g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")))
    if g("SQ_ACTIVE_INST_VALU") and g("SQ_WAVE_CYCLES"):
        print("VALU active              %.1f %% of wave cycles" % (100 * g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES")))
    if g("SQ_LDS_BANK_CONFLICT") and g("SQ_LDS_IDX_ACTIVE"):
        print("LDS bank conflicts       %.1f %% of LDS-active cycles" % (100 * g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE")))
    if g("SQ_INSTS_SALU") and g("SQ_INSTS_VALU"):
        print("SALU per VALU            %.2f" % (g("SQ_INSTS_SALU") / g("SQ_INSTS_VALU")))
        print("LDS per VALU             %.2f" % (g("SQ_INSTS_LDS") / g("SQ_INSTS_VALU")))
    if a.ops_per_launch and g("SQ_INSTS_VALU"):
        slots = g("SQ_INSTS_VALU") * a.lane_ops_per_inst
        print("useful lane-ops / VALU lane-op slots  %.4f  (%.3g ops over %.3g slots per MC launch)"
              % (a.ops_per_launch / slots, a.ops_per_launch, slots))


if __name__ == "__main__":
    main()
