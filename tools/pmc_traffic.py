#!/usr/bin/env python3
"""HBM bytes per MC step of the score kernel(s) from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE, separate runs of the same bench command).

MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are kilobytes at the L2's
fabric side; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
reads, so it is doubled.  Per kernel the first dispatch (walkers_init) is
skipped and the rest averaged (a kernel only walkers_init launches is left out); the per-step figure sums the
instantiations (the MFE step = packed 16-bit kernel + FP32 fallback launch).

usage: pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv > traffic.json
"""
import collections
import csv
import json
import sys

# the kernels of one step's score window (kernels.hip, mfe_cells.hip, pf_cells.hip, outside_cells.hip):
# the fold kernels, and with pair terms the outside pass and the score combine
SCORE_KERNELS = ("score_kernel", "mfe_cells_kernel", "mfe_pair_kernel", "pf_cells_kernel", "pf_ring_kernel", "outside_cells_kernel",
                 "outside_ring_kernel", "bppm_kernel", "combine_kernel")


def per_kernel(path, counter):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if any(k in r["Kernel_Name"] for k in SCORE_KERNELS) and r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for name, disp in acc.items():
        ids = sorted(disp)
        if len(ids) < 2:   # launched only by walkers_init (the initial full folds): not a step kernel
            continue
        vals = [disp[i] for i in ids[1:]]
        out[name] = (sum(vals) / len(vals), len(vals))
    return out


def main():
    """usage: pmc_traffic.py <FETCH_SIZE csv> <WRITE_SIZE csv> [dominant kernel name]"""
    f = per_kernel(sys.argv[1], "FETCH_SIZE")
    w = per_kernel(sys.argv[2], "WRITE_SIZE")
    # a kernel launched in fewer than half of the steps the fold kernels ran in
    # (the first MC step's full-fold path before any table slot is stored) is
    # left out of the per-step figure and listed apart
    nmax = max([n for k, (_, n) in f.items() if "combine_kernel" not in k] or [0])
    rare = {k for k, (_, n) in f.items() if 2 * n < nmax}
    kernels, skipped = {}, {}
    total = 0.0
    for name in sorted(set(f) | set(w)):
        if name in rare:
            skipped[name] = {"fetch_size_kb_raw": f[name][0], "write_size_kb": w.get(name, (0.0, 0))[0],
                             "launches": f[name][1]}
            continue
        fk = f.get(name, (0.0, 0))[0]
        wk = w.get(name, (0.0, 0))[0]
        b = (2.0 * fk + wk) * 1024.0
        total += b
        kernels[name] = {"fetch_size_kb_raw": fk, "write_size_kb": wk, "bytes": b,
                         "launches": f.get(name, (0, 0))[1]}
    def short(name):   # as rocprof lists it, without namespaces and parameters
        return name.replace("(anonymous namespace)::", "").replace("void ", "").replace("adx::", "").split("(")[0]
    # the kernel bench.py prices (roofline.traffic): argv[3] when given -- the
    # outside pass of the pair-term workloads -- else the one with the most bytes
    top = max(kernels, key=lambda k: kernels[k]["bytes"]) if kernels else ""
    dom = next((k for k in kernels if len(sys.argv) > 3 and sys.argv[3] in k), top)
    out = {"kernel": short(dom), "kernel_bytes_per_launch": kernels[dom]["bytes"] if dom else None,
           "most_bytes_kernel": short(top), "kernels": kernels, "bytes_per_launch": total,
           "not_per_step": skipped, "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM); KB = 1024 B"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
