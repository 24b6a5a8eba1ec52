#!/usr/bin/env python3
"""Latency / throughput probe of the score kernel (ablation + profiling helper).

    ADX_LIB=path/to/lib.so python tools/pf_latency.py [--W 4096] [--reps 3] [--N 100]
Prints per-call device ms for a 1-walker and a W-walker score_batch.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from addapt_amd import native, workloads  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--W", type=int, default=4096)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--N", type=int, default=100)
ap.add_argument("--fold", default="pf")
a = ap.parse_args()
tmpl, active = workloads.synthetic(a.N)
apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
eng = native.Engine(tmpl, [active], workloads.default_objective(), aptamer=apt, fold_mode=a.fold)
seqs = workloads.walker_sequences(tmpl, [active], a.W)
one = []
for _ in range(a.reps):
    eng.score_batch(seqs[:1])
    one.append(eng.last_kernel_ms())
many = []
for _ in range(a.reps):
    eng.score_batch(seqs)
    many.append(eng.last_kernel_ms())
lib = os.path.basename(os.environ.get("ADX_LIB", "default"))
V = eng.info.n_variants
print("%-14s 1-walker %.3f ms (%.1f us/PF)   %d walkers %.3f ms (%.2f us/PF chip-wide)"
      % (lib, min(one), 1e3 * min(one) / V, a.W, min(many), 1e3 * min(many) / (V * a.W)))
