#!/usr/bin/env python3
"""Per-wave phase breakdown of mfe_pair_kernel (two diagonals per barrier) in
MC steps (incremental refolds; diagnostic stamp build:
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so, tools/build_ablate.sh).
usage: mfe_pair_stamps.py [N] [W] [steps]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from addapt_amd import native, workloads  # noqa: E402

L = native.lib()
L.adx_debug_stamps_pair.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
W = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
tmpl, active = workloads.synthetic(N)
apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
eng = native.Engine(tmpl, [active], workloads.default_objective(), aptamer=apt, fold_mode="mfe",
                    thermostat=native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300))
seqs = workloads.walker_sequences(tmpl, [active], W)
eng.walkers_init(list(range(W)), seqs)
eng.run_steps(1)
buf = (C.c_ulonglong * 256)()
L.adx_debug_stamps_pair(buf, 1)
eng.run_steps(steps)
L.adx_debug_stamps_pair(buf, 1)
_, _, c = eng.download()
scored = W * steps * float(c[:, 0].sum() + c[:, 1].sum() + c[:, 3].sum()) / max(1, c.sum())
G = scored * 2   # fold groups
cols = ["setup", "top", "L", "F", "Bcell", "Bblock", "Bfold", "M", "Q", "barrier", "total",
        "s.restore", "s.seq", "s.motif", "s.rstore", "s.cells", "s.cellw"]
print("cycles per fold group per wave (N=%d, W=%d, %d steps, %.0f groups)" % (N, W, steps, G))
print("wave " + " ".join("%8s" % n for n in cols))
for w in range(16):
    if not any(buf[w * 16 + k] for k in range(16)):
        continue
    v = [buf[w * 16 + k] // max(1, G) for k in (8, 0, 1, 2, 9, 10, 3, 4, 5, 6)]
    sub = [buf[w * 16 + k] // max(1, G) for k in (11, 12, 13, 7, 14, 15)]  # s.cellw: this wave's cell pass before the barrier
    print("%4d " % w + " ".join("%8d" % x for x in v) + " %8d" % sum(v) + " " + " ".join("%8d" % x for x in sub))
