#!/usr/bin/env python3
"""Per-wave phase breakdown of pf_cells_kernel (diagnostic stamp build:
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so).  Runs PF MC steps (N=100 bench
objective; "tables" = the barrier + block_or after s.prolog, s.loads, s.rissue).  Waves 0-7 = B (interior loops), 8-9 M, 10-11 F, 12 Q, 13 records.
usage: pf_cells_stamps.py [N] [W] [steps]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from addapt_amd import native, workloads  # noqa: E402

L = native.lib()
L.adx_debug_stamps_pf.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
W = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
tmpl, active = workloads.synthetic(N)
apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
eng = native.Engine(tmpl, [active], workloads.default_objective(), aptamer=apt,
                    thermostat=native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300))
seqs = workloads.walker_sequences(tmpl, [active], W)
eng.walkers_init(list(range(W)), seqs)
eng.run_steps(1)
buf = (C.c_ulonglong * 192)()
L.adx_debug_stamps_pf(buf, 1)
eng.run_steps(steps)
L.adx_debug_stamps_pf(buf, 1)
_, _, c = eng.download()
scored = W * steps * float(c[:, 0].sum() + c[:, 1].sum() + c[:, 3].sum()) / max(1, c.sum())
G = scored * max(1, eng.info.n_variants // 2)   # workgroups: one per (walker, apo/holo group)
cols = ["cellpass", "tables", "Bcell", "Bshape", "work", "Bwrite", "barrier", "restore", "s.prolog", "s.loads", "s.rissue"]
print("cycles per workgroup per wave (N=%d, W=%d, %d steps, %.1f workgroups)" % (N, W, steps, G))
print("wave " + " ".join("%9s" % n for n in cols))
for w in range(16):
    print("%4d " % w + " ".join("%9d" % (buf[w * 12 + k] // max(1, G)) for k in range(11)))
