#!/usr/bin/env python3
"""Per-wave phase breakdown of pf_ring_kernel (diagnostic stamp build:
ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so).  Runs PF MC steps of the
config-4 objective without pair terms at N (default 150).  Waves 0-6 = B
(interior loops), 7 F, 8 Q (q5 + prep), 9 R (records), 10-13 M (qm rows).
Columns: setup, B cell records, B shapes, role step work, tail, Q q5, Q prep,
barrier (cycles per workgroup).
usage: ring_stamps.py [N] [W] [steps]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from addapt_amd import native, workloads  # noqa: E402

L = native.lib()
L.adx_debug_stamps_ring.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 150
W = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
tmpl, active = workloads.synthetic(N)
apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
eng = native.Engine(tmpl, [active], workloads.default_objective(), aptamer=apt,
                    thermostat=native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300))
seqs = workloads.walker_sequences(tmpl, [active], W)
eng.walkers_init(list(range(W)), seqs)
eng.run_steps(1)
buf = (C.c_ulonglong * 128)()
L.adx_debug_stamps_ring(buf, 1)
eng.run_steps(steps)
L.adx_debug_stamps_ring(buf, 1)
_, _, c = eng.download()
scored = W * steps * float(c[:, 0].sum() + c[:, 1].sum() + c[:, 3].sum()) / max(1, c.sum())
G = scored * eng.info.n_variants   # workgroups: one per (walker, variant)
cols = ["setup", "Brec", "Bshape", "step", "tail", "q5", "prep", "barrier"]
print("cycles per workgroup per wave (N=%d, W=%d, %d steps, %.1f workgroups)" % (N, W, steps, G))
print("wave " + " ".join("%9s" % n for n in cols))
for w in range(14):
    print("%4d " % w + " ".join("%9d" % (buf[w * 8 + k] // max(1, G)) for k in range(8)))
