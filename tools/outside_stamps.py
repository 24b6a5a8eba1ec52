#!/usr/bin/env python3
"""Per-wave phase breakdown of the lanes = cells outside kernels (diagnostic
stamp build: ADX_LIB=addapt_amd/_lib/ablate/lib_stamp.so).  Runs config-3
MC steps (N = 100: outside_cells_kernel) or config-4 ones (N > 100:
outside_ring_kernel, its own stamp table).
usage: outside_stamps.py [N] [W] [steps]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from addapt_amd import native, workloads  # noqa: E402

L = native.lib()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
read = L.adx_debug_stamps_outside_ring if N > 100 else L.adx_debug_stamps_outside
read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
W = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
tmpl, active = workloads.synthetic(N)
apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
eng = native.Engine(tmpl, [active], workloads.config_objective(N, bppm=True), aptamer=apt,
                    thermostat=native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300))
seqs = workloads.walker_sequences(tmpl, [active], W)
eng.walkers_init(list(range(W)), seqs)
eng.run_steps(1)
buf = (C.c_ulonglong * 128)()
read(buf, 1)
eng.run_steps(steps)
read(buf, 1)
_, _, c = eng.download()
scored = W * steps * float(c[:, 0].sum() + c[:, 1].sum() + c[:, 3].sum()) / max(1, c.sum())
G = 2 * scored   # outside folds (apo, holo) of the scored walkers
cols = ["setup", "q5b", "Bcell", "Bshape", "M", "F/tail", "barrier"]
print("cycles per outside fold per wave (N=%d, W=%d, %d steps, %.1f folds)" % (N, W, steps, G))
print("wave " + " ".join("%9s" % n for n in cols))
for w in range(16):
    print("%4d " % w + " ".join("%9d" % (buf[w * 8 + k] // max(1, G)) for k in range(7)))
