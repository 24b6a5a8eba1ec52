#!/usr/bin/env python3
"""Per-wave phase breakdown of the lanes = cells MFE kernel (diagnostic stamp
build: ADX_LIB=.../lib_stamp.so ADX_MFE_KERNEL=cells).  usage: cells_stamps.py [N] [W]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from addapt_amd import native, workloads  # noqa: E402

L = native.lib()
L.adx_debug_stamps_cells.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tmpl, active = workloads.synthetic(N)
apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
eng = native.Engine(tmpl, [active], workloads.default_objective(), aptamer=apt, fold_mode="mfe")
seqs = workloads.walker_sequences(tmpl, [active], W)
buf = (C.c_ulonglong * 256)()
eng.score_batch(seqs)
L.adx_debug_stamps_cells(buf, 1)
eng.score_batch(seqs)
L.adx_debug_stamps_cells(buf, 1)
G = 2 * W   # fold groups
cols = ["F", "B", "Msetup", "Mchunks", "Mtail", "Q", "barrier", "top"]
print("cycles per fold group per wave (N=%d, W=%d, %.3f ms)" % (N, W, eng.last_kernel_ms()))
print("wave " + " ".join("%9s" % n for n in cols))
for w in range(int(os.environ.get("ADX_NWV", "10"))):
    v = [buf[w * 16 + k] // G for k in (1, 2, 6, 7, 3, 4, 5, 0)]
    print("%4d " % w + " ".join("%9d" % x for x in v))
