#!/usr/bin/env python3
"""Per-wave phase breakdown of one PF (diagnostic stamp build, ADX_LIB=.../lib_stamp.so)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from addapt_amd import native, workloads  # noqa: E402

L = native.lib()
L.adx_debug_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
tmpl, active = workloads.synthetic(int(sys.argv[1]) if len(sys.argv) > 1 else 100)
fold = sys.argv[2] if len(sys.argv) > 2 else "pf"
apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
eng = native.Engine(tmpl, [active], workloads.default_objective(), aptamer=apt, fold_mode=fold)
buf = (C.c_ulonglong * 256)()
eng.score_batch([tmpl])
L.adx_debug_stamps(buf, 1)
eng.score_batch([tmpl])
L.adx_debug_stamps(buf, 1)
V = eng.info.n_variants
# stamp ids (kernels.hip STAMP(k)): 10 loop top + qm1 pass, 0 descriptors + chunk 0,
# 6 q5, 5 qm items, 4 qb cells + finalize, 9 barrier
cols = [(10, "top"), (0, "late"), (6, "q5"), (5, "qm"), (4, "qb"), (7, "prep"), (9, "barrier")]
print("cycles per PF per wave (avg over %d variants)" % V)
print("wave " + " ".join("%9s" % n for _, n in cols))
for w in range(16):
    print("%4d " % w + " ".join("%9d" % (buf[w * 16 + k] // V) for k, _ in cols))
