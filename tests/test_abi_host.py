"""The C-ABI library (addapt_amd/_lib/libaddapt_gpu.so) without a GPU: it
loads, exports every entry point include/addapt_gpu.h declares, and its host
side (parameter loading, structure energies, kT, status/error reporting)
agrees with the oracle.  No compute is launched."""
import os
import random
import re
import subprocess

import pytest

from addapt_amd import workloads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "addapt_gpu.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(adx_[A-Za-z_0-9]+)\s*\(", txt)))


def test_header_and_binding_agree(native):
    assert sorted(native.EXPORTS) == declared()


def test_library_exports_every_symbol(native):
    path = native.lib()._name
    out = subprocess.run(["nm", "-D", "--defined-only", path], stdout=subprocess.PIPE,
                         text=True, check=True).stdout
    syms = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [s for s in declared() if s not in syms]
    assert not missing, missing


def test_abi_version_and_kT(native, oracle):
    assert native.lib().adx_abi_version() == native.ABI_VERSION == 4
    # scoring.cc:69-70: kT = exp_params->kT / 1000 at 37 C
    assert abs(native.kT() - (37.0 + 273.15) * 1.98717 / 1000.0) < 1e-12
    assert abs(native.kT() - oracle.KT_KCAL) < 1e-12


def _random_structure(rng, n):
    pairs = {("A", "U"), ("U", "A"), ("C", "G"), ("G", "C"), ("G", "U"), ("U", "G")}
    for _ in range(100):
        seq = "".join(rng.choice("ACGU") for _ in range(n))
        s = ["."] * n
        st = []
        for k in range(n):
            if st and k - st[-1] > 3 and (seq[st[-1]], seq[k]) in pairs and rng.random() < 0.5:
                o = st.pop()
                s[o], s[k] = "(", ")"
            elif rng.random() < 0.3:
                st.append(k)
        if s.count("(") >= 2:
            return seq, "".join(s)
    return seq, "." * n


def test_eval_structure_matches_oracle(native, oracle):
    P = native.default_params()
    rng = random.Random(11)
    cases = [("ACGUGAAAACGU", "((((....))))"),
             (workloads.THEO_SEQ, workloads.THEO_FOLD),
             (workloads.THEO_SEQ, "....((((((....)))...)))....")]
    for n in (20, 40, 80, 120):
        for _ in range(5):
            cases.append(_random_structure(rng, n))
    for seq, st in cases:
        a = P.eval_structure(seq, st)
        b = oracle.eval_structure(seq, st)
        assert abs(a - b) < 1e-9, (seq, st, a, b)


def test_errors_are_reported_not_thrown(native):
    with pytest.raises(native.AdxError) as e:
        native.Params("/nonexistent/file.par")
    assert e.value.args and "nonexistent" in str(e.value)
