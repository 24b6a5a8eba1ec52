"""Synthetic workloads and the roofline term counter. No GPU."""
import json
import os

import pytest

from addapt_amd import roofline, workloads

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_python_mt19937_matches_libstdcxx():
    with open(os.path.join(GOLDEN, "rng_mt19937.json")) as f:
        g = json.load(f)
    for case in g["raw"]:
        r = workloads.MT19937(case["seed"])
        assert [r() for _ in range(len(case["out"]))] == case["out"]
    for case in g["uniform_int"]:
        r = workloads.MT19937(case["seed"])
        assert [r.uniform_int(0, case["hi"]) for _ in range(len(case["out"]))] == case["out"]


@pytest.mark.parametrize("N", [60, 100, 150])
def test_synthetic_layout(oracle, N):
    tmpl, act = workloads.synthetic(N)
    assert len(tmpl) == len(act) == N
    o = (N - 27) // 2
    assert tmpl[o:o + 27] == workloads.THEO_SEQ.lower()
    assert tmpl[:o].isupper() and tmpl[o + 27:].isupper()
    comp = dict(A="U", U="A", G="C", C="G")
    for k in range(6):
        assert act[k] == "(" and act[N - 1 - k] == ")"
        assert tmpl[N - 1 - k] == comp[tmpl[k]]
    assert act[o - 6:o] == "x" * 6 and act[o + 27:o + 33] == "x" * 6
    # the active ensemble is non-empty, so ln p is finite
    assert oracle.pf_energy(tmpl.upper(), act) < 0


def test_walker_sequences(oracle):
    tmpl, act = workloads.synthetic(100)
    seqs = workloads.walker_sequences(tmpl, [act], 8)
    assert seqs == workloads.walker_sequences(tmpl, [act], 8)
    assert len(set(seqs)) == 8
    for s in seqs:
        for i, (a, b) in enumerate(zip(tmpl, s)):
            if not a.isupper():
                assert a == b          # frozen positions never change
        for k in range(6):             # enforced partners stay complementary
            assert dict(A="U", U="A", G="C", C="G")[s[k]] == s[99 - k]


@pytest.mark.parametrize("N", [60, 72])
def test_roofline_term_counts_match_oracle(oracle, N):
    tmpl, act = workloads.synthetic(N)
    for cst in (None, act):
        _, n_int, n_ml = oracle.pf_energy_counted(tmpl.upper(), cst)
        a, _ = roofline.pf_terms(tmpl, cst)
        assert a == n_int, (cst, a, n_int)


def test_flops_scale():
    tmpl, _ = workloads.synthetic(100)
    f = roofline.pf_flops(tmpl)
    assert 0.5e6 < f < 2e6   # ~1.03 MFLOP per PF at N = 100
