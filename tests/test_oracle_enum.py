"""Independent check of the oracle's partition function: for short sequences,
enumerate every pseudoknot-free secondary structure (hairpins >= 3 nt,
canonical + GU pairs, hard constraints), evaluate each with the oracle's
loop-energy evaluator and compare sum exp(-E/kT) with the McCaskill
recursion (oracle/fold.c).  Also MFE = min E.  No GPU.
"""
import math
import random

import pytest

KT = (37.0 + 273.15) * 1.98717 / 1000.0
PAIRS = {("A", "U"), ("U", "A"), ("C", "G"), ("G", "C"), ("G", "U"), ("U", "G")}


def structures(seq, cst=None):
    """All dot-brackets compatible with DB_DEFAULT|ENFORCE_BP constraints."""
    n = len(seq)
    forced = {}
    if cst:
        st = []
        for k, c in enumerate(cst):
            if c == "(":
                st.append(k)
            elif c == ")":
                o = st.pop()
                forced[o], forced[k] = k, o

    memo = {}

    def rec(i, j):
        # structures on [i, j] (inclusive) as lists of pair sets
        if i > j:
            return [()]
        key = (i, j)
        if key in memo:
            return memo[key]
        out = []
        # i unpaired
        if not (cst and (cst[i] in "|<>()" )):
            out += rec(i + 1, j)
        for k in range(i + 4, j + 1):
            if (seq[i], seq[k]) not in PAIRS:
                continue
            if cst:
                if cst[i] == "x" or cst[k] == "x" or cst[i] == ">" or cst[k] == "<":
                    continue
                if cst[i] == ")" or cst[k] == "(":
                    continue
                if i in forced and forced[i] != k:
                    continue
                if k in forced and forced[k] != i:
                    continue
                # a pair must not cross an enforced pair
                bad = False
                for a, b in forced.items():
                    if a < b and ((i < a < k < b) or (a < i < b < k)):
                        bad = True
                        break
                if bad:
                    continue
            for inner in rec(i + 1, k - 1):
                for rest in rec(k + 1, j):
                    out.append(((i, k),) + inner + rest)
        memo[key] = out
        return out

    res = []
    for ps in rec(0, n - 1):
        if cst:
            paired = {p for pr in ps for p in pr}
            if any(c in "|<>()" and k not in paired for k, c in enumerate(cst)):
                continue
            if any(forced.get(a) is not None and forced[a] != b for a, b in ps):
                continue
        s = ["."] * n
        for a, b in ps:
            s[a], s[b] = "(", ")"
        res.append("".join(s))
    return res


def enum_pf(oracle, seq, cst=None):
    Z = 0.0
    emin = math.inf
    for s in structures(seq, cst):
        e = oracle.eval_structure(seq, s)
        if e >= 1e6:
            continue
        Z += math.exp(-e / KT)
        emin = min(emin, e)
    return Z, emin


SEQS = ["GGGAAACCC", "ACGUGAAAACGU", "GCGCUUCGGCGC", "GGACUUCGGUCC"]
random.seed(7)
for _ in range(6):
    SEQS.append("".join(random.choice("ACGU") for _ in range(random.randint(10, 14))))


@pytest.mark.parametrize("seq", SEQS)
def test_pf_matches_enumeration(oracle, seq):
    Z, emin = enum_pf(oracle, seq)
    g = oracle.pf_energy(seq)
    assert abs(-KT * math.log(Z) - g) < 1e-6, (seq, -KT * math.log(Z), g)
    e, _ = oracle.mfe(seq)
    assert abs(e - round(emin, 2)) < 1e-6, (seq, e, emin)


@pytest.mark.parametrize("seq,cst", [
    ("ACGUGAAAACGU", "xxxx........"),
    ("ACGUGAAAACGU", "((........))"),
    ("GCGCUUCGGCGC", "..|........."),
    ("GCGCUUCGGCGC", "....xxxx...."),
    ("GGACUUCGGUCC", "(..........)"),
])
def test_constrained_pf_matches_enumeration(oracle, seq, cst):
    Z, _ = enum_pf(oracle, seq, cst)
    g = oracle.pf_energy(seq, cst)
    if Z == 0.0:
        assert g > 1e5 or math.isinf(g)
    else:
        assert abs(-KT * math.log(Z) - g) < 1e-6, (seq, cst, -KT * math.log(Z), g)
