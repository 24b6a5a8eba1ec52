"""Oracle base-pair probability score term (ADX_TERM_PAIR): its value is
ln P(i,j) (or ln(1 - P)) of the condition's unconstrained ensemble, P from
the oracle's own bppm (orc_bppm, itself pinned by the reference's bppm
threshold tests and by enumeration below).  No GPU."""
import math

import numpy as np

from addapt_amd import workloads


def test_pair_term_value(oracle):
    tmpl, active = workloads.synthetic(60)
    seq = workloads.walker_sequences(tmpl, [active], 1)[0]
    m = oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, oracle.theo_bonus())
    terms = [("apo", ("pair", 0, 59), False, 1.0), ("holo", ("pair", 1, 58), True, 2.0)]
    sf = oracle.ScoreFunction(terms, aptamer=m)
    s, tv = sf.score(seq, [active])
    _, Pa = oracle.bppm(seq.upper())
    _, Ph = oracle.bppm(seq.upper(), None, m)
    assert math.isclose(tv[0], math.log(1.0 - Pa[0, 59]), rel_tol=1e-12)
    assert math.isclose(tv[1], math.log(Ph[1, 58]), rel_tol=1e-12)
    assert math.isclose(s, tv[0] + 2.0 * tv[1], rel_tol=1e-12)


def test_bppm_matches_enumeration(oracle):
    """P(i,j) = sum over structures containing (i,j) of exp(-E/kT) / Z."""
    from tests.test_oracle_enum import KT, structures

    seq = "GGGAAAUCCCAGCU"
    Z = 0.0
    acc = np.zeros((len(seq), len(seq)))
    for db in structures(seq):
        e = oracle.eval_structure(seq, db)
        if e >= 1e6:
            continue
        wgt = math.exp(-e / KT)
        Z += wgt
        stk = []
        for k, c in enumerate(db):
            if c == "(":
                stk.append(k)
            elif c == ")":
                a = stk.pop()
                acc[a, k] += wgt
                acc[k, a] += wgt
    _, P = oracle.bppm(seq)
    assert np.abs(P - acc / Z).max() < 1e-9
