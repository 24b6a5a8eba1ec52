"""GPU parity of the outside pass / base-pair probabilities (SURVEY.md §8 A16,
configs 3-4): RnaFold::base_pair_prob (scoring.cc:37-51) through adx_fold_bpp,
adx_bppm_batch and the ADX_TERM_PAIR score term, against the oracle's FP64
adjoint sweep (oracle/fold.c orc_bppm).

Tolerances: FP32 inside + outside with per-nucleotide scaling vs FP64:
|P_gpu - P_oracle| <= 2e-4 absolute per pair (whole matrices); score terms
within the bound 1e-4 kcal/mol per fold induces (tests/parity_bounds.py:
a pair probability is a ratio of two ensembles like a macrostate's); MC
trajectories bit-exact with the oracle forced through Metropolis near-ties
(|crit - u| <= 1e-6).
"""
import math
import random

import numpy as np
import pytest

from addapt_amd import workloads
from parity_bounds import close_score, close_term, score_bound

pytestmark = pytest.mark.gpu

P_TOL = 2e-4


def rand_seq(rng, n):
    return "".join(rng.choice("ACGU") for _ in range(n))


def test_fold_bpp_matches_oracle(native, oracle):
    rng = random.Random(23)
    cases = [("GGGGAAACCCC", None), ("ACGUGAAAACGU", "((((....))))"), (workloads.THEO_SEQ, None)]
    for n in (20, 45, 80, 100, 150):
        for _ in range(2):
            cases.append((rand_seq(rng, n), None))
    cases.append((cases[-3][0], "." * 10 + "x" * 5 + "." * 85))
    for seq, cst in cases:
        f = native.Fold(seq)
        if cst:
            f.add_constraint(cst)
        _, ref = oracle.bppm(seq, cst)
        n = len(seq)
        got = np.array([[f.bpp(i + 1, j + 1) for j in range(n)] for i in range(n)])
        assert np.abs(got - ref).max() <= P_TOL, (seq, cst, np.abs(got - ref).max())


def test_fold_bpp_motif(native, oracle):
    apt, fold = workloads.THEO_SEQ, workloads.THEO_FOLD
    e = oracle.theo_bonus()
    for seq in (apt, "GGGA" + apt + "UCCC"):
        f = native.Fold(seq)
        f.add_motif(apt, fold, e)
        _, ref = oracle.bppm(seq, None, oracle.make_motif(apt, fold, e))
        n = len(seq)
        got = np.array([[f.bpp(i + 1, j + 1) for j in range(n)] for i in range(n)])
        assert np.abs(got - ref).max() <= P_TOL, (seq, np.abs(got - ref).max())


def _objective(N):
    # config 3: default objective + apo/holo base-pair probability terms
    return workloads.default_objective() + [("apo", ("pair", 0, N - 1), False, 1.0),
                                            ("holo", ("pair", 0, N - 1), True, 1.0)]


def _engine(native, tmpl, macro, terms, thermostat=None, contexts=None):
    apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
    return native.Engine(tmpl, macro, terms, aptamer=apt, contexts=contexts,
                         thermostat=thermostat or native.make_thermostat("fixed", t=1.0))


def _oracle_sf(oracle, terms, contexts=None):
    m = oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, oracle.theo_bonus())
    return oracle.ScoreFunction(terms, aptamer=m, contexts=contexts)


@pytest.mark.parametrize("N", [60, 100, 150])
def test_bppm_batch(native, oracle, N):
    tmpl, active = workloads.synthetic(N)
    eng = _engine(native, tmpl, [active], _objective(N))
    seqs = workloads.walker_sequences(tmpl, [active], 6)
    m = oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, oracle.theo_bonus())
    for cond in ("apo", "holo"):
        got = eng.bppm_batch(seqs, cond)
        for w in range(6):
            _, ref = oracle.bppm(seqs[w].upper(), None, m if cond == "holo" else None)
            err = np.abs(got[w] - ref).max()
            assert err <= P_TOL, (N, cond, w, err)


def _close_terms(tv, tref, terms):
    return all(close_term(a, b, terms[k % len(terms)][2]) for k, (a, b) in enumerate(zip(tv, tref)))


@pytest.mark.parametrize("N", [60, 100, 150])
def test_score_with_pair_terms(native, oracle, N):
    tmpl, active = workloads.synthetic(N)
    terms = _objective(N)
    eng = _engine(native, tmpl, [active], terms)
    seqs = workloads.walker_sequences(tmpl, [active], 12)
    sc, tv, _ = eng.score_batch(seqs)
    sf = _oracle_sf(oracle, terms)
    for w in range(12):
        ref, tref = sf.score(seqs[w], [active])
        assert _close_terms(tv[w], tref, terms), (w, list(tv[w]), tref)
        assert close_score(sc[w], ref, tref, terms), (w, sc[w], ref)


def test_pair_terms_with_contexts(native, oracle):
    tmpl, active = workloads.synthetic(60)
    terms = [("apo", ("pair", 2, 57), True, 1.0), ("holo", ("pair", 0, 59), False, 0.5),
             ("holo", 0, True, 1.0)]
    ctx = [("GGAC", "UUA"), ("", "CCCA")]
    eng = _engine(native, tmpl, [active], terms, contexts=ctx)
    seqs = workloads.walker_sequences(tmpl, [active], 4)
    sc, tv, _ = eng.score_batch(seqs)
    sf = _oracle_sf(oracle, terms, contexts=ctx)
    for w in range(4):
        ref, tref = sf.score(seqs[w], [active])
        assert _close_terms(tv[w], tref, terms), (w, list(tv[w]), tref)
        assert close_score(sc[w], ref, tref, terms), (w, sc[w], ref)


def test_mc_trajectory_with_pair_terms(native, oracle):
    tmpl, active = workloads.synthetic(60)
    terms = _objective(60)
    th = native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=30)
    eng = _engine(native, tmpl, [active], terms, thermostat=th)
    seeds = [0, 1, 2, 3]
    seqs = workloads.walker_sequences(tmpl, [active], len(seeds))
    therm_o = oracle.thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=30)
    steps = 25
    eng.walkers_init(seeds, seqs)
    tr = eng.run_steps(steps, trace=True)
    final, scores, counters = eng.download()
    sf = _oracle_sf(oracle, terms)
    for w, seed in enumerate(seeds):
        forced = [int(x) for x in tr["outcome"][:, w]]
        ref = oracle.mc_run(sf, seqs[w], [active], therm_o, seed, steps, forced=forced, tie_eps=1e-6)
        assert ref["rc"] == 0
        assert list(tr["position"][:, w]) == ref["pos"], w
        assert tr["base"][w::len(seeds)] == ref["base"], w
        assert list(tr["outcome"][:, w]) == ref["outcome"], w
        assert final[w].upper() == ref["seq"].upper(), w
        assert list(counters[w]) == ref["counters"]


@pytest.mark.parametrize("N,motif_pairs", [(60, False), (80, True), (100, False), (110, False), (150, False),
                                           (150, True), ("longest", False)])
def test_mc_pair_terms_proposed_scores(native, oracle, N, motif_pairs):
    """Configs 3 / 4 shape: inside folds first (N <= 100: pf_cells_kernel,
    else pf_ring_kernel), the outside pass on the proposal's stored inside tables
    (N <= 100: outside_cells_kernel; N > 100: outside_ring_kernel on the ring
    kernel's diagonal-major slot), then the scores.  Every
    scored proposal's score matches the oracle's from-scratch score of that
    proposal (within the derived bound).  motif_pairs: pair terms inside the
    ligand motif (credited from the motif's closing cell in the holo fold).
    "longest": the longest template a pair-term context accepts (<= 190)."""
    if N == "longest":
        for N in range(190, 149, -1):
            try:
                _engine(native, workloads.synthetic(N)[0], [workloads.synthetic(N)[1]], _objective(N))
                break
            except native.AdxError as e:
                assert e.status == native.EUNSUPPORTED, e
    tmpl, active = workloads.synthetic(N)
    terms = _objective(N)
    if motif_pairs:
        o = (N - 27) // 2   # the aptamer's site in the synthetic template
        terms = workloads.default_objective() + [("holo", ("pair", o + 4, o + 22), True, 1.0),
                                                ("apo", ("pair", o, o + 26), False, 0.5),
                                                ("holo", ("pair", o + 7, o + 16), True, 0.25)]
    th = native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=30)
    eng = _engine(native, tmpl, [active], terms, thermostat=th)
    seeds = [21, 22, 23]
    seqs = workloads.walker_sequences(tmpl, [active], 64)
    eng.walkers_init(seeds + list(range(100, 161)), seqs)
    steps = 10
    tr = eng.run_steps(steps, trace=True)
    _, _, counters = eng.download()
    assert (counters.sum(axis=1) == steps).all()
    sf = _oracle_sf(oracle, terms)
    therm_o = oracle.thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=30)
    for w, seed in enumerate(seeds):
        forced = [int(x) for x in tr["outcome"][:, w]]
        ref = oracle.mc_run(sf, seqs[w], [active], therm_o, seed, steps, forced=forced, tie_eps=1e-6)
        assert ref["rc"] == 0
        assert list(tr["position"][:, w]) == ref["pos"], w
        for s in range(steps):
            if ref["outcome"][s] != 2:
                a, b = tr["proposed_score"][s, w], ref["proposed_score"][s]
                assert close_score(a, b, tr["term_values"][s, w], terms), (N, w, s, a, b)


@pytest.mark.parametrize("N", [100, 150])
def test_mc_pair_terms_full_size(native, oracle, N):
    """Configs 3 / 4 at their per-GPU size (4096 walkers; N = 100: pf_cells +
    outside_cells, N = 150: pf_ring + outside_ring): counters sum to the steps,
    and sampled walkers' final scores (pair probabilities included) equal the
    oracle's from-scratch scores of their final sequences."""
    tmpl, active = workloads.synthetic(N)
    terms = _objective(N)
    th = native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    eng = _engine(native, tmpl, [active], terms, thermostat=th)
    W = 4096
    seqs = workloads.walker_sequences(tmpl, [active], W)
    eng.walkers_init(list(range(W)), seqs)
    eng.run_steps(2)
    final, scores, counters = eng.download()
    assert (counters.sum(axis=1) == 2).all()
    inside, outside = eng.last_kernel_names()
    assert (inside.startswith("pf_cells_kernel") and outside == "outside_cells_kernel") if N <= 100 else \
        (inside.startswith("pf_ring_kernel") and outside == "outside_ring_kernel"), (inside, outside)
    sf = _oracle_sf(oracle, terms)
    for w in list(range(0, W, 683)) + [W - 1]:
        ref, tref = sf.score(final[w], [active])
        assert close_score(scores[w], ref, tref, terms), (N, w, scores[w], ref)
