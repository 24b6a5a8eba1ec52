"""Full-cycle oracle parity at full size (BASELINE configs 2, 3, 4 per GPU):
4096 walkers x 300 steps = one whole annealing cycle (5 -> 0 in 300,
sampling.cc:332-338) of the reference loop (sampling.cc:55-99), traced.

Eight walkers spread over the batch are replayed through the oracle's
MonteCarlo::apply restatement (oracle.mc_run, Metropolis near-ties forced to
the engine's outcome): positions, bases and outcomes are bit-exact over all
300 steps, and every proposed score agrees within the bound the north star's
fold bar implies (tests/parity_bounds.py; MFE: exact integer energies, 1e-12
relative).  Then every walker's stored score must equal a from-scratch score
of its final sequence bit for bit (adx_walkers_rescore: the step's own
kernels, no stored tables read) -- with pair terms for configs 3 / 4, whose
outside passes run on the incrementally refolded inside tables -- and the
stateless batch path (adx_score_batch) within the derived bound."""
import math
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from addapt_amd import workloads
from parity_bounds import close_score

pytestmark = pytest.mark.gpu

W, STEPS = 4096, 300
CONFIGS = {"config2": (100, "mfe", False), "config3": (100, "pf", True), "config4": (150, "pf", True)}


def _close_mfe(a, b):
    if math.isinf(b) or math.isnan(b):
        return (math.isnan(a) and math.isnan(b)) or a == b
    return abs(a - b) <= 1e-12 * max(1.0, abs(b))


@pytest.mark.parametrize("name", list(CONFIGS))
def test_full_cycle_oracle_replay(native, oracle, name):
    N, fold, bppm = CONFIGS[name]
    tmpl, active = workloads.synthetic(N)
    terms = workloads.config_objective(N, bppm=bppm)
    apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
    th = native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    eng = native.Engine(tmpl, [active], terms, aptamer=apt, thermostat=th, fold_mode=fold)
    seqs = workloads.walker_sequences(tmpl, [active], W)
    seeds = list(range(W))
    eng.walkers_init(seeds, seqs)
    tr = eng.run_steps(STEPS, trace=True)
    final, scores, counters = eng.download()
    assert (counters.sum(axis=1) == STEPS).all()

    # stored (incremental refolds) vs every walker refolded from scratch by the
    # step's own kernels: bit-identical
    fresh, _ = eng.rescore()
    bad = np.nonzero(scores != fresh)[0]
    assert bad.size == 0, [(int(w), scores[w], fresh[w]) for w in bad[:8]]
    # vs the stateless batch path (bppm_kernel / score_kernel): MFE exact, PF
    # within the derived bound
    sc, tv, _ = eng.score_batch(final)
    for w in range(W):
        if fold == "mfe":
            assert _close_mfe(scores[w], sc[w]), (name, w, scores[w], sc[w])
        else:
            assert close_score(scores[w], sc[w], tv[w], terms), (name, w, scores[w], sc[w])

    m = oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, oracle.theo_bonus())
    sf = oracle.ScoreFunction(terms, aptamer=m, mode=fold)
    therm_o = oracle.thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    sample = [0, 511, 1170, 1755, 2340, 2925, 3510, W - 1]
    tie = 1e-12 if fold == "mfe" else 1e-6

    def replay(w):
        forced = [int(x) for x in tr["outcome"][:, w]]
        return oracle.mc_run(sf, seqs[w], [active], therm_o, seeds[w], STEPS, forced=forced, tie_eps=tie)

    with ThreadPoolExecutor(max_workers=8) as ex:   # ctypes drops the GIL: the replays run in parallel
        refs = list(ex.map(replay, sample))
    scored = 0
    for w, ref in zip(sample, refs):
        assert ref["rc"] == 0
        assert list(tr["position"][:, w]) == ref["pos"], (name, w)
        assert tr["base"][w::W] == ref["base"], (name, w)
        assert list(tr["outcome"][:, w]) == ref["outcome"], (name, w)
        for s in range(STEPS):
            if ref["outcome"][s] == 2:
                continue
            scored += 1
            a, b = tr["proposed_score"][s, w], ref["proposed_score"][s]
            if fold == "mfe":
                assert _close_mfe(a, b), (name, w, s, a, b)
            else:
                assert close_score(a, b, tr["term_values"][s, w], terms), (name, w, s, a, b)
            assert tr["random_threshold"][s, w] == ref["random_threshold"][s]
        assert final[w].upper() == ref["seq"].upper(), (name, w)
        assert list(counters[w]) == ref["counters"], (name, w)
    assert scored > len(sample) * STEPS // 2
