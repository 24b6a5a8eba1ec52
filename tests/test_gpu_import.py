"""Walkers whose configurations were replaced (adx_walkers_import: the
replica-exchange swap of BASELINE config 5) fold from scratch until a proposal
of theirs is accepted; from then on they refold incrementally on that
proposal's tables (the step tail's accept revalidates them).  After the import and 30
more steps every stored score must equal a from-scratch fold of the walker's
configuration by the step's own kernels (adx_walkers_rescore), bit for bit,
and equal the oracle's score (the bound of tests/parity_bounds.py)."""
import numpy as np
import pytest
import torch

from addapt_amd import workloads
from parity_bounds import close_score

pytestmark = pytest.mark.gpu

CASES = {"mfe100": (100, "mfe"), "pf100": (100, "pf"), "pf150": (150, "pf")}


@pytest.mark.parametrize("name", list(CASES))
def test_import_then_incremental(native, oracle, name):
    N, fold = CASES[name]
    W = 256
    tmpl, active = workloads.synthetic(N)
    terms = workloads.default_objective()
    apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
    th = native.make_thermostat("fixed", t=0.6)
    eng = native.Engine(tmpl, [active], terms, aptamer=apt, thermostat=th, fold_mode=fold)
    eng.walkers_init(list(range(W)), workloads.walker_sequences(tmpl, [active], W))
    eng.run_steps(10)
    seqs = torch.empty(W * N, dtype=torch.uint8, device="cuda")
    sc = torch.empty(W, dtype=torch.float64, device="cuda")
    eng.export_walkers(seqs.data_ptr(), sc.data_ptr())
    seqs2 = seqs.view(W, N).roll(1, 0).contiguous()   # every walker takes its neighbour's configuration
    sc2 = sc.roll(1).contiguous()
    torch.cuda.synchronize()
    eng.import_walkers(seqs2.data_ptr(), sc2.data_ptr())
    before, bscores, _ = eng.download()
    assert np.array_equal(bscores, np.roll(sc.cpu().numpy(), 1))
    eng.run_steps(30)
    final, scores, counters = eng.download()
    assert (counters.sum(axis=1) == 40).all()
    accepted = int(counters[:, 1].sum() + counters[:, 3].sum())
    assert accepted > 0
    fresh, _ = eng.rescore()
    bad = np.nonzero(scores != fresh)[0]
    assert bad.size == 0, [(int(w), scores[w], fresh[w]) for w in bad[:8]]
    m = oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, oracle.theo_bonus())
    sf = oracle.ScoreFunction(terms, aptamer=m, mode=fold)
    for w in range(0, W, 37):
        ref, tref = sf.score(final[w], [active])
        if fold == "mfe":
            assert abs(scores[w] - ref) <= 1e-12 * max(1.0, abs(ref)), (w, scores[w], ref)
        else:
            assert close_score(scores[w], ref, tref, terms), (w, scores[w], ref)
