"""Full-size consistency over one whole annealing cycle (BASELINE configs 2 / 3
shape: 4096 walkers x 300 steps at N = 100, annealing 5 -> 0 in 300).

After 300 incremental MC steps every walker's stored score must equal a
from-scratch score of its final sequence (adx_score_batch: no stored tables)
BIT FOR BIT -- the incremental refolds restore unchanged cells and sum every
cell in the order a full fold does -- and the counters must account for every
step.  A third run at N = 150 starts GC-rich walkers whose folds leave the
16-bit MFE path's exact range, so the int16 -> FP32 fallback (KArgs::ovf)
runs inside incremental steps too."""
import numpy as np
import pytest

from addapt_amd import workloads

pytestmark = pytest.mark.gpu


def _run(native, N, W, steps, fold, seqs_fn=None):
    tmpl, active = workloads.synthetic(N)
    terms = workloads.default_objective()
    apt = (workloads.THEO_SEQ, workloads.THEO_FOLD, native.theo_energy())
    th = native.make_thermostat("annealing", t_hi=5.0, t_lo=0.0, cycle_len=300)
    eng = native.Engine(tmpl, [active], terms, aptamer=apt, thermostat=th, fold_mode=fold)
    seqs = workloads.walker_sequences(tmpl, [active], W)
    if seqs_fn:
        seqs = seqs_fn(seqs)
    eng.walkers_init(list(range(W)), seqs)
    sc0, _, dg0 = eng.score_batch(seqs)
    eng.run_steps(steps)
    final, scores, counters = eng.download()
    sc, _, dg = eng.score_batch(final)
    return eng, seqs, final, scores, counters, sc, sc0, dg0


@pytest.mark.parametrize("fold", ["mfe", "pf"])
def test_one_cycle_full_size_consistency(native, fold):
    W, steps = 4096, 300
    eng, seqs, final, scores, counters, sc, _, _ = _run(native, 100, W, steps, fold)
    assert (counters.sum(axis=1) == steps).all()
    assert int(counters.sum()) == W * steps
    assert int(counters[:, 2].sum()) > 0 and int(counters[:, 3].sum()) > 0   # unchanged and improved steps
    moved = sum(1 for a, b in zip(seqs, final) if a != b)
    assert moved > W // 2, moved
    assert np.isfinite(scores).all()
    bad = np.nonzero(scores != sc)[0]
    assert bad.size == 0, [(int(w), scores[w], sc[w]) for w in bad[:8]]


def test_one_cycle_mfe_int16_fallback_inside_steps(native):
    """GC-rich walkers at N = 150: their first folds are below -120 kcal/mol (the
    packed 16-bit path's exact range), so the FP32 refold of KArgs::ovf runs
    inside the MC steps; the stored scores still equal from-scratch scores."""
    N, W, steps = 150, 256, 300
    o = (N - 27) // 2

    def gc_rich(seqs):
        out = []
        for w, s in enumerate(seqs):
            if w % 4 == 1:
                s = list(s)
                for i, c in enumerate(s):
                    if c.isupper() and 6 <= i < N - 6 and not (o - 6 <= i < o + 33):
                        s[i] = "G" if i < N // 2 else "C"
                s = "".join(s)
            out.append(s)
        return out

    eng, seqs, final, scores, counters, sc, sc0, dg0 = _run(native, N, W, steps, "mfe", gc_rich)
    deep = [w for w in range(W) if w % 4 == 1]
    assert (dg0[deep].min(axis=1) < -120.0).all(), dg0[deep].min(axis=1)[:8]
    assert (counters.sum(axis=1) == steps).all()
    bad = np.nonzero(scores != sc)[0]
    assert bad.size == 0, [(int(w), scores[w], sc[w]) for w in bad[:8]]
