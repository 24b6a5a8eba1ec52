"""Oracle MFE with the ligand motif (fold.c orc_mfe_energy), the energy the
MFE score term (BASELINE config 2) reads.  No GPU.

Checks:
* without a motif it equals the traceback MFE (orc_mfe, already pinned by
  the reference's mfe annotations and by exhaustive enumeration);
* with a contiguous ADD-mode motif (vrna_sc_add_hi_motif, scoring.cc:92-100)
  it equals  min(MFE, min_o MFE(seq | motif forced at o) + bonus)  (bonus
  rounded to dcal/mol: the MFE is integer dcal throughout) -- the
  ligand bonus applies to every structure that contains the motif's pairs
  and unpaired bases at occurrence o (hard constraints: pairs '()' and
  unpaired 'x');
* hard constraints restrict the minimum like the PF's.
"""
import random

import pytest

from addapt_amd import workloads

random.seed(11)
RAND = ["".join(random.choice("ACGU") for _ in range(random.randint(20, 60))) for _ in range(8)]


@pytest.mark.parametrize("seq", RAND + [workloads.THEO_SEQ, workloads.RHF6_SEQ.upper()])
def test_mfe_energy_matches_traceback(oracle, seq):
    e, _ = oracle.mfe(seq)
    assert oracle.mfe_energy(seq) == pytest.approx(e, abs=1e-9)


def _bonus_dcal(oracle):
    return round(oracle.theo_bonus() * 100) / 100


def _motif_forced(seq, o):
    cst = ["."] * len(seq)
    for k, c in enumerate(workloads.THEO_FOLD):
        cst[o + k] = "x" if c == "." else c
    return "".join(cst)


@pytest.mark.parametrize("N", [60, 80, 100])
def test_mfe_with_motif_is_min_over_occurrences(oracle, N):
    seq, _ = workloads.synthetic(N)
    seq = seq.upper()
    m = oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, oracle.theo_bonus(), oracle.MOTIF_ADD)
    occ = [o for o in range(len(seq) - 26) if seq[o:o + 27] == workloads.THEO_SEQ]
    assert occ
    expect = oracle.mfe_energy(seq)
    for o in occ:
        expect = min(expect, oracle.mfe_energy(seq, _motif_forced(seq, o)) + _bonus_dcal(oracle))
    assert oracle.mfe_energy(seq, None, m) == pytest.approx(expect, abs=1e-6)


def test_mfe_theo_holo(oracle):
    seq = workloads.THEO_SEQ
    m = oracle.make_motif(seq, workloads.THEO_FOLD, oracle.theo_bonus(), oracle.MOTIF_ADD)
    e_motif = oracle.eval_structure(seq, workloads.THEO_FOLD)
    assert oracle.mfe_energy(seq, None, m) == pytest.approx(
        min(oracle.mfe_energy(seq), e_motif + _bonus_dcal(oracle)), abs=1e-6)


@pytest.mark.parametrize("N", [60, 100])
def test_constrained_mfe_is_bounded_by_free(oracle, N):
    seq, cst = workloads.synthetic(N)
    seq = seq.upper()
    free = oracle.mfe_energy(seq)
    act = oracle.mfe_energy(seq, cst)
    assert act >= free - 1e-9
    e, s = oracle.mfe(seq, cst)
    assert act == pytest.approx(e, abs=1e-9)


@pytest.mark.parametrize("N", [60, 100])
def test_default_motif_mode_is_auto(oracle, N):
    """The oracle's default motif convention (AUTO, as the engine's): REPLACE in
    MFE folds, ADD in partition functions."""
    seq, _ = workloads.synthetic(N)
    seq = seq.upper()
    b = oracle.theo_bonus()
    mk = lambda *mode: oracle.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, b, *mode)
    assert oracle.mfe_energy(seq, None, mk()) == oracle.mfe_energy(seq, None, mk(oracle.MOTIF_REPLACE))
    assert oracle.pf_energy(seq, None, mk()) == oracle.pf_energy(seq, None, mk(oracle.MOTIF_ADD))
    assert oracle.mfe_energy(seq, None, mk()) > oracle.mfe_energy(seq, None, mk(oracle.MOTIF_ADD))
