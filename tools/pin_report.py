#!/usr/bin/env python3
"""Report the oracle against every fold value the reference's tests hold.

The five RNAfold annotations (test_scoring.cc:52-55, 86-87, 152-154) and the
macrostate / base-pair-probability thresholds (test_scoring.cc:83-259), for
a parameter file (default: the shipped one) and a motif mode (default AUTO = 0,
the engine's default: ADD in partition functions, REPLACE in the MFE; 1 = ADD,
2 = REPLACE),
plus the 204 per-position ensemble classes of rhf(6) (test_scoring.cc:54-55,
tests/pseudo_bracket.py).  The holo aptamer MFE annotation -9.22 is RNAfold's
MFE under the REPLACE reading; it is reported for REPLACE and, as information,
for the chosen mode.

Usage: python tools/pin_report.py [params.par] [motif_mode]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from addapt_amd import workloads  # noqa: E402
from oracle import oracle as O  # noqa: E402

HAIRPIN = "ACGUGAAAACGU"


def main():
    par = sys.argv[1] if len(sys.argv) > 1 else O.DEFAULT_PAR
    mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    P = O.Params(par)
    theo = O.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, O.theo_bonus(), mode)
    rhf = workloads.RHF6_SEQ.upper()
    rows = []

    def ann(name, got, want):
        rows.append((abs(got - want) <= 0.005, name, "%.4f" % got, "%.2f" % want))

    e, s = O.mfe(HAIRPIN, params=P)
    ann("hairpin MFE " + s, e, -2.20)
    e, s = O.mfe(workloads.THEO_SEQ, params=P)
    ann("THEO apo MFE " + s, e, -6.20)
    theo_rep = O.make_motif(workloads.THEO_SEQ, workloads.THEO_FOLD, O.theo_bonus(), O.MOTIF_REPLACE)
    ann("THEO holo MFE (REPLACE)", O.mfe_energy(workloads.THEO_SEQ, None, theo_rep, params=P), -9.22)
    info = [("THEO holo MFE (mode %d)" % mode, O.mfe_energy(workloads.THEO_SEQ, None, theo, params=P), -9.22)]
    ann("rhf(6) apo ensemble", O.pf_energy(rhf, params=P), -29.58)
    ann("rhf(6) holo ensemble", O.pf_energy(rhf, None, theo, params=P), -33.82)

    def thr(name, p, op, t):
        rows.append(((p > t) if op == ">" else (p < t), name, "%.4g" % p, op + " %g" % t))

    for cst, op, t in [("...(....)...", ">", 0.95), ("..((....))..", ">", 0.85),
                       (".(((....))).", ">", 0.75), ("((((....))))", ">", 0.65),
                       ("(((......)))", ">", 0.65), ("((........))", ">", 0.65),
                       ("(..........)", ">", 0.65), ("xxxxxxxxxxxx", "<", 0.05),
                       ("xxxx........", "<", 0.05), ("....xxxx....", ">", 0.95),
                       ("........xxxx", "<", 0.05)]:
        thr("hairpin " + cst, O.macrostate_prob(HAIRPIN, cst, params=P), op, t)
    for holo, cst, op, t in [(False, "....((((((....)))...)))....", ">", 0.65),
                             (False, "(.........................)", "<", 0.05),
                             (True, "....((((((....)))...)))....", "<", 0.01),
                             (True, "(.........................)", ">", 0.95)]:
        thr(("holo " if holo else "apo ") + cst,
            O.macrostate_prob(workloads.THEO_SEQ, cst, theo if holo else None, params=P), op, t)
    thr("rhf(6) apo active", O.macrostate_prob(rhf, workloads.RHF6_ACTIVE, params=P), "<", 7e-5)
    thr("rhf(6) holo active", O.macrostate_prob(rhf, workloads.RHF6_ACTIVE, theo, params=P), ">", 4e-3)

    _, Ph = O.bppm(HAIRPIN, params=P)
    exp = {(0, 11): 0.70, (1, 10): 0.95, (2, 9): 0.95, (3, 8): 0.95}
    for (i, j), t in exp.items():
        thr("hairpin P%s" % ((i, j),), Ph[i, j], ">", t)
    n = len(HAIRPIN)
    worst = max(Ph[i, j] for i in range(n) for j in range(i, n) if (i, j) not in exp)
    thr("hairpin other P max", worst, "<", 0.1)

    seq = workloads.THEO_SEQ
    _, Pa = O.bppm(seq, params=P)
    _, Pho = O.bppm(seq, None, theo, params=P)
    apo_pairs = {(4, 22), (5, 21), (6, 20), (7, 16), (8, 15), (9, 14)}
    holo_pairs = {(0, 26), (4, 22), (5, 21), (7, 16), (8, 15), (9, 14)}
    n = len(seq)
    for name, PP, pairs in (("THEO apo", Pa, apo_pairs), ("THEO holo", Pho, holo_pairs)):
        for (i, j) in sorted(pairs):
            thr("%s P%s" % (name, (i, j)), PP[i, j], ">", 0.7)
        worst = max(PP[i, j] for i in range(n) for j in range(i, n) if (i, j) not in pairs)
        thr("%s other P max" % name, worst, "<", 0.3)

    _, Ra = O.bppm(rhf, params=P)
    _, Rh = O.bppm(rhf, None, theo, params=P)
    constitutive = {(0, 29): 0.75, (1, 28): 0.80, (2, 27): 0.85, (3, 26): 0.85, (4, 25): 0.85,
                    (5, 24): 0.85, (6, 23): 0.80, (8, 19): 0.95, (9, 18): 0.95, (10, 17): 0.95,
                    (11, 16): 0.95, (81, 95): 0.90, (82, 94): 0.90, (83, 93): 0.90,
                    (84, 92): 0.90, (85, 91): 0.90, (86, 90): 0.75}
    for (i, j), t in constitutive.items():
        thr("rhf apo P%s" % ((i, j),), Ra[i, j], ">", t)
        thr("rhf holo P%s" % ((i, j),), Rh[i, j], ">", t)
    apo = {(33, 73): 0.30, (34, 72): 0.30, (35, 71): 0.30, (36, 70): 0.25, (37, 69): 0.10,
           (40, 65): 0.35, (41, 64): 0.35, (42, 63): 0.35, (43, 62): 0.35, (44, 61): 0.30,
           (45, 60): 0.25, (47, 58): 0.35, (48, 57): 0.40}
    for (i, j), t in apo.items():
        thr("rhf apo-only apo P%s" % ((i, j),), Ra[i, j], ">", t)
        thr("rhf apo-only holo P%s" % ((i, j),), Rh[i, j], "<", 1e-3)
    holo = {(30, 43): (0.55, 0.25), (31, 42): (0.75, 0.35), (32, 41): (0.75, 0.35),
            (33, 40): (0.75, 0.35), (46, 80): (0.50, 0.05), (47, 79): (0.60, 0.05),
            (49, 77): (0.85, 0.05), (50, 76): (0.95, 0.05), (54, 72): (0.95, 0.20),
            (55, 71): (0.95, 0.20), (57, 66): (0.95, 0.50), (58, 65): (0.95, 0.50),
            (59, 64): (0.95, 0.50)}
    for (i, j), (th, ta) in holo.items():
        thr("rhf holo-only apo P%s" % ((i, j),), Ra[i, j], "<", ta)
        thr("rhf holo-only holo P%s" % ((i, j),), Rh[i, j], ">", th)

    from tests.pseudo_bracket import APO_ANNOT, HOLO_ANNOT, position_probs, pseudo_bracket
    for name, Rm, annot in (("apo", Ra, APO_ANNOT), ("holo", Rh, HOLO_ANNOT)):
        pb = pseudo_bracket(position_probs(Rm))
        for k, (got, want) in enumerate(zip(pb, annot)):
            rows.append((got == want, "rhf %s ensemble class [%d]" % (name, k), got, want))

    bad = 0
    for name, got, want in info:
        print("info %-44s %-12.4f %.2f" % (name, got, want))
    for ok, name, got, want in rows:
        if not ok or "-v" in sys.argv:
            print("%-4s %-44s %-12s %s" % ("ok" if ok else "FAIL", name, got, want))
        bad += not ok
    print("%d / %d pins hold (%s, motif mode %d)" % (len(rows) - bad, len(rows), os.path.basename(par), mode))


if __name__ == "__main__":
    main()
