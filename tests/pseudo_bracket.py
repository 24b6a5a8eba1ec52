"""ViennaRNA's ensemble pseudo-bracket classes, restated for the parity tests.

RNAfold -p prints, under the MFE structure, one character per position that
classes the position's pairing in the Boltzmann ensemble (the line the
reference's fixtures hold at /root/reference/tests/test_scoring.cc:54-55,
made by RNAfold --MEA [--motif ...], /root/reference/tools/test_seq:8-9).
ViennaRNA's published rule (RNAfold(1) man page, "-p": "'.' and ',' for
unpaired ... '|' for paired ... '{' '}' for weakly paired upstream /
downstream, '(' ')' for strongly paired"; the thresholds are those of
vrna_bpp_symbol: 0.667 on single-precision sums):

    P0 = P(unpaired), P1 = sum_j>i P(i.j) (pairs upstream), P2 = sum_j<i P(j.i)
    P0 > 0.667 -> '.';  P1 > 0.667 -> '(';  P2 > 0.667 -> ')'
    P1 + P2 > P0 -> '{' if P1/(P1+P2) > 0.667, '}' if P2/(P1+P2) > 0.667, else '|'
    P0 > P1 + P2 -> ','   else ':'

The sums are accumulated in float32 as vrna_db_from_probs does.
"""
import numpy as np

# /root/reference/tests/test_scoring.cc:54-55 (rhf(6), 102 nt): RNAfold's
# ensemble classes of the apo fold and of the holo fold (THEO motif, -9.22).
APO_ANNOT = ("(((((((.((((....))))...))))))).,,({{,{..|||{{(,((,{....,.||{}}}})),..,}))).,,||."
             "(((((((...))))))).....")
HOLO_ANNOT = ("(((((((.((((....))))...))))))){(((......)))}..{{.((...((.(((....)))....))...)).}|"
              "((((((...)))))),.....")
APO_DG, HOLO_DG = -29.58, -33.82   # the same lines' ensemble free energies (kcal/mol)

T = np.float32(0.667)


def position_probs(P):
    """[(P0, P1, P2)] per position from an upper-triangular pair-probability matrix."""
    n = P.shape[0]
    out = []
    for k in range(n):
        up, dn, un = np.float32(0), np.float32(0), np.float32(1)
        for i in range(k):
            dn += np.float32(P[i, k])
            un -= np.float32(P[i, k])
        for j in range(k + 1, n):
            up += np.float32(P[k, j])
            un -= np.float32(P[k, j])
        out.append((un, up, dn))
    return out


def symbol(x):
    p0, p1, p2 = (np.float32(v) for v in x)
    if p0 > T:
        return "."
    if p1 > T:
        return "("
    if p2 > T:
        return ")"
    if p1 + p2 > p0:
        if p1 / (p1 + p2) > T:
            return "{"
        if p2 / (p1 + p2) > T:
            return "}"
        return "|"
    if p0 > p1 + p2:
        return ","
    return ":"


def pseudo_bracket(probs):
    return "".join(symbol(x) for x in probs)


def class_margin(x, want):
    """Signed distance of position probabilities x from the nearest boundary of class
    `want` (> 0: x is in the class; the minimum over the rule's inequalities)."""
    p0, p1, p2 = (float(v) for v in x)
    t = 0.667
    s = p1 + p2
    conds = {
        ".": [p0 - t],
        "(": [t - p0, p1 - t],
        ")": [t - p0, t - p1, p2 - t],
        "{": [t - p0, t - p1, t - p2, s - p0, (p1 / s - t) if s else -1.0],
        "}": [t - p0, t - p1, t - p2, s - p0, (t - p1 / s) if s else -1.0, (p2 / s - t) if s else -1.0],
        "|": [t - p0, t - p1, t - p2, s - p0, (t - p1 / s) if s else -1.0, (t - p2 / s) if s else -1.0],
        ",": [t - p0, t - p1, t - p2, p0 - s],
    }[want]
    return min(conds)
