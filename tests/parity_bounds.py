"""Score tolerances derived from the north star's fold bar (BASELINE.json:
fold free energies within 1e-4 kcal/mol).

A macrostate term is ln p with p = exp((G_tot - G_act) / kT)
(scoring.cc:53-71, 233-259), so two folds each within DG_TOL move ln p by at
most  e = 2 * DG_TOL / kT  (~3.25e-4 at 37 C).  An unfavourable term is
ln(1 - p); d ln(1 - p) = -p / (1 - p) d ln p, so its bound is e * p / (1 - p).
A base-pair probability P(i, j) is the same kind of ratio (the ensemble of
structures holding (i, j) over the whole ensemble), so pair terms get the same
e (favourable) or e * P / (1 - P) (unfavourable).  A weighted score's bound is
the weighted sum over terms (and contexts), plus a floor for FP64 rounding of
the sum.  The term values the bound reads are the oracle's (or, in a
trajectory replay, the engine's own trace: the bound is insensitive to
errors that small).

MFE folds are integer dcal/mol on both sides: their scores are compared to
1e-12 relative, not with this bound.
"""
import math

DG_TOL = 1e-4                                  # kcal/mol, north_star
KT = (37.0 + 273.15) * 1.98717 / 1000.0        # scoring.cc:69-70
E_TERM = 2.0 * DG_TOL / KT
FLOOR = 1e-9


def term_bound(value, favorable, weight=1.0):
    """Bound on |term_gpu - term_oracle| for one term whose oracle value is
    `value` (ln p if favourable, else ln(1 - p))."""
    if not math.isfinite(value):
        return 0.0                             # p = 0 / 1 exactly: must agree exactly
    if favorable:
        return abs(weight) * E_TERM
    q = math.exp(value)                        # 1 - p
    if q <= 0.0:
        return math.inf
    return abs(weight) * E_TERM * (1.0 - q) / q


def score_bound(term_values, terms):
    """Bound on |score_gpu - score_oracle|; term_values is the flat
    contexts x terms list (orc_score / adx_score_batch order), terms the
    (condition, macrostate|("pair", i, j), favourable, weight) tuples."""
    nt = len(terms)
    tol = FLOOR
    for k, v in enumerate(term_values):
        t = terms[k % nt]
        tol += term_bound(float(v), t[2], t[3])
    return tol


def close_term(a, b, favorable, weight=1.0):
    if not math.isfinite(b):
        return a == b
    return abs(a - b) <= term_bound(b, favorable, 1.0) + FLOOR


def close_score(a, b, term_values, terms):
    if not math.isfinite(b):
        return a == b
    return abs(a - b) <= score_bound(term_values, terms)
