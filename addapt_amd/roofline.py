"""Algorithmic work of one McCaskill inside pass (for bench.py's roofline).

FLOPs per partition function (DESIGN.md "Roofline"):
  3 per interior-loop term  qb[p][q] * f(i,j,p,q) accumulated, counted for
                            every pair of pairable cells (i,j) ⊃ (p,q) with
                            n1 + n2 <= 30 allowed by the hard constraint;
  2 per multiloop-closing term qm[i+1][k-1] * qm1[k][j-1], k in [i+6, j-5],
                            for every pairable (i,j);
  2 per qm split term       (pre + qm[i][k-1]) * qm1[k][j], k in [i, j-4],
                            for every cell (i,j) with 4 <= j-i <= N-6.
Exterior, hairpin and O(1)-per-cell work are not counted.  Pure numpy, no
oracle (the product may not call the checker).

The MFE (min-plus) pass visits the same terms: 2 ops per interior term
(c[p][q] + E, min) and 2 per multiloop / split term (add, min).

The outside pass (bppm_kernel) gathers the same interior terms (3 FLOP each)
and two multiloop sums per cell: qmb (N - j - 4 split terms, 2 FLOP) and qm1b
(i - 1 terms of two products, 4 FLOP).
"""
import numpy as np

PAIR = np.zeros((5, 5), dtype=np.int8)
for a, b, t in ((2, 3, 1), (3, 2, 2), (3, 4, 3), (4, 3, 4), (1, 4, 5), (4, 1, 6)):
    PAIR[a, b] = t
CODE = {"A": 1, "C": 2, "G": 3, "U": 4, "T": 4}


def _hc(cst, N):
    """allowed[i][j] (1-based) and up/dn runs for a dot-bracket constraint."""
    partner = np.zeros(N + 2, dtype=np.int64)
    enc = np.zeros(N + 2, dtype=np.int64)
    unp = np.ones(N + 2, dtype=bool)
    flg = np.zeros(N + 2, dtype=np.int64)
    stk = []
    for i in range(1, N + 1):
        c = cst[i - 1] if cst else "."
        enc[i] = stk[-1] if stk else 0
        if c == "(":
            stk.append(i)
        elif c == ")":
            a = stk.pop()
            partner[a], partner[i] = i, a
            enc[i] = stk[-1] if stk else 0
        if c == "x":
            flg[i] |= 1
        if c == "<":
            flg[i] |= 2
        if c == ">":
            flg[i] |= 4
        if c in "|<>" or c in "()":
            unp[i] = False
    I = np.arange(N + 2)[:, None]
    J = np.arange(N + 2)[None, :]
    fi, fj = flg[:, None], flg[None, :]
    ok = ((fi | fj) & 1) == 0
    ok &= (fi & 2) == 0
    ok &= (fj & 4) == 0
    pi, pj = partner[:, None], partner[None, :]
    ok &= np.where(pi > 0, pi == J, np.where(pj > 0, pj == I, enc[:, None] == enc[None, :]))
    up = np.zeros(N + 3, dtype=np.int64)
    for i in range(N, 0, -1):
        up[i] = up[i + 1] + 1 if unp[i] else 0
    dn = np.zeros(N + 2, dtype=np.int64)
    for i in range(1, N + 1):
        dn[i] = dn[i - 1] + 1 if unp[i] else 0
    return ok, up, dn


def pf_terms(seq, cst=None):
    """(interior terms, multiloop terms) of one inside pass."""
    N = len(seq)
    S = np.zeros(N + 2, dtype=np.int64)
    S[1:N + 1] = [CODE.get(c.upper(), 0) for c in seq]
    ok, up, dn = _hc(cst, N)
    I = np.arange(N + 2)[:, None]
    J = np.arange(N + 2)[None, :]
    pairable = (PAIR[S[:, None], S[None, :]] > 0) & ok & (J - I >= 4)
    pairable[0, :] = pairable[:, 0] = False
    pairable[N + 1, :] = pairable[:, N + 1] = False
    n_int = 0
    ii, jj = np.nonzero(pairable)
    for i, j in zip(ii, jj):
        for n1 in range(0, 31):
            p = i + 1 + n1
            if p >= j - 4 or (n1 > 0 and up[i + 1] < n1):
                break
            n2max = min(30 - n1, j - 1 - (p + 4))
            if n2max < 0:
                continue
            qs = np.arange(j - 1, j - 2 - n2max, -1)
            n2s = j - 1 - qs
            valid = (n2s == 0) | (dn[j - 1] >= n2s)
            n_int += int(np.count_nonzero(pairable[p, qs] & valid))
    d = jj - ii
    n_ml = int(np.clip(d - 10, 0, None).sum())
    dd = np.arange(4, max(4, N - 5))
    n_ml += int(((N - dd) * (dd - 3)).sum())
    return n_int, n_ml


def cell_terms(seq, cst=None):
    """Per-cell term counts of one inside pass, (N+2) x (N+2), 1-based:
    interior terms of the pairable (i, j) (as pf_terms), its multiloop-closing
    terms, and the qm split terms of (i, j).  Sums over all cells equal
    pf_terms; sums over the refolded band give an incremental refold's work."""
    N = len(seq)
    S = np.zeros(N + 2, dtype=np.int64)
    S[1:N + 1] = [CODE.get(c.upper(), 0) for c in seq]
    ok, up, dn = _hc(cst, N)
    I = np.arange(N + 2)[:, None]
    J = np.arange(N + 2)[None, :]
    pairable = (PAIR[S[:, None], S[None, :]] > 0) & ok & (J - I >= 4)
    pairable[0, :] = pairable[:, 0] = False
    pairable[N + 1, :] = pairable[:, N + 1] = False
    pad = np.zeros((N + 2 + 32, N + 2 + 32), dtype=bool)
    pad[:N + 2, :N + 2] = pairable
    upi = up[np.minimum(np.arange(N + 2) + 1, N + 1)][:, None]   # up[i + 1]
    dnj = dn[np.maximum(np.arange(N + 2) - 1, 0)][None, :]       # dn[j - 1]
    n_int = np.zeros((N + 2, N + 2), dtype=np.int64)
    Ii = np.broadcast_to(I, (N + 2, N + 2))
    Jj = np.broadcast_to(J, (N + 2, N + 2))
    for n1 in range(0, 31):
        for n2 in range(0, 31 - n1):
            P = Ii + 1 + n1
            Q = Jj - 1 - n2
            m = pairable & (Q - P >= 4)
            if n1 > 0:
                m &= upi >= n1
            if n2 > 0:
                m &= dnj >= n2
            m &= pad[P, np.maximum(Q, 0)]
            n_int += m
    n_mlc = np.where(pairable, np.clip(J - I - 10, 0, None), 0)
    d = J - I
    n_split = np.where((d >= 4) & (d <= N - 6) & (I >= 1) & (J <= N), d - 3, 0)
    return n_int, n_mlc, n_split


def band_mask(N, m_lo, m_hi, widen=1):
    """Cells (i, i+d) an incremental refold recomputes for changed positions
    m_lo..m_hi (1-based): rows max(1, m_lo-w-d) .. min(N-d, m_hi+w), w = widen
    (1 for the fold cells, 2 for the qm rows; mfe_cells.hip clo/chi, qlo/qhi).
    m_lo = None: the whole triangle (a fold from scratch)."""
    I = np.arange(N + 2)[:, None]
    J = np.arange(N + 2)[None, :]
    d = J - I
    tri = (I >= 1) & (J <= N) & (d >= 0)
    if m_lo is None:
        return tri
    return tri & (I >= np.maximum(1, m_lo - widen - d)) & (I <= np.minimum(N - d, m_hi + widen))


def band_terms(counts, m_lo, m_hi):
    """(interior, multiloop) terms of the cells a refold over m_lo..m_hi recomputes."""
    n_int, n_mlc, n_split = counts
    N = n_int.shape[0] - 2
    f = band_mask(N, m_lo, m_hi, 1)
    q = band_mask(N, m_lo, m_hi, 2)
    return int(n_int[f].sum()), int(n_mlc[f].sum() + n_split[q].sum())


def pf_flops(seq, cst=None):
    a, b = pf_terms(seq, cst)
    return 3 * a + 2 * b


def mfe_ops(seq, cst=None):
    a, b = pf_terms(seq, cst)
    return 2 * a + 2 * b


def outside_flops(seq, cst=None):
    a, _ = pf_terms(seq, cst)
    N = len(seq)
    ml = 0
    for d in range(4, N):
        for i in range(1, N - d + 1):
            j = i + d
            ml += 2 * max(0, N - j - 4) + 4 * (i - 1)
    return 3 * a + ml


# gfx950 VALU peaks (MI355X_MICROARCH.md: 256 CUs, 2.4 GHz).
# 4 SIMD-32 per CU, a wave64 VALU instruction in 2 cycles (MI355X_MICROARCH.md):
# 128 lane-instructions per clock per CU
CUS, CLOCK_HZ, LANE_OPS_PER_CLK = 256, 2.4e9, 128


def valu_peak(fold):
    """(peak, note) in TFLOP/s (pf) or Top/s (mfe) for the work bench.py counts."""
    if fold == "pf":
        return 157.3, ("fp32 VALU (no MFMA: the McCaskill recurrence is a sum of data-dependent "
                       "products, not a contraction); peak = gfx950 fp32 vector rate (packed FMA), "
                       "157.3 TFLOP/s")
    peak = CUS * CLOCK_HZ * LANE_OPS_PER_CLK * 2 / 1e12
    return peak, ("packed int16 VALU (v_pk_add_i16 / v_pk_min_i16 on apo|holo halves; min-plus is "
                  "not an MFMA contraction); peak = 256 CUs x 128 lanes/clk x 2 halves x 2.4 GHz = "
                  "%.1f Top/s" % peak)
