"""Synthetic workloads of BASELINE.json.

* rhf(6): the 102-nt device of the reference's tests
  (/root/reference/tests/test_scoring.cc:50-63), THEO aptamer (:45-48).
* synthetic(N): random ACGU template from mt19937(20161015) with the THEO
  aptamer frozen (lower case) at offset (N-27)//2, macrostate "active" =
  enforced 6-bp helix (0..5 with N-6..N-1) + 'x' on the 6 nt flanking the
  aptamer; walker w re-randomises its mutable bases from mt19937(1000 + w) and
  runs with MC seed w.

The generator uses its own mt19937 / libstdc++-uniform_int code (no oracle).
"""
THEO_SEQ = "GAUACCAGCCGAAAGGCCCUUGGCAGC"
THEO_FOLD = "(...((.(((....)))....))...)"
THEO_KD_UM = 0.32

RHF6_SEQ = ("guuuuagagcuagaaauagcaaguuaaaauaaggcuaguccCuUUUCGCCgauaccagccgaaaggcccuuggcagc"
            "GACggcaccgagucggugcuuuuuu")
RHF6_ACTIVE = ("(............................)xx..xxxxx..xxxxxx(...............................)"
               ".(.............)......")

COMP = {"A": "U", "U": "A", "G": "C", "C": "G"}


class MT19937:
    def __init__(self, seed):
        self.mt = [0] * 624
        self.mt[0] = seed & 0xFFFFFFFF
        for i in range(1, 624):
            prev = self.mt[i - 1]
            self.mt[i] = (1812433253 * (prev ^ (prev >> 30)) + i) & 0xFFFFFFFF
        self.idx = 624

    def _twist(self):
        mt = self.mt
        for i in range(624):
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
            mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.idx = 0

    def __call__(self):
        if self.idx >= 624:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    def uniform_int(self, a, b):
        """libstdc++ >= 11 uniform_int_distribution<int>(a, b) (Lemire)."""
        R = (b - a + 1) & 0xFFFFFFFF
        prod = self() * R
        low = prod & 0xFFFFFFFF
        if low < R:
            thr = ((-R) & 0xFFFFFFFF) % R
            while low < thr:
                prod = self() * R
                low = prod & 0xFFFFFFFF
        return a + (prod >> 32)


def synthetic(N=100, seed=20161015):
    """Return (template, active_macrostate) for config 2-5 style runs."""
    if N < 27 + 2 * 6 + 12 + 8:
        raise ValueError("N too small for the synthetic layout")
    g = MT19937(seed)
    seq = ["ACGU"[g.uniform_int(0, 3)] for _ in range(N)]
    o = (N - 27) // 2
    for k in range(27):
        seq[o + k] = THEO_SEQ[k].lower()
    cst = ["."] * N
    for k in range(6):
        cst[k] = "("
        cst[N - 1 - k] = ")"
        seq[N - 1 - k] = COMP[seq[k]]
    for k in range(1, 7):
        cst[o - k] = "x"
        cst[o + 27 - 1 + k] = "x"
    return "".join(seq), "".join(cst)


def walker_sequences(template, macrostates, W, seed_base=1000):
    """Walker w: re-randomise every freely mutable base from mt19937(seed_base + w),
    writing Watson-Crick complements on constrained partners."""
    N = len(template)
    partner = {}
    for m in macrostates:
        stk = []
        for i, c in enumerate(m):
            if c == "(":
                stk.append(i)
            elif c == ")":
                a = stk.pop()
                partner.setdefault(a, set()).add(i)
                partner.setdefault(i, set()).add(a)
    free = [i for i in range(N) if template[i].isupper() and all(m[i] != ")" for m in macrostates)]
    out = []
    for w in range(W):
        g = MT19937(seed_base + w)
        s = list(template)
        for i in free:
            b = "ACGU"[g.uniform_int(0, 3)]
            s[i] = b
            stack = [(i, b)]
            seen = {i}
            while stack:
                p, bp = stack.pop()
                for q in partner.get(p, ()):
                    if q not in seen:
                        seen.add(q)
                        s[q] = COMP[bp]
                        stack.append((q, COMP[bp]))
        out.append("".join(s))
    return out


def config_objective(N, bppm=False, active_index=0):
    """Objective of the bench configs: the default objective (configs 2, 5), plus
    (configs 3-4) apo/holo base-pair probability terms on the outermost pair of
    the enforced helix: apo "not pair(0, N-1)", holo "pair(0, N-1)"."""
    terms = default_objective(active_index)
    if bppm:
        terms = terms + [("apo", ("pair", 0, N - 1), False, 1.0), ("holo", ("pair", 0, N - 1), True, 1.0)]
    return terms


def default_objective(active_index=0):
    """objective: {apo: "not active", holo: "active"} (config.cc:72-81)."""
    return [("apo", active_index, False, 1.0), ("holo", active_index, True, 1.0)]
