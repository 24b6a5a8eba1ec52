"""ctypes wrapper around oracle/_build/liboracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package (addapt_amd/).
See adx_oracle.h for what is restated and how it is pinned.
"""
import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")
DEFAULT_PAR = os.path.join(os.path.dirname(HERE), "addapt_amd", "data", "rna_turner2004_addapt.par")
KT_KCAL = (37.0 + 273.15) * 1.98717 / 1000.0

REJECT, ACCEPT_WORSENED, ACCEPT_UNCHANGED, ACCEPT_IMPROVED = range(4)
OUTCOME_NAMES = ["REJECT", "ACCEPT_WORSENED", "ACCEPT_UNCHANGED", "ACCEPT_IMPROVED"]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


class Motif(C.Structure):
    _fields_ = [("seq", C.c_char_p), ("fold", C.c_char_p), ("energy_kcal", C.c_double),
                ("mode", C.c_int)]


class Term(C.Structure):
    _fields_ = [("condition", C.c_int), ("macrostate", C.c_int), ("favorable", C.c_int),
                ("weight", C.c_double), ("kind", C.c_int), ("pair_i", C.c_int), ("pair_j", C.c_int)]


class Context(C.Structure):
    _fields_ = [("before", C.c_char_p), ("after", C.c_char_p)]


class ScoreFxn(C.Structure):
    _fields_ = [("P", C.c_void_p), ("n_terms", C.c_int), ("terms", C.POINTER(Term)),
                ("aptamer", C.POINTER(Motif)), ("n_contexts", C.c_int),
                ("contexts", C.POINTER(Context)), ("mode", C.c_int)]


class Thermostat(C.Structure):
    _fields_ = [("kind", C.c_int), ("t_fixed", C.c_double), ("t_hi", C.c_double),
                ("t_lo", C.c_double), ("cycle_len", C.c_int), ("target_rate", C.c_double),
                ("period", C.c_int), ("t_init", C.c_double)]


class Trace(C.Structure):
    _fields_ = [("pos", C.POINTER(C.c_int)), ("base", C.c_char_p), ("outcome", C.POINTER(C.c_int)),
                ("temperature", C.POINTER(C.c_double)), ("proposed_score", C.POINTER(C.c_double)),
                ("current_score", C.POINTER(C.c_double)),
                ("random_threshold", C.POINTER(C.c_double)), ("seqs", C.c_char_p)]


class McOpts(C.Structure):
    _fields_ = [("tie_eps", C.c_double), ("forced_outcome", C.POINTER(C.c_int))]


class MT(C.Structure):
    _fields_ = [("mt", C.c_uint32 * 624), ("idx", C.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_params_load.restype = C.c_void_p
        L.orc_params_load.argtypes = [C.c_char_p]
        L.orc_last_error.restype = C.c_char_p
        L.orc_mfe_energy.restype = C.c_double
        L.orc_mfe_energy.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(Motif)]
        L.orc_pf_energy.restype = C.c_double
        L.orc_pf_energy.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(Motif)]
        L.orc_pf_energy_counted.restype = C.c_double
        L.orc_pf_energy_counted.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(Motif),
                                            C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.orc_bppm.restype = C.c_double
        L.orc_bppm.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(Motif),
                               C.POINTER(C.c_double)]
        L.orc_eval_structure.restype = C.c_double
        L.orc_eval_structure.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
        L.orc_mfe.restype = C.c_int
        L.orc_mfe.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_char_p]
        L.orc_mt_seed.argtypes = [C.POINTER(MT), C.c_uint32]
        L.orc_mt_next.restype = C.c_uint32
        L.orc_mt_next.argtypes = [C.POINTER(MT)]
        L.orc_uniform_int.restype = C.c_int
        L.orc_uniform_int.argtypes = [C.POINTER(MT), C.c_int, C.c_int]
        L.orc_canonical.restype = C.c_double
        L.orc_canonical.argtypes = [C.POINTER(MT)]
        L.orc_nth_element.restype = None
        L.orc_nth_element.argtypes = [C.POINTER(C.c_double), C.c_long, C.c_long]
        L.orc_auto_clamp.restype = C.c_double
        L.orc_auto_clamp.argtypes = [C.c_double]
        L.orc_mutate_recursively.restype = C.c_int
        L.orc_mutate_recursively.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.c_int,
                                             C.c_int, C.c_char]
        L.orc_can_be_freely_mutated.restype = C.c_int
        L.orc_can_be_freely_mutated.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_char_p),
                                                C.c_int, C.c_int]
        L.orc_score.restype = C.c_double
        L.orc_score.argtypes = [C.POINTER(ScoreFxn), C.c_char_p, C.c_int, C.POINTER(C.c_char_p),
                                C.c_int, C.POINTER(C.c_double)]
        L.orc_mc_run.restype = C.c_int
        L.orc_mc_run.argtypes = [C.POINTER(ScoreFxn), C.c_char_p, C.c_int, C.POINTER(C.c_char_p),
                                 C.c_int, C.POINTER(Thermostat), C.c_uint32, C.c_int,
                                 C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(Trace),
                                 C.POINTER(McOpts)]
        L.orc_mc_run_batch.restype = C.c_double
        L.orc_mc_run_batch.argtypes = [C.POINTER(ScoreFxn), C.c_char_p, C.c_int, C.c_int,
                                       C.POINTER(C.c_char_p), C.c_int, C.POINTER(Thermostat),
                                       C.POINTER(C.c_uint32), C.c_int, C.c_int,
                                       C.POINTER(C.c_int64)]
        _lib = L
    return _lib


def _b(s):
    return s.encode() if isinstance(s, str) else s


def _strarr(strs):
    arr = (C.c_char_p * max(1, len(strs)))()
    for k, s in enumerate(strs):
        arr[k] = _b(s)
    return arr


class Params:
    def __init__(self, path=DEFAULT_PAR):
        self.ptr = lib().orc_params_load(_b(path))
        if not self.ptr:
            raise RuntimeError(lib().orc_last_error().decode())


_default_params = None


def default_params():
    global _default_params
    if _default_params is None:
        _default_params = Params()
    return _default_params


MOTIF_AUTO, MOTIF_ADD, MOTIF_REPLACE = 0, 1, 2   # the engine's ADX_MOTIF_* numbering


def make_motif(seq, fold, energy_kcal, mode=MOTIF_AUTO):
    """mode MOTIF_AUTO (0, default as the engine: ADD in PF, REPLACE in MFE),
    MOTIF_ADD (1), MOTIF_REPLACE (2)."""
    m = Motif(_b(seq), _b(fold), energy_kcal, mode)
    m._keep = (seq, fold)
    return m


def theo_bonus(kd_uM=0.32):
    """kT * ln(Kd / 1e6) as in scoring.cc:92-100 (kcal/mol)."""
    return KT_KCAL * math.log(kd_uM / 1e6)


def pf_energy(seq, constraint=None, motif=None, params=None):
    P = params or default_params()
    return lib().orc_pf_energy(P.ptr, _b(seq), _b(constraint) if constraint else None,
                               C.byref(motif) if motif is not None else None)


def pf_energy_counted(seq, constraint=None, motif=None, params=None):
    P = params or default_params()
    a, b = C.c_int64(0), C.c_int64(0)
    g = lib().orc_pf_energy_counted(P.ptr, _b(seq), _b(constraint) if constraint else None,
                                    C.byref(motif) if motif is not None else None,
                                    C.byref(a), C.byref(b))
    return g, a.value, b.value


def bppm(seq, constraint=None, motif=None, params=None):
    P = params or default_params()
    n = len(seq)
    out = np.zeros((n, n), dtype=np.float64)
    g = lib().orc_bppm(P.ptr, _b(seq), _b(constraint) if constraint else None,
                       C.byref(motif) if motif is not None else None,
                       out.ctypes.data_as(C.POINTER(C.c_double)))
    return g, out


def eval_structure(seq, structure, params=None):
    P = params or default_params()
    return lib().orc_eval_structure(P.ptr, _b(seq), _b(structure))


def mfe_energy(seq, constraint=None, motif=None, params=None):
    """MFE (kcal/mol) incl. the ligand motif (fold.c orc_mfe_energy)."""
    P = params or default_params()
    return lib().orc_mfe_energy(P.ptr, _b(seq), _b(constraint) if constraint else None,
                                C.byref(motif) if motif is not None else None)


def mfe(seq, constraint=None, params=None):
    P = params or default_params()
    buf = C.create_string_buffer(len(seq) + 1)
    e = lib().orc_mfe(P.ptr, _b(seq), _b(constraint) if constraint else None, buf)
    return e / 100.0, buf.value.decode()


def macrostate_prob(seq, constraint, motif=None, params=None):
    """ViennaRnaFold::macrostate_prob (scoring.cc:53-71) incl. the float return of vrna_pf."""
    g_tot = float(np.float32(pf_energy(seq, None, motif, params)))
    g_act = float(np.float32(pf_energy(seq, constraint, motif, params)))
    return math.exp((g_tot - g_act) / KT_KCAL)


class Rng:
    def __init__(self, seed):
        self.s = MT()
        lib().orc_mt_seed(C.byref(self.s), seed)

    def next(self):
        return lib().orc_mt_next(C.byref(self.s))

    def uniform_int(self, a, b):
        return lib().orc_uniform_int(C.byref(self.s), a, b)

    def canonical(self):
        return lib().orc_canonical(C.byref(self.s))


def nth_element(values, k):
    """std::nth_element(v, v + k, v + n) as libstdc++ 11 runs it; returns the
    rearranged list (the reference's median step, sampling.cc:389-393)."""
    a = (C.c_double * len(values))(*values)
    lib().orc_nth_element(a, k, len(values))
    return list(a)


def auto_clamp(t):
    """std::max(t, 0.0) (sampling.cc:395-396): -0.0 and NaN pass through."""
    return lib().orc_auto_clamp(t)


def mutate_recursively(seq, macrostates, pos, base):
    buf = C.create_string_buffer(_b(seq), len(seq) + 1)
    rc = lib().orc_mutate_recursively(buf, len(seq), _strarr(macrostates), len(macrostates), pos,
                                      _b(base))
    return rc, buf.value.decode()


def can_be_freely_mutated(seq, macrostates, pos):
    return bool(lib().orc_can_be_freely_mutated(_b(seq), len(seq), _strarr(macrostates),
                                                len(macrostates), pos))


class ScoreFunction:
    """terms: list of (condition 'apo'/'holo', target, favorable bool, weight) where
    target is a macrostate index (MacrostateProbTerm) or ("pair", i, j) (base-pair
    probability term, 0-based device positions)."""

    def __init__(self, terms, aptamer=None, contexts=None, params=None, mode="pf"):
        self.P = params or default_params()
        self._terms = (Term * max(1, len(terms)))()
        for k, (cond, mi, fav, w) in enumerate(terms):
            if isinstance(mi, tuple):
                self._terms[k] = Term(1 if cond == "holo" else 0, 0, 1 if fav else 0, w, 1, mi[1], mi[2])
            else:
                self._terms[k] = Term(1 if cond == "holo" else 0, mi, 1 if fav else 0, w, 0, 0, 0)
        self._apt = aptamer
        ctx = contexts or []
        self._ctx = (Context * max(1, len(ctx)))()
        self._ctx_keep = ctx
        for k, (b, a) in enumerate(ctx):
            self._ctx[k] = Context(_b(b), _b(a))
        self.s = ScoreFxn(self.P.ptr, len(terms), self._terms,
                          C.pointer(aptamer) if aptamer is not None else None, len(ctx), self._ctx,
                          {"pf": 0, "mfe": 1}[mode])

    def score(self, seq, macrostates):
        nt = self.s.n_terms * max(1, self.s.n_contexts)
        tv = (C.c_double * max(1, nt))()
        r = lib().orc_score(C.byref(self.s), _b(seq), len(seq), _strarr(macrostates),
                            len(macrostates), tv)
        return r, list(tv)[:nt]


def thermostat(kind="fixed", **kw):
    t = Thermostat()
    t.kind = {"fixed": 0, "annealing": 1, "auto": 2}[kind]
    t.t_fixed = kw.get("t", 1.0)
    t.t_hi = kw.get("t_hi", 1.0)
    t.t_lo = kw.get("t_lo", 0.0)
    t.cycle_len = kw.get("cycle_len", 1)
    t.target_rate = kw.get("rate", 0.5)
    t.period = kw.get("period", 100)
    t.t_init = kw.get("t0", 1.0)
    return t


def mc_run(scorefxn, seq, macrostates, therm, seed, num_steps, forced=None, tie_eps=0.0,
           want_seqs=False):
    n = len(seq)
    buf = C.create_string_buffer(_b(seq), n + 1)
    pos = (C.c_int * num_steps)()
    base = C.create_string_buffer(num_steps + 1)
    outc = (C.c_int * num_steps)()
    temp = (C.c_double * num_steps)()
    prop = (C.c_double * num_steps)()
    curs = (C.c_double * num_steps)()
    thr = (C.c_double * num_steps)()
    seqs = C.create_string_buffer(num_steps * n + 1) if want_seqs else None
    tr = Trace(pos, C.cast(base, C.c_char_p), outc, temp, prop, curs, thr,
               C.cast(seqs, C.c_char_p) if seqs is not None else None)
    opts = None
    if forced is not None:
        fo = (C.c_int * num_steps)(*forced)
        opts = McOpts(tie_eps, fo)
        opts._keep = fo
    fs = C.c_double(0)
    cnt = (C.c_int64 * 4)()
    rc = lib().orc_mc_run(C.byref(scorefxn.s), buf, n, _strarr(macrostates), len(macrostates),
                          C.byref(therm), seed, num_steps, C.byref(fs), cnt, C.byref(tr),
                          C.byref(opts) if opts is not None else None)
    out = dict(rc=rc, seq=buf.value.decode(), score=fs.value, counters=list(cnt),
               pos=list(pos), base=base.raw[:num_steps].decode(), outcome=list(outc),
               temperature=list(temp), proposed_score=list(prop), current_score=list(curs),
               random_threshold=list(thr))
    if want_seqs:
        raw = seqs.raw
        out["seqs"] = [raw[i * n:(i + 1) * n].decode() for i in range(num_steps)]
    return out


def mc_run_batch(scorefxn, seqs, macrostates, therm, seeds, num_steps, n_threads):
    n = len(seqs[0])
    W = len(seqs)
    buf = C.create_string_buffer(b"".join(_b(s) for s in seqs), n * W + 1)
    sd = (C.c_uint32 * W)(*seeds)
    cnt = (C.c_int64 * 4)()
    t = lib().orc_mc_run_batch(C.byref(scorefxn.s), buf, n, W, _strarr(macrostates),
                               len(macrostates), C.byref(therm), sd, num_steps, n_threads, cnt)
    return t, list(cnt)
