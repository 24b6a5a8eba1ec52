"""ctypes binding of the engine's C ABI (include/addapt_gpu.h).

This is the Python face of the product: it loads the in-tree
``addapt_amd/_lib/libaddapt_gpu.so`` (built by ``__graft_entry__.build()``)
and fails loudly when it is missing -- there is no CPU fallback.
"""
import ctypes as C
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ADX_LIB") or os.path.join(HERE, "_lib", "libaddapt_gpu.so")
DEFAULT_PARAMS = os.path.join(HERE, "data", "rna_turner2004_addapt.par")

ABI_VERSION = 4   # include/addapt_gpu.h ADX_ABI_VERSION (v4 renumbered the motif modes)
OK, EINVAL, EHIP, ECONSTRAINT, EPARAM, ENOMEM, EMOVE, ESTATE, ENODEV, EUNSUPPORTED = range(10)
APO, HOLO = 0, 1
THERMO_FIXED, THERMO_ANNEAL, THERMO_AUTO = 0, 1, 2
MOTIF_AUTO, MOTIF_ADD, MOTIF_REPLACE = 0, 1, 2   # include/addapt_gpu.h; AUTO is the default
FOLD_PF, FOLD_MFE = 0, 1
TERM_MACROSTATE, TERM_PAIR = 0, 1
OUTCOMES = ["REJECT", "ACCEPT_WORSENED", "ACCEPT_UNCHANGED", "ACCEPT_IMPROVED"]


class AdxError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("adx status %d: %s" % (status, msg))
        self.status = status


class Term(C.Structure):
    _fields_ = [("condition", C.c_int), ("macrostate", C.c_int), ("favorable", C.c_int),
                ("weight", C.c_double), ("kind", C.c_int), ("pair_i", C.c_int), ("pair_j", C.c_int)]


class Thermostat(C.Structure):
    _fields_ = [("kind", C.c_int), ("t_fixed", C.c_double), ("t_hi", C.c_double),
                ("t_lo", C.c_double), ("cycle_len", C.c_int), ("target_rate", C.c_double),
                ("period", C.c_int), ("t_init", C.c_double)]


class ContextDesc(C.Structure):
    _fields_ = [("before", C.c_char_p), ("after", C.c_char_p)]


class RunDesc(C.Structure):
    _fields_ = [("params", C.c_void_p), ("sequence", C.c_char_p), ("n_macrostates", C.c_int),
                ("macrostates", C.POINTER(C.c_char_p)), ("n_terms", C.c_int),
                ("terms", C.POINTER(Term)), ("aptamer_seq", C.c_char_p),
                ("aptamer_fold", C.c_char_p), ("aptamer_energy_kcal", C.c_double),
                ("motif_mode", C.c_int), ("n_contexts", C.c_int),
                ("contexts", C.POINTER(ContextDesc)), ("thermostat", Thermostat),
                ("device", C.c_int), ("fold_mode", C.c_int)]


class Info(C.Structure):
    _fields_ = [("length", C.c_int), ("n_variants", C.c_int), ("n_terms", C.c_int),
                ("n_mutable", C.c_int), ("max_walkers", C.c_int), ("scale_per_nt", C.c_double)]


class Trace(C.Structure):
    _fields_ = [("position", C.POINTER(C.c_int32)), ("base", C.c_char_p),
                ("outcome", C.POINTER(C.c_int32)), ("temperature", C.POINTER(C.c_double)),
                ("proposed_score", C.POINTER(C.c_double)), ("current_score", C.POINTER(C.c_double)),
                ("random_threshold", C.POINTER(C.c_double)), ("term_values", C.POINTER(C.c_double))]


# Every symbol include/addapt_gpu.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "adx_last_error", "adx_abi_version", "adx_params_load", "adx_params_free", "adx_kT",
    "adx_eval_structure", "adx_fold_create", "adx_fold_add_motif", "adx_fold_add_constraint",
    "adx_fold_pf", "adx_fold_mfe", "adx_fold_bpp", "adx_fold_free", "adx_ctx_create", "adx_ctx_destroy",
    "adx_ctx_info", "adx_walkers_init", "adx_run_steps", "adx_last_kernel_ms", "adx_last_score_kernel_ms",
    "adx_last_kernel_split_ms",
    "adx_last_kernel_names",
    "adx_walkers_download", "adx_score_batch", "adx_variant_desc", "adx_walkers_export",
    "adx_walkers_import", "adx_walkers_import_after", "adx_walkers_export_on", "adx_set_temperature", "adx_bppm_batch",
    "adx_walkers_rescore",
]

_lib = None


def lib():
    """Load the HIP engine; raise if it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("addapt_amd native engine not built: %s missing "
                              "(run __graft_entry__.build())" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        # a stale build (or an ADX_LIB ablation library) of another ABI would
        # silently swap enum meanings (v4: motif AUTO = 0, ADD = 1, REPLACE = 2)
        got = L.adx_abi_version()
        if got != ABI_VERSION:
            raise ImportError("%s has ABI version %d, this binding needs %d (rebuild: "
                              "__graft_entry__.build())" % (LIB_PATH, got, ABI_VERSION))
        L.adx_last_error.restype = C.c_char_p
        L.adx_kT.restype = C.c_double
        L.adx_params_load.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        L.adx_params_free.argtypes = [C.c_void_p]
        L.adx_eval_structure.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.POINTER(C.c_double)]
        L.adx_fold_create.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_void_p)]
        L.adx_fold_add_motif.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_double]
        L.adx_fold_add_constraint.argtypes = [C.c_void_p, C.c_char_p]
        L.adx_fold_pf.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
        L.adx_fold_mfe.argtypes = [C.c_void_p, C.POINTER(C.c_float)]
        L.adx_fold_bpp.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double)]
        L.adx_fold_free.argtypes = [C.c_void_p]
        L.adx_ctx_create.argtypes = [C.POINTER(RunDesc), C.POINTER(C.c_void_p)]
        L.adx_ctx_destroy.argtypes = [C.c_void_p]
        L.adx_ctx_info.argtypes = [C.c_void_p, C.POINTER(Info)]
        L.adx_walkers_init.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.POINTER(C.c_uint32)]
        L.adx_run_steps.argtypes = [C.c_void_p, C.c_int, C.POINTER(Trace)]
        L.adx_last_kernel_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        L.adx_last_score_kernel_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int)]
        L.adx_last_kernel_split_ms.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.adx_last_kernel_names.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.c_char_p, C.c_int]
        L.adx_walkers_export.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.adx_walkers_import.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.adx_walkers_import_after.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.adx_walkers_export_on.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.adx_set_temperature.argtypes = [C.c_void_p, C.c_double]
        L.adx_walkers_download.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_double),
                                           C.POINTER(C.c_int64)]
        L.adx_score_batch.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.POINTER(C.c_double),
                                      C.POINTER(C.c_double), C.POINTER(C.c_float)]
        L.adx_walkers_rescore.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.adx_bppm_batch.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_int, C.c_int,
                                     C.POINTER(C.c_double)]
        L.adx_variant_desc.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int),
                                       C.POINTER(C.c_int), C.POINTER(C.c_int)]
        _lib = L
    return _lib


def _check(status):
    if status != OK:
        raise AdxError(status, lib().adx_last_error().decode())


def _b(s):
    return s.encode() if isinstance(s, str) else s


def kT():
    return lib().adx_kT()


def theo_energy(kd_uM=0.32):
    """kT * ln(Kd / 1 M) -- the bonus scoring.cc:91-99 passes to vrna_sc_add_hi_motif."""
    return kT() * math.log(kd_uM / 1e6)


class Params:
    def __init__(self, path=DEFAULT_PARAMS):
        self.ptr = C.c_void_p()
        _check(lib().adx_params_load(_b(path), C.byref(self.ptr)))

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.adx_params_free(self.ptr)
            self.ptr = None

    def eval_structure(self, seq, structure):
        e = C.c_double()
        _check(lib().adx_eval_structure(self.ptr, _b(seq), _b(structure), C.byref(e)))
        return e.value


_params = None


def default_params():
    global _params
    if _params is None:
        _params = Params()
    return _params


class Fold:
    """Per-fold layer: the six ViennaRNA calls of scoring.cc, one-to-one."""

    def __init__(self, seq, with_bppm=False, params=None, device=0):
        self.params = params or default_params()
        self.ptr = C.c_void_p()
        _check(lib().adx_fold_create(self.params.ptr, _b(seq), int(with_bppm), device,
                                     C.byref(self.ptr)))

    def add_motif(self, seq, fold, energy):
        _check(lib().adx_fold_add_motif(self.ptr, _b(seq), _b(fold), energy))

    def add_constraint(self, db):
        _check(lib().adx_fold_add_constraint(self.ptr, _b(db)))

    def pf(self):
        g = C.c_float()
        _check(lib().adx_fold_pf(self.ptr, C.byref(g)))
        return g.value

    def mfe(self):
        g = C.c_float()
        _check(lib().adx_fold_mfe(self.ptr, C.byref(g)))
        return g.value

    def bpp(self, i, j):
        p = C.c_double()
        _check(lib().adx_fold_bpp(self.ptr, i, j, C.byref(p)))
        return p.value

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.adx_fold_free(self.ptr)
            self.ptr = None


def make_thermostat(kind="fixed", t=1.0, t_hi=1.0, t_lo=0.0, cycle_len=1, rate=0.5, period=100,
                    t0=1.0):
    th = Thermostat()
    th.kind = {"fixed": THERMO_FIXED, "annealing": THERMO_ANNEAL, "auto": THERMO_AUTO}[kind]
    th.t_fixed, th.t_hi, th.t_lo, th.cycle_len = t, t_hi, t_lo, cycle_len
    th.target_rate, th.period, th.t_init = rate, period, t0
    return th


class Engine:
    """Batched Monte Carlo context (adx_ctx_*).

    terms: list of (condition 'apo'|'holo', target, favorable bool, weight); target is a
    macrostate index (MacrostateProbTerm) or ("pair", i, j) (base-pair probability term,
    0-based device positions)
    aptamer: None or (seq, fold, energy_kcal); contexts: list of (before, after).
    fold_mode: "pf" (ensembles, vrna_pf) or "mfe" (minimum free energies, ADX_FOLD_MFE).
    """

    def __init__(self, sequence, macrostates, terms, aptamer=None, thermostat=None, contexts=None,
                 motif_mode=MOTIF_AUTO, params=None, device=0, fold_mode="pf"):
        self.params = params or default_params()
        self.N = len(sequence)
        d = RunDesc()
        d.params = self.params.ptr
        d.sequence = _b(sequence)
        self._ms = (C.c_char_p * max(1, len(macrostates)))(*[_b(m) for m in macrostates])
        d.n_macrostates = len(macrostates)
        d.macrostates = self._ms
        self._terms = (Term * max(1, len(terms)))()
        for k, (cond, mi, fav, w) in enumerate(terms):
            c = HOLO if cond in ("holo", HOLO) else APO
            if isinstance(mi, tuple):
                self._terms[k] = Term(c, 0, int(bool(fav)), w, TERM_PAIR, mi[1], mi[2])
            else:
                self._terms[k] = Term(c, mi, int(bool(fav)), w, TERM_MACROSTATE, 0, 0)
        d.n_terms = len(terms)
        d.terms = self._terms
        if aptamer is not None:
            d.aptamer_seq, d.aptamer_fold, d.aptamer_energy_kcal = _b(aptamer[0]), _b(aptamer[1]), aptamer[2]
        d.motif_mode = motif_mode
        ctx = contexts or []
        self._ctx = (ContextDesc * max(1, len(ctx)))()
        for k, (b, a) in enumerate(ctx):
            self._ctx[k] = ContextDesc(_b(b), _b(a))
        d.n_contexts = len(ctx)
        d.contexts = self._ctx
        self._ctx_lens = [(len(b), len(a)) for b, a in ctx]
        d.thermostat = thermostat if thermostat is not None else make_thermostat()
        d.device = device
        d.fold_mode = {"pf": FOLD_PF, "mfe": FOLD_MFE}[fold_mode]
        self.fold_mode = fold_mode
        self._desc = d
        self.ptr = C.c_void_p()
        _check(lib().adx_ctx_create(C.byref(d), C.byref(self.ptr)))
        self.info = Info()
        _check(lib().adx_ctx_info(self.ptr, C.byref(self.info)))
        self.n_terms_total = len(terms) * max(1, len(ctx))
        self.W = 0

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.adx_ctx_destroy(self.ptr)
            self.ptr = None

    def variant(self, v):
        c, cond, m = C.c_int(), C.c_int(), C.c_int()
        _check(lib().adx_variant_desc(self.ptr, v, C.byref(c), C.byref(cond), C.byref(m)))
        return c.value, cond.value, m.value

    def score_batch(self, seqs):
        W = len(seqs)
        buf = b"".join(_b(s) for s in seqs)
        sc = np.zeros(W, np.float64)
        tv = np.zeros(W * max(1, self.n_terms_total), np.float64)
        dg = np.zeros(W * self.info.n_variants, np.float32)
        _check(lib().adx_score_batch(self.ptr, W, buf, sc.ctypes.data_as(C.POINTER(C.c_double)),
                                     tv.ctypes.data_as(C.POINTER(C.c_double)),
                                     dg.ctypes.data_as(C.POINTER(C.c_float))))
        return sc, tv.reshape(W, -1)[:, :self.n_terms_total], dg.reshape(W, -1)

    def bppm_batch(self, seqs, condition="apo", context=0):
        """(W, L, L) base-pair probability matrices of the (context, condition) fold."""
        W = len(seqs)
        buf = b"".join(_b(s) for s in seqs)
        c = HOLO if condition in ("holo", HOLO) else APO
        L = self.N
        if self._ctx_lens:
            L += sum(self._ctx_lens[context])
        out = np.zeros(W * L * L, np.float64)
        _check(lib().adx_bppm_batch(self.ptr, W, buf, c, context,
                                    out.ctypes.data_as(C.POINTER(C.c_double))))
        return out.reshape(W, L, L)

    def walkers_init(self, seeds, seqs=None):
        W = len(seeds)
        sd = (C.c_uint32 * W)(*seeds)
        buf = b"".join(_b(s) for s in seqs) if seqs is not None else None
        _check(lib().adx_walkers_init(self.ptr, W, buf, sd))
        self.W = W

    def run_steps(self, steps, trace=False):
        tr = None
        out = None
        if trace:
            R = steps * self.W
            out = dict(position=np.zeros(R, np.int32), outcome=np.zeros(R, np.int32),
                       temperature=np.zeros(R), proposed_score=np.zeros(R), current_score=np.zeros(R),
                       random_threshold=np.zeros(R), term_values=np.zeros(R * max(1, self.n_terms_total)))
            base = C.create_string_buffer(R + 1)
            tr = Trace(out["position"].ctypes.data_as(C.POINTER(C.c_int32)), C.cast(base, C.c_char_p),
                       out["outcome"].ctypes.data_as(C.POINTER(C.c_int32)),
                       out["temperature"].ctypes.data_as(C.POINTER(C.c_double)),
                       out["proposed_score"].ctypes.data_as(C.POINTER(C.c_double)),
                       out["current_score"].ctypes.data_as(C.POINTER(C.c_double)),
                       out["random_threshold"].ctypes.data_as(C.POINTER(C.c_double)),
                       out["term_values"].ctypes.data_as(C.POINTER(C.c_double)))
        _check(lib().adx_run_steps(self.ptr, steps, C.byref(tr) if tr is not None else None))
        if trace:
            out["base"] = base.raw[:steps * self.W].decode()
            for k in ("position", "outcome", "temperature", "proposed_score", "current_score",
                      "random_threshold"):
                out[k] = out[k].reshape(steps, self.W)
            out["term_values"] = out["term_values"].reshape(steps, self.W, -1)[:, :, :self.n_terms_total]
        return out

    def last_kernel_ms(self):
        ms = C.c_double()
        _check(lib().adx_last_kernel_ms(self.ptr, C.byref(ms)))
        return ms.value

    def export_walkers(self, dev_seqs_ptr, dev_scores_ptr, on_stream=None):
        """Device-to-device copy of the walkers' sequence codes (W*N uint8) and
        scores (W float64) into caller-owned device buffers (raw pointers).
        `on_stream` (a raw HIP stream handle, e.g.
        torch.cuda.current_stream().cuda_stream -- 0 is the null stream) orders
        the copy between that stream's earlier and later work without a host
        synchronisation; None: synchronous."""
        if on_stream is None:
            _check(lib().adx_walkers_export(self.ptr, C.c_void_p(dev_seqs_ptr), C.c_void_p(dev_scores_ptr)))
        else:
            _check(lib().adx_walkers_export_on(self.ptr, C.c_void_p(dev_seqs_ptr), C.c_void_p(dev_scores_ptr),
                                               C.c_void_p(int(on_stream))))

    def import_walkers(self, dev_seqs_ptr, dev_scores_ptr, after_stream=None):
        """Copy configurations back in; `after_stream` (a raw HIP stream handle;
        0 is the null stream, not "none") orders the copy after the work queued
        there, and that stream's later work after the copy, without a host
        synchronisation; None: the synchronous import."""
        if after_stream is None:
            _check(lib().adx_walkers_import(self.ptr, C.c_void_p(dev_seqs_ptr), C.c_void_p(dev_scores_ptr)))
        else:
            _check(lib().adx_walkers_import_after(self.ptr, C.c_void_p(dev_seqs_ptr),
                                                  C.c_void_p(dev_scores_ptr), C.c_void_p(int(after_stream))))

    def set_temperature(self, t):
        _check(lib().adx_set_temperature(self.ptr, float(t)))

    def last_score_kernel_ms(self):
        """(average score-kernel launch ms, launches) of the last run_steps."""
        ms, n = C.c_double(), C.c_int()
        _check(lib().adx_last_score_kernel_ms(self.ptr, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def last_kernel_split_ms(self):
        """(average inside-fold ms, average outside-pass ms) per step of the last run_steps."""
        a, b = C.c_double(), C.c_double()
        _check(lib().adx_last_kernel_split_ms(self.ptr, C.byref(a), C.byref(b)))
        return a.value, b.value

    def last_kernel_names(self):
        """(fold kernel(s), outside pass or "") the last run_steps launched."""
        a, b = C.create_string_buffer(256), C.create_string_buffer(256)
        _check(lib().adx_last_kernel_names(self.ptr, a, 256, b, 256))
        return a.value.decode(), b.value.decode()

    def rescore(self):
        """(scores, term values) of every walker's current configuration folded
        from scratch by the MC step's own kernels (adx_walkers_rescore); the
        stored scores are not touched."""
        W = self.W
        sc = np.zeros(W, np.float64)
        tv = np.zeros(W * max(1, self.n_terms_total), np.float64)
        _check(lib().adx_walkers_rescore(self.ptr, sc.ctypes.data_as(C.POINTER(C.c_double)),
                                         tv.ctypes.data_as(C.POINTER(C.c_double))))
        return sc, tv.reshape(W, -1)[:, :self.n_terms_total]

    def download(self):
        W = self.W
        buf = C.create_string_buffer(W * self.N + 1)
        sc = np.zeros(W, np.float64)
        cnt = np.zeros(W * 4, np.int64)
        _check(lib().adx_walkers_download(self.ptr, buf, sc.ctypes.data_as(C.POINTER(C.c_double)),
                                          cnt.ctypes.data_as(C.POINTER(C.c_int64))))
        raw = buf.raw[:W * self.N].decode()
        seqs = [raw[w * self.N:(w + 1) * self.N] for w in range(W)]
        return seqs, sc, cnt.reshape(W, 4)
