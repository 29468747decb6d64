"""ctypes wrapper for the CPU restatement in oracle/arrow_oracle.cpp -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only
as the checker.  The product (pbccs_amd) never imports it.  Parity pin: see arrow_oracle.cpp's header.
"""
import ctypes
import math
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

INSERTION, DELETION, SUBSTITUTION = 0, 1, 2
FORWARD, REVERSE = 0, 1

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c_d, c_i, c_p, c_s = ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p
        D = ctypes.POINTER(ctypes.c_double)
        I = ctypes.POINTER(ctypes.c_int)
        Lg = ctypes.POINTER(ctypes.c_long)
        L.orc_scorer_new.restype = c_p
        L.orc_scorer_new.argtypes = [c_s, D, c_d, c_d, c_d]
        L.orc_scorer_free.argtypes = [c_p]
        L.orc_scorer_add_read.argtypes = [c_p, c_s, c_i, c_i, c_i, c_d]
        L.orc_scorer_num_reads.argtypes = [c_p]
        L.orc_scorer_read_info.argtypes = [c_p, c_i, I, I, I, D, I]
        L.orc_scorer_band_stats.argtypes = [c_p, c_i, ctypes.POINTER(ctypes.c_longlong),
                                            ctypes.POINTER(ctypes.c_longlong), I, I]
        L.orc_scorer_score.restype = c_d
        L.orc_scorer_score.argtypes = [c_p, c_i, c_i, c_i, c_s, c_d]
        L.orc_scorer_scores.argtypes = [c_p, c_i, c_i, c_i, c_s, c_d, D]
        L.orc_scorer_baseline.restype = c_d
        L.orc_scorer_baseline.argtypes = [c_p]
        L.orc_scorer_template.argtypes = [c_p, c_i, ctypes.c_char_p, c_i]
        L.orc_scorer_apply.argtypes = [c_p, c_i, I, I, I, c_s]
        L.orc_scorer_zscores.argtypes = [c_p, D, D, D]
        L.orc_refine.argtypes = [c_p, c_i, c_i, c_i, Lg, Lg, I, c_i, I]
        L.orc_qvs.argtypes = [c_p, I, c_i]
        L.orc_enum_unique.argtypes = [c_s, c_i, c_i, I, I, c_s, c_i]
        L.orc_enum_nearby.argtypes = [c_s, c_i, I, c_i, I, I, c_s, c_i]
        L.orc_apply_mutations.argtypes = [c_s, c_i, I, I, I, c_s, c_s, c_i, I, c_i]
        L.orc_context_params.argtypes = [D, D]
        L.orc_poa_consensus.argtypes = [ctypes.POINTER(c_s), c_i, c_i, c_i, c_s, c_i, c_s, c_i, c_i]
        L.orc_sparse_poa.argtypes = [ctypes.POINTER(c_s), c_i, c_i, ctypes.c_long, I, I, I, I, c_s, c_i]
        L.orc_poa_kat_reads.restype = ctypes.c_long
        L.orc_poa_kat_reads.argtypes = [c_i, c_s, ctypes.c_long, I]
        _lib = L
    return _lib


def _darr(vals):
    return (ctypes.c_double * len(vals))(*vals)


def _iarr(vals):
    return (ctypes.c_int * len(vals))(*vals)


def mutation_end(mtype, start):
    return start if mtype == INSERTION else start + 1


class Scorer:
    """Mirror of ConsensusCore::Arrow::MultiReadMutationScorer (CPU restatement)."""

    def __init__(self, tpl, snr, score_diff=12.5, fast_threshold=-12.5, add_threshold=float("nan")):
        self._h = lib().orc_scorer_new(tpl.encode(), _darr(snr), score_diff, fast_threshold, add_threshold)
        if not self._h:
            raise ValueError("invalid template")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_scorer_free(self._h)
            self._h = None

    def add_read(self, seq, strand=FORWARD, ts=0, te=None, threshold=float("nan")):
        if te is None:
            te = len(self.template())
        return lib().orc_scorer_add_read(self._h, seq.encode(), strand, ts, te, threshold)

    def num_reads(self):
        return lib().orc_scorer_num_reads(self._h)

    def read_info(self, r):
        a, ts, te, fl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        ll = ctypes.c_double()
        lib().orc_scorer_read_info(self._h, r, ctypes.byref(a), ctypes.byref(ts), ctypes.byref(te),
                                   ctypes.byref(ll), ctypes.byref(fl))
        return {"active": bool(a.value), "ts": ts.value, "te": te.value, "ll": ll.value, "flipflops": fl.value}

    def band_stats(self, r):
        """Diagnostics: (alpha used cells, beta used cells, tallest alpha column, tallest beta column)."""
        au, bu, ah, bh = ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_int(), ctypes.c_int()
        lib().orc_scorer_band_stats(self._h, r, ctypes.byref(au), ctypes.byref(bu), ctypes.byref(ah), ctypes.byref(bh))
        return au.value, bu.value, ah.value, bh.value

    def pass_log(self, r):
        """Diagnostics: read r's last FillAlphaBeta, per pass (alpha?, used cells, tallest column, first column
        taller than 64 rows or -1, used cells before it)."""
        buf = (ctypes.c_longlong * (5 * 16))()
        f = lib().orc_scorer_pass_log
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_longlong), ctypes.c_int]
        n = f(self._h, r, buf, 16)
        return [tuple(buf[5 * k:5 * k + 5]) for k in range(max(0, min(n, 16)))]

    def score(self, mtype, start, base="-", fast_threshold=-1.7976931348623157e308):
        nb = b"" if mtype == DELETION else base.encode()
        return lib().orc_scorer_score(self._h, mtype, start, mutation_end(mtype, start), nb, fast_threshold)

    def scores(self, mtype, start, base="-", unscored=0.0):
        out = (ctypes.c_double * max(1, self.num_reads()))()
        nb = b"" if mtype == DELETION else base.encode()
        n = lib().orc_scorer_scores(self._h, mtype, start, mutation_end(mtype, start), nb, unscored, out)
        return list(out[:n])

    def baseline(self):
        return lib().orc_scorer_baseline(self._h)

    def template(self, strand=FORWARD):
        buf = ctypes.create_string_buffer(1 << 20)
        n = lib().orc_scorer_template(self._h, strand, buf, len(buf))
        return buf.value.decode()

    def apply(self, muts):
        types = _iarr([m[0] for m in muts])
        starts = _iarr([m[1] for m in muts])
        ends = _iarr([mutation_end(m[0], m[1]) for m in muts])
        bases = "".join(m[2] if m[0] != DELETION else "-" for m in muts).encode()
        return lib().orc_scorer_apply(self._h, len(muts), types, starts, ends, bases)

    def zscores(self):
        zg, za = ctypes.c_double(), ctypes.c_double()
        zs = (ctypes.c_double * max(1, self.num_reads()))()
        lib().orc_scorer_zscores(self._h, ctypes.byref(zg), ctypes.byref(za), zs)
        return zg.value, za.value, list(zs[: self.num_reads()])

    def refine(self, max_iter=40, separation=10, neighborhood=20):
        nt, na = ctypes.c_long(), ctypes.c_long()
        cap = 100000
        log = (ctypes.c_int * (4 * cap))()
        nlog = ctypes.c_int()
        conv = lib().orc_refine(self._h, max_iter, separation, neighborhood, ctypes.byref(nt), ctypes.byref(na),
                                log, cap, ctypes.byref(nlog))
        applied = [(log[4 * k], log[4 * k + 1], log[4 * k + 2], chr(log[4 * k + 3])) for k in range(min(cap, nlog.value))]
        return {"converged": conv == 1, "error": conv < 0, "n_tested": nt.value, "n_applied": na.value,
                "applied": applied}

    def alignment(self, r):
        """RecursorBase::Alignment of read r (Viterbi): (target, query); None for a sum-product scorer."""
        cap = 1 << 20
        t = ctypes.create_string_buffer(cap)
        q = ctypes.create_string_buffer(cap)
        n = _qlib().qorc_scorer_alignment(self._h, r, t, q, cap)
        if n == -1:
            return None
        assert n >= 0
        return t.value.decode(), q.value.decode()

    def qvs(self):
        L = len(self.template())
        out = (ctypes.c_int * max(1, L))()
        n = lib().orc_qvs(self._h, out, L)
        if n < 0:
            raise RuntimeError("qv failure")
        return list(out[:n])


def unique_mutations(tpl, b=0, e=None):
    if e is None:
        e = len(tpl)
    cap = 8 * len(tpl) + 8
    t, s = (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
    bs = ctypes.create_string_buffer(cap)
    n = lib().orc_enum_unique(tpl.encode(), b, e, t, s, bs, cap)
    return [(t[k], s[k], bs.raw[k:k + 1].decode()) for k in range(n)]


def nearby_mutations(tpl, centers, nbhd):
    cap = 8 * len(tpl) + 8
    t, s = (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
    bs = ctypes.create_string_buffer(cap)
    n = lib().orc_enum_nearby(tpl.encode(), len(centers), _iarr(centers), nbhd, t, s, bs, cap)
    return [(t[k], s[k], bs.raw[k:k + 1].decode()) for k in range(n)]


def apply_mutations(tpl, muts):
    types = _iarr([m[0] for m in muts])
    starts = _iarr([m[1] for m in muts])
    ends = _iarr([mutation_end(m[0], m[1]) for m in muts])
    bases = "".join(m[2] if m[0] != DELETION else "-" for m in muts).encode()
    cap = len(tpl) + len(muts) + 2
    out = ctypes.create_string_buffer(cap)
    mtp = (ctypes.c_int * (len(tpl) + 1))()
    n = lib().orc_apply_mutations(tpl.encode(), len(muts), types, starts, ends, bases, out, cap, mtp, len(tpl) + 1)
    if n < 0:
        raise RuntimeError("apply failed")
    return out.value.decode(), list(mtp)


def context_params(snr):
    out = (ctypes.c_double * 32)()
    lib().orc_context_params(_darr(snr), out)
    return [list(out[4 * c: 4 * c + 4]) for c in range(8)]


def polish_zmw(draft, reads, snr, min_zscore=-5.0, max_iter=40, separation=10, neighborhood=20, qvs=True):
    """The ccs per-ZMW polish step after the POA (include/pacbio/ccs/Consensus.h:436-512), restated.

    reads: list of dicts {seq, strand, ts, te}.  Returns the same fields the reference result carries.
    """
    s = Scorer(draft, snr)
    status = [s.add_read(r["seq"], r["strand"], r["ts"], r["te"], min_zscore) for r in reads]
    zg, za, zs = s.zscores()
    ref = s.refine(max_iter, separation, neighborhood)
    out = {"add_read_results": status, "zg": zg, "za": za, "zscores": zs, "baseline_lls": [],
           "converged": ref["converged"], "n_tested": ref["n_tested"], "n_applied": ref["n_applied"],
           "applied": ref["applied"], "template": s.template()}
    out["baseline_lls"] = [s.read_info(r)["ll"] for r in range(s.num_reads())]
    if qvs and ref["converged"]:
        q = s.qvs()
        out["qvs"] = q
        out["pred_acc"] = 1.0 - sum(10.0 ** (v / -10.0) for v in q) / max(1, len(q))
    return out


# ================================================================ Quiver family (oracle/quiver_oracle.cpp)
QV_PARAM_NAMES = ("Match", "Mismatch", "MismatchS", "Branch", "BranchS", "DeletionN", "DeletionWithTag",
                  "DeletionWithTagS", "Nce", "NceS")
INCORPORATE, EXTRA, DELETE, MERGE = 1, 2, 4, 8
BASIC_MOVES, ALL_MOVES = 7, 15


def _qlib():
    L = lib()
    if not getattr(L, "_q_ready", False):
        c_f, c_i, c_p, c_s = ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p
        F = ctypes.POINTER(ctypes.c_float)
        I = ctypes.POINTER(ctypes.c_int)
        LL = ctypes.POINTER(ctypes.c_longlong)
        Lg = ctypes.POINTER(ctypes.c_long)
        for n in ("qorc_log_add",):
            getattr(L, n).restype = c_f
            getattr(L, n).argtypes = [c_f, c_f]
        for n in ("qorc_exp_ps", "qorc_log_ps"):
            getattr(L, n).restype = c_f
            getattr(L, n).argtypes = [c_f]
        L.qorc_scorer_new.restype = c_p
        L.qorc_scorer_new.argtypes = [c_s, F, c_i, c_f, c_f, c_f, c_i]
        L.qorc_scorer_free.argtypes = [c_p]
        L.qorc_scorer_add_read.argtypes = [c_p, c_s, F, F, F, F, F, c_i, c_i, c_i, c_f, c_i]
        L.qorc_scorer_score.restype = c_f
        L.qorc_scorer_score.argtypes = [c_p, c_i, c_i, c_i, c_s, c_i]
        L.qorc_ms_score.restype = c_f
        L.qorc_ms_score.argtypes = [c_p, c_i, c_i, c_i, c_i, c_s]
        L.qorc_scorer_scores.argtypes = [c_p, c_i, c_i, c_i, c_s, c_f, F]
        L.qorc_scorer_is_favorable.argtypes = [c_p, c_i, c_i, c_i, c_s, c_i]
        L.qorc_scorer_baseline.restype = c_f
        L.qorc_scorer_baseline.argtypes = [c_p]
        L.qorc_scorer_num_reads.argtypes = [c_p]
        L.qorc_scorer_read_info.argtypes = [c_p, c_i, I, I, I, F, I, LL, LL, LL, LL]
        L.qorc_scorer_cell.restype = c_f
        L.qorc_scorer_cell.argtypes = [c_p, c_i, c_i, c_i, c_i]
        L.qorc_scorer_template.argtypes = [c_p, c_s, c_i]
        L.qorc_scorer_apply.argtypes = [c_p, c_i, I, I, I, c_s]
        L.qorc_refine.argtypes = [c_p, c_i, c_i, c_i, Lg, Lg]
        L.qorc_qvs.argtypes = [c_p, I, c_i]
        L.qorc_scorer_alignment.argtypes = [c_p, c_i, c_s, c_s, c_i]
        L._q_ready = True
    return L


def _farr(vals):
    return (ctypes.c_float * len(vals))(*vals)


def qv_params(d):
    """QvModelParams as the 20 floats of the C ABI (dict keys as in QuiverConfig.hpp:79-92; Merge/MergeS
    may be scalars or 4-lists)."""
    out = [float(d[k]) for k in QV_PARAM_NAMES]
    for k in ("Merge", "MergeS"):
        v = d[k]
        out += [float(x) for x in v] if isinstance(v, (list, tuple)) else [float(v)] * 4
    return out


QUIVER_RECURSORS = ("SparseSse", "SparseSimple", "DenseSse", "DenseSimple")


class QuiverScorer:
    """Mirror of ConsensusCore::MultiReadMutationScorer<R> (CPU restatement).  recursor: SparseSse (the MRMS
    typedefs' SparseSseQvRecursor), SparseSimple, DenseSse (SseQvRecursor), DenseSimple (SimpleQvRecursor) --
    the four recursor types ConsensusCore's typed tests run (MutationScorer.hpp:93-99)."""

    def __init__(self, tpl, params, moves=ALL_MOVES, score_diff=12.5, fast_threshold=-12.5, add_threshold=1.0,
                 sum_product=False, recursor="SparseSse"):
        k = QUIVER_RECURSORS.index(recursor)
        flags = (1 if sum_product else 0) | (2 if k in (1, 3) else 0) | (4 if k >= 2 else 0)
        self._h = _qlib().qorc_scorer_new(tpl.encode(), _farr(qv_params(params)), moves, score_diff, fast_threshold,
                                          add_threshold, flags)

    def __del__(self):
        if getattr(self, "_h", None):
            _qlib().qorc_scorer_free(self._h)
            self._h = None

    def add_read(self, seq, strand=FORWARD, ts=0, te=None, features=None, threshold=None):
        """features: dict with optional ins/subs/del/del_tag/merge lists (del_tag as characters)."""
        if te is None:
            te = len(self.template())
        f = features or {}
        arrs = []
        for k in ("ins", "subs", "del", "del_tag", "merge"):
            v = f.get(k)
            if v is None:
                arrs.append(None)
            elif k == "del_tag":
                arrs.append(_farr([float(ord(c)) if isinstance(c, str) else float(c) for c in v]))
            else:
                arrs.append(_farr([float(x) for x in v]))
        use_cfg = 1 if threshold is None else 0
        return _qlib().qorc_scorer_add_read(self._h, seq.encode(), *arrs, strand, ts, te,
                                             0.0 if threshold is None else threshold, use_cfg)

    def score(self, mtype, start, base="-", fast=False, end=None):
        nb = b"" if mtype == DELETION else base.encode()
        return _qlib().qorc_scorer_score(self._h, mtype, start, end if end is not None else mutation_end(mtype, start),
                                         nb, 1 if fast else 0)

    def read_score_mutation(self, r, mtype, start, base="-"):
        nb = b"" if mtype == DELETION else base.encode()
        return _qlib().qorc_ms_score(self._h, r, mtype, start, mutation_end(mtype, start), nb)

    def scores(self, mtype, start, base="-", unscored=0.0):
        out = (ctypes.c_float * max(1, self.num_reads()))()
        nb = b"" if mtype == DELETION else base.encode()
        n = _qlib().qorc_scorer_scores(self._h, mtype, start, mutation_end(mtype, start), nb, unscored, out)
        return list(out[:n])

    def is_favorable(self, mtype, start, base="-", fast=False):
        nb = b"" if mtype == DELETION else base.encode()
        return bool(_qlib().qorc_scorer_is_favorable(self._h, mtype, start, mutation_end(mtype, start), nb,
                                                      1 if fast else 0))

    def baseline(self):
        return _qlib().qorc_scorer_baseline(self._h)

    def num_reads(self):
        return _qlib().qorc_scorer_num_reads(self._h)

    def read_info(self, r):
        a, ts, te, fl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        sc = ctypes.c_float()
        ua, ub, aa, ab = ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_longlong()
        _qlib().qorc_scorer_read_info(self._h, r, ctypes.byref(a), ctypes.byref(ts), ctypes.byref(te), ctypes.byref(sc),
                                      ctypes.byref(fl), ctypes.byref(ua), ctypes.byref(ub), ctypes.byref(aa),
                                      ctypes.byref(ab))
        return {"active": bool(a.value), "ts": ts.value, "te": te.value, "score": sc.value, "flipflops": fl.value,
                "used": (ua.value, ub.value), "allocated": (aa.value, ab.value)}

    def cell(self, r, which, i, j):
        return _qlib().qorc_scorer_cell(self._h, r, which, i, j)

    def template(self):
        buf = ctypes.create_string_buffer(1 << 20)
        _qlib().qorc_scorer_template(self._h, buf, len(buf))
        return buf.value.decode()

    def apply(self, muts):
        types = _iarr([m[0] for m in muts])
        starts = _iarr([m[1] for m in muts])
        ends = _iarr([mutation_end(m[0], m[1]) for m in muts])
        bases = "".join(m[2] if m[0] != DELETION else "-" for m in muts).encode()
        return _qlib().qorc_scorer_apply(self._h, len(muts), types, starts, ends, bases)

    def refine(self, max_iter=40, separation=10, neighborhood=20):
        nt, na = ctypes.c_long(), ctypes.c_long()
        conv = _qlib().qorc_refine(self._h, max_iter, separation, neighborhood, ctypes.byref(nt), ctypes.byref(na))
        return {"converged": conv == 1, "error": conv < 0, "n_tested": nt.value, "n_applied": na.value}

    def alignment(self, r):
        """RecursorBase::Alignment of read r (Viterbi): (target, query); None for a sum-product scorer."""
        cap = 1 << 20
        t = ctypes.create_string_buffer(cap)
        q = ctypes.create_string_buffer(cap)
        n = _qlib().qorc_scorer_alignment(self._h, r, t, q, cap)
        if n == -1:
            return None
        assert n >= 0
        return t.value.decode(), q.value.decode()

    def qvs(self):
        L = len(self.template())
        out = (ctypes.c_int * max(1, L))()
        n = _qlib().qorc_qvs(self._h, out, L)
        return list(out[:n])


def qv_eval_moves(seq, tpl, params, cells, features=None, pin_start=True, pin_end=True):
    """QvEvaluator's Inc / Del / Extra / Merge (QvEvaluator.hpp:153-207) at the (i, j) cells: four lists, NaN outside
    a move's domain.  features: dict of ins/subs/del/del_tag/merge lists (del_tag as characters)."""
    L = _qlib()
    f = L.qorc_eval_moves
    F = ctypes.POINTER(ctypes.c_float)
    f.argtypes = [ctypes.c_char_p] + [F] * 5 + [ctypes.c_char_p, F, ctypes.c_int, ctypes.c_int,
                                                 ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                                 ctypes.c_int, F]
    feats = features or {}
    arrs = []
    for k in ("ins", "subs", "del", "del_tag", "merge"):
        v = feats.get(k)
        if v is None:
            arrs.append(None)
        else:
            arrs.append(_farr([float(ord(c)) if isinstance(c, str) else float(c) for c in v]))
    n = len(cells)
    out = (ctypes.c_float * max(1, 4 * n))()
    f(seq.encode(), *arrs, tpl.encode(), _farr(qv_params(params)), 1 if pin_start else 0, 1 if pin_end else 0,
      _iarr([c[0] for c in cells] or [0]), _iarr([c[1] for c in cells] or [0]), n, out)
    return [list(out[k * n:(k + 1) * n]) for k in range(4)]


def quiver_log_add(a, b):
    return _qlib().qorc_log_add(a, b)


# ---------------------------------------------------------------- POA (oracle/poa_oracle.cpp)
POA_GLOBAL, POA_SEMIGLOBAL, POA_LOCAL = 0, 1, 2
INT_MAX = 2**31 - 1


def _cstrs(seqs):
    arr = (ctypes.c_char_p * max(1, len(seqs)))()
    for k, s in enumerate(seqs):
        arr[k] = None if s is None else s.encode()
    return arr


def poa_consensus(reads, mode=POA_GLOBAL, min_coverage=-INT_MAX, graphviz_flags=None):
    """PoaConsensus::FindConsensus(reads, mode, minCoverage): the consensus, plus ToGraphViz(flags) when
    graphviz_flags is given (1 = COLOR_NODES, 2 = VERBOSE_NODES)."""
    cap = sum(len(r) for r in reads) + 16
    seq = ctypes.create_string_buffer(cap)
    dot = ctypes.create_string_buffer(512 * (cap + 8) + 4096) if graphviz_flags is not None else None
    n = lib().orc_poa_consensus(_cstrs(reads), len(reads), mode, min_coverage, seq, cap, dot,
                                len(dot) if dot is not None else 0, graphviz_flags or 0)
    if n < 0:
        raise ValueError("Input sequences must have nonzero length.")
    return (seq.value.decode(), dot.value.decode()) if dot is not None else seq.value.decode()


def sparse_poa(reads, min_coverage=None, max_coverage=None):
    """SparsePoa driven as Consensus.h's PoaConsensus does (None reads get key -1).  Returns
    {"consensus", "keys" (per input read; -2 = not reached), "summaries" (per POA key: rc, read, tpl)}."""
    n = len(reads)
    keys = (ctypes.c_int * max(1, n))()
    nk = ctypes.c_int()
    rc = (ctypes.c_int * max(1, n))()
    ext = (ctypes.c_int * max(4, 4 * n))()
    cap = sum(len(r) for r in reads if r) + 16
    seq = ctypes.create_string_buffer(cap)
    lib().orc_sparse_poa(_cstrs(reads), n, -1 if min_coverage is None else min_coverage,
                         2**62 if max_coverage is None else max_coverage, keys, ctypes.byref(nk), rc, ext, seq, cap)
    summ = [{"rc": bool(rc[k]), "read": (ext[4 * k], ext[4 * k + 1]), "tpl": (ext[4 * k + 2], ext[4 * k + 3])}
            for k in range(nk.value)]
    return {"consensus": seq.value.decode(), "keys": list(keys[:n]), "summaries": summ}


def poa_kat_reads(kind):
    """The 100 seeded sequences of TestSparsePoa.cpp's SingleReadx100 (kind 0) / SingleAndHalfx100 (kind 1)."""
    cap = 100 * 20001
    buf = ctypes.create_string_buffer(cap)
    lens = (ctypes.c_int * 100)()
    total = lib().orc_poa_kat_reads(kind, buf, cap, lens)
    assert total > 0
    raw = buf.raw[:total].decode()
    out, o = [], 0
    for L in lens:
        out.append(raw[o:o + L])
        o += L
    return out
