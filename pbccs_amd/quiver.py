"""Quiver family mirror (ConsensusCore/include/ConsensusCore/Quiver/): QvModelParams, QuiverConfig,
QuiverConfigTable and MultiReadMutationScorer over the HIP engine's C ABI (include/pbccs_amd.h,
pbccs_quiver_*).  Viterbi = SparseSseQvRecursor, sum-product = SparseSseQvSumProductRecursor
(Quiver/MultiReadMutationScorer.hpp:242-245).  No CPU fallback."""
import ctypes
import math

from . import lib as _lib_mod
from .lib import load

INCORPORATE, EXTRA, DELETE, MERGE = 1, 2, 4, 8
BASIC_MOVES, ALL_MOVES = 7, 15
_PARAM_FIELDS = ("Match", "Mismatch", "MismatchS", "Branch", "BranchS", "DeletionN", "DeletionWithTag",
                 "DeletionWithTagS", "Nce", "NceS")


class QvModelParams:
    """QvModelParams (QuiverConfig.hpp:79-176): Merge / MergeS may be one rate or four per-base rates."""

    def __init__(self, chemistry="*", model="", **kw):
        self.ChemistryName, self.ModelName = chemistry, model
        for k in _PARAM_FIELDS:
            setattr(self, k, float(kw.get(k, 0.0)))
        for k in ("Merge", "MergeS"):
            v = kw.get(k, 0.0)
            setattr(self, k, [float(x) for x in v] if isinstance(v, (list, tuple)) else [float(v)] * 4)

    def _c(self):
        c = _lib_mod.CQvModelParams()
        for k, cn in zip(_PARAM_FIELDS, ("match", "mismatch", "mismatch_s", "branch", "branch_s", "deletion_n",
                                         "deletion_with_tag", "deletion_with_tag_s", "nce", "nce_s")):
            setattr(c, cn, getattr(self, k))
        for i in range(4):
            c.merge[i] = self.Merge[i]
            c.merge_s[i] = self.MergeS[i]
        return c


RECURSORS = ("SparseSse", "SparseSimple", "DenseSse", "DenseSimple")   # PBCCS_QV_RECURSOR_* order


class QuiverConfig:
    """QuiverConfig (QuiverConfig.hpp:181-199); BandingOptions(diagCross, scoreDiff) -> score_diff.
    recursor picks the recursor type of ConsensusCore's typedefs (Quiver/MutationScorer.hpp:93-99):
    SparseSse (SparseSseQvRecursor, the MultiReadMutationScorer default), SparseSimple, DenseSse
    (SseQvRecursor) or DenseSimple (SimpleQvRecursor)."""

    def __init__(self, params, moves=ALL_MOVES, score_diff=12.5, fast_score_threshold=-12.5, add_threshold=1.0,
                 sum_product=False, recursor="SparseSse"):
        self.QvParams, self.MovesAvailable = params, moves
        self.ScoreDiff, self.FastScoreThreshold, self.AddThreshold = score_diff, fast_score_threshold, add_threshold
        self.SumProduct = sum_product
        self.Recursor = recursor

    def _c(self):
        c = _lib_mod.CQuiverConfig()
        c.params = self.QvParams._c()
        c.moves_available = self.MovesAvailable
        c.score_diff = self.ScoreDiff
        c.fast_score_threshold = self.FastScoreThreshold
        c.add_threshold = self.AddThreshold
        c.sum_product = 1 if self.SumProduct else 0
        c.recursor = RECURSORS.index(self.Recursor)
        return c


class QuiverConfigTable:
    """QuiverConfigTable (QuiverConfig.cpp:67-138): Insert (by chemistry), InsertAs, InsertDefault ("*")."""

    def __init__(self):
        self.entries = []

    def InsertAs(self, name, config):
        if name == "*":
            raise ValueError("Cannot Insert(...) a QuiverConfig with chemistry '*'")
        return self._insert(name, config)

    def Insert(self, config):
        return self.InsertAs(config.QvParams.ChemistryName, config)

    def InsertDefault(self, config):
        return self._insert("*", config)

    def _insert(self, name, config):
        if any(n == name for n, _ in self.entries):
            return False
        self.entries.insert(0, (name, config))
        return True


class QvSequenceFeatures:
    """QvSequenceFeatures (Features.hpp:69-100): the bases and the five QV tracks (InsQv, SubsQv, DelQv, DelTag,
    MergeQv); a missing track reads as zeros; DelTag may hold characters or their float codes."""

    def __init__(self, seq, ins_qv=None, subs_qv=None, del_qv=None, del_tag=None, merge_qv=None):
        n = len(seq)
        self.Sequence = seq
        self.SequenceAsFloat = [float(ord(c)) for c in seq]

        def track(v, tag=False):
            if v is None:
                return [0.0] * n
            if len(v) != n:
                raise ValueError("feature track length differs from the sequence")
            return [float(ord(x)) if tag and isinstance(x, str) else float(x) for x in v]
        self.InsQv, self.SubsQv, self.DelQv = track(ins_qv), track(subs_qv), track(del_qv)
        self.DelTag, self.MergeQv = track(del_tag, True), track(merge_qv)

    def Length(self):
        return len(self.Sequence)

    def __getitem__(self, i):
        return self.Sequence[i]

    def _c(self):
        f = _lib_mod.CQvFeatures()
        f.seq = self.Sequence.encode()
        f.len = len(self.Sequence)
        self._keep = []
        for name, v in (("ins_qv", self.InsQv), ("subs_qv", self.SubsQv), ("del_qv", self.DelQv),
                        ("del_tag", self.DelTag), ("merge_qv", self.MergeQv)):
            a = (ctypes.c_float * max(1, len(v)))(*v)
            self._keep.append(a)
            setattr(f, name, ctypes.cast(a, ctypes.POINTER(ctypes.c_float)))
        return f


class QvEvaluator:
    """QvEvaluator (Quiver/QvEvaluator.hpp:90-317): the move scores of one read against a template, evaluated on
    the device by the recursions' own evaluator (pbccs_qv_evaluator_moves).  Inc / Del / Extra / Merge take one
    cell; Moves takes many (one launch).  A cell outside a move's domain (the reference asserts) gives NaN."""

    def __init__(self, features, tpl, params, pin_start=True, pin_end=True, read_name="", engine=None):
        from . import default_engine
        self._f = features if isinstance(features, QvSequenceFeatures) else QvSequenceFeatures(features)
        self._tpl, self._p = tpl, params
        self._pins = (bool(pin_start), bool(pin_end))
        self._name = read_name
        self._eng = engine or default_engine()

    def ReadName(self):
        return self._name

    def Basecalls(self):
        return self._f.Sequence

    def Template(self, tpl=None):
        if tpl is None:
            return self._tpl
        self._tpl = tpl

    def ReadLength(self):
        return self._f.Length()

    def TemplateLength(self):
        return len(self._tpl)

    def PinStart(self):
        return self._pins[0]

    def PinEnd(self):
        return self._pins[1]

    def IsMatch(self, i, j):
        return self._f.Sequence[i] == self._tpl[j]

    def Moves(self, cells):
        """(Inc, Del, Extra, Merge) lists at the (i, j) cells."""
        n = len(cells)
        if n == 0:
            return [], [], [], []
        ci = (ctypes.c_int * n)(*[c[0] for c in cells])
        cj = (ctypes.c_int * n)(*[c[1] for c in cells])
        outs = [(ctypes.c_float * n)() for _ in range(4)]
        f = self._f._c()
        p = self._p._c()
        _lib_mod.check(load().pbccs_qv_evaluator_moves(self._eng._h, ctypes.byref(f), self._tpl.encode(),
                                                        len(self._tpl), ctypes.byref(p), int(self._pins[0]),
                                                        int(self._pins[1]), ci, cj, n, *outs))
        return tuple(list(o) for o in outs)

    def Inc(self, i, j):
        return self.Moves([(i, j)])[0][0]

    def Del(self, i, j):
        return self.Moves([(i, j)])[1][0]

    def Extra(self, i, j):
        return self.Moves([(i, j)])[2][0]

    def Merge(self, i, j):
        return self.Moves([(i, j)])[3][0]


class QuiverMultiReadMutationScorer:
    """MultiReadMutationScorer<SparseSse{Qv,QvSumProduct}Recursor> (Quiver/MultiReadMutationScorer.cpp)."""

    def __init__(self, configs, tpl, engine=None):
        from . import default_engine
        if isinstance(configs, QuiverConfig):
            t = QuiverConfigTable()
            t.InsertDefault(configs)
            configs = t
        self._eng = engine or default_engine()
        n = len(configs.entries)
        arr = (_lib_mod.CQuiverConfig * n)(*[c._c() for _, c in configs.entries])
        names = (ctypes.c_char_p * n)(*[name.encode() for name, _ in configs.entries])
        h = ctypes.c_void_p()
        _lib_mod.check(load().pbccs_quiver_scorer_create(self._eng._h, arr, names, n, tpl.encode(), len(tpl),
                                                          ctypes.byref(h)))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            load().pbccs_quiver_scorer_destroy(self._h)
            self._h = None

    def AddRead(self, seq, strand=0, template_start=0, template_end=None, ins_qv=None, subs_qv=None, del_qv=None,
                del_tag=None, merge_qv=None, chemistry="*", threshold=None):
        if template_end is None:
            template_end = self.TemplateLength()

        def arr(v, tag=False):
            if v is None:
                return None
            vals = [float(ord(x)) if tag and isinstance(x, str) else float(x) for x in v]
            return (ctypes.c_float * len(vals))(*vals)

        active = ctypes.c_int()
        _lib_mod.check(load().pbccs_quiver_scorer_add_read(
            self._h, seq.encode(), len(seq), arr(ins_qv), arr(subs_qv), arr(del_qv), arr(del_tag, True),
            arr(merge_qv), chemistry.encode(), strand, template_start, template_end,
            float("nan") if threshold is None else threshold, ctypes.byref(active)))
        return bool(active.value)

    def ScoreMany(self, muts, fast=False):
        n = len(muts)
        arr = (_lib_mod.CMutation * max(1, n))(*[m._c() for m in muts])
        out = (ctypes.c_float * max(1, n))()
        _lib_mod.check(load().pbccs_quiver_scorer_score_many(self._h, arr, n, 1 if fast else 0, out))
        return list(out[:n])

    def Score(self, m):
        return self.ScoreMany([m])[0]

    def FastScore(self, m):
        return self.ScoreMany([m], fast=True)[0]

    def ReadScoreMutation(self, i, m):
        """MutationScorer::ScoreMutation on read i's scorer (read coordinates, absolute score)."""
        v = ctypes.c_float()
        c = m._c()
        _lib_mod.check(load().pbccs_quiver_scorer_read_score_mutation(self._h, i, ctypes.byref(c), ctypes.byref(v)))
        return v.value

    def Scores(self, m, unscored_value=0.0):
        out = (ctypes.c_float * max(1, self.NumReads()))()
        c = m._c()
        _lib_mod.check(load().pbccs_quiver_scorer_scores(self._h, ctypes.byref(c), unscored_value, out))
        return list(out[: self.NumReads()])

    def IsFavorable(self, m):
        v = ctypes.c_int()
        c = m._c()
        _lib_mod.check(load().pbccs_quiver_scorer_is_favorable(self._h, ctypes.byref(c), 0, ctypes.byref(v)))
        return bool(v.value)

    def FastIsFavorable(self, m):
        v = ctypes.c_int()
        c = m._c()
        _lib_mod.check(load().pbccs_quiver_scorer_is_favorable(self._h, ctypes.byref(c), 1, ctypes.byref(v)))
        return bool(v.value)

    def ApplyMutations(self, muts):
        arr = (_lib_mod.CMutation * max(1, len(muts)))(*[m._c() for m in muts])
        _lib_mod.check(load().pbccs_quiver_scorer_apply_mutations(self._h, arr, len(muts)))

    def Template(self, strand=0):
        buf = ctypes.create_string_buffer(1 << 22)
        n = ctypes.c_int()
        _lib_mod.check(load().pbccs_quiver_scorer_template(self._h, strand, buf, len(buf), ctypes.byref(n)))
        return buf.value.decode()

    def TemplateLength(self):
        return len(self.Template())

    def NumReads(self):
        return load().pbccs_quiver_scorer_num_reads(self._h)

    def ReadInfo(self, i):
        a, s, ts, te = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib_mod.check(load().pbccs_quiver_scorer_read_info(self._h, i, ctypes.byref(a), ctypes.byref(s),
                                                             ctypes.byref(ts), ctypes.byref(te)))
        return {"active": bool(a.value), "strand": s.value, "template_start": ts.value, "template_end": te.value}

    def BaselineScore(self):
        v = ctypes.c_float()
        _lib_mod.check(load().pbccs_quiver_scorer_baseline_score(self._h, ctypes.byref(v)))
        return v.value

    def BaselineScores(self):
        out = (ctypes.c_float * max(1, self.NumReads()))()
        n = ctypes.c_int()
        _lib_mod.check(load().pbccs_quiver_scorer_baseline_scores(self._h, out, self.NumReads(), ctypes.byref(n)))
        return list(out[: n.value])

    def NumFlipFlops(self):
        out = (ctypes.c_int * max(1, self.NumReads()))()
        _lib_mod.check(load().pbccs_quiver_scorer_num_flipflops(self._h, out))
        return list(out[: self.NumReads()])

    def Alignment(self, i):
        """RecursorBase::Alignment of read i (Viterbi): (Target(), Query()) of the PairwiseAlignment."""
        cap = 2 * len(self.Template()) + 4096
        for _ in range(2):
            t = ctypes.create_string_buffer(cap)
            q = ctypes.create_string_buffer(cap)
            n = ctypes.c_int()
            rc = load().pbccs_quiver_scorer_alignment(self._h, i, t, q, cap, ctypes.byref(n))
            if rc == -5 and n.value > cap:
                cap = n.value
                continue
            _lib_mod.check(rc)
            return t.raw[:n.value].decode(), q.raw[:n.value].decode()
        raise _lib_mod.PbccsError(-5, "buffer too small")

    def AllocatedEntries(self, i):
        a, b = ctypes.c_longlong(), ctypes.c_longlong()
        _lib_mod.check(load().pbccs_quiver_scorer_allocated_entries(self._h, i, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value


def RefineConsensus(mms, max_iterations=40, mutation_separation=10, mutation_neighborhood=20):
    o = _lib_mod.CRefineOptions(max_iterations, mutation_separation, mutation_neighborhood)
    nt, na, conv = ctypes.c_longlong(0), ctypes.c_longlong(0), ctypes.c_int()
    _lib_mod.check(load().pbccs_quiver_refine_consensus(mms._h, ctypes.byref(o), ctypes.byref(nt), ctypes.byref(na),
                                                        ctypes.byref(conv)))
    return bool(conv.value), nt.value, na.value


def ConsensusQVs(mms):
    cap = mms.TemplateLength()
    out = (ctypes.c_int * max(1, cap))()
    n = ctypes.c_int()
    _lib_mod.check(load().pbccs_quiver_consensus_qvs(mms._h, out, cap, ctypes.byref(n)))
    return list(out[: n.value])


def _struct_dtype(ctype):
    """numpy dtype with the memory layout of a ctypes Structure (pointers as uint64): lets the batch entry point's
    input arrays be filled column-wise instead of one ctypes attribute at a time."""
    import numpy as np
    scalars = {ctypes.c_int: np.int32, ctypes.c_float: np.float32, ctypes.c_longlong: np.int64,
               ctypes.c_double: np.float64, ctypes.c_ubyte: np.uint8}

    def field(ft):
        if isinstance(ft, type) and issubclass(ft, ctypes.Structure):   # nested struct (CCcsOutput.polish)
            return _struct_dtype(ft)
        if isinstance(ft, type) and issubclass(ft, ctypes.Array):       # fixed array (snr[4], status_counts[5])
            return (field(ft._type_), (ft._length_,))
        if ft in scalars:
            return scalars[ft]
        assert ctypes.sizeof(ft) == 8   # pointers and char*
        return np.uint64

    names, formats, offsets = [], [], []
    for name, ft in ctype._fields_:
        names.append(name)
        offsets.append(getattr(ctype, name).offset)
        formats.append(field(ft))
    return np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": ctypes.sizeof(ctype)})


class PreparedQuiverBatch:
    """The batch entry point's inputs marshalled once (host structures pointing at the caller's arrays): the bench
    builds it outside its timed region, as the Arrow bench's PreparedBatch; run() is the native call."""

    def __init__(self, zmws, configs, qvs=True):
        import numpy as np
        self.zmws = zmws   # the read arrays are passed in place
        if isinstance(configs, QuiverConfig):
            t = QuiverConfigTable()
            t.InsertDefault(configs)
            configs = t
        nc = len(configs.entries)
        carr = (_lib_mod.CQuiverConfig * nc)(*[c._c() for _, c in configs.entries])
        names = (ctypes.c_char_p * nc)(*[name.encode() for name, _ in configs.entries])
        n = len(zmws)
        keep = []
        reads = [r for z in zmws for r in z["reads"]]
        nr = len(reads)
        seqs = [r["seq"].encode() for r in reads]
        lens = np.fromiter(map(len, seqs), dtype=np.int64, count=nr)
        off = np.zeros(nr, dtype=np.int64)
        if nr > 1:
            np.cumsum(lens[:-1], out=off[1:])
        rd = np.zeros(max(1, nr), dtype=_struct_dtype(_lib_mod.CQuiverRead))
        if nr:
            sbuf = np.frombuffer(b"".join(seqs) + b"\0", dtype=np.uint8)
            keep.append(sbuf)
            rd["seq"][:nr] = sbuf.ctypes.data + off
            rd["len"][:nr] = lens
        # QV tracks: each read's float32 array is passed in place (a read without the track passes NULL: zeros on
        # the C side, which copies every track once into its host pool)
        lens_l = lens.tolist()
        for field, key in (("ins_qv", "ins"), ("subs_qv", "subs"), ("del_qv", "del"), ("del_tag", "del_tag"),
                           ("merge_qv", "merge")):
            ptr = [0] * nr
            for i, r in enumerate(reads):
                v = (r.get("features") or {}).get(key)
                if v is None:
                    continue
                if isinstance(v, np.ndarray):   # numeric tracks (tags as character codes)
                    a = np.ascontiguousarray(v, dtype=np.float32)
                elif key == "del_tag":
                    a = np.array([float(ord(x)) if isinstance(x, str) else float(x) for x in v], dtype=np.float32)
                else:
                    a = np.asarray(v, dtype=np.float32)
                if a.size != lens_l[i] or a.ndim != 1:
                    raise ValueError(f"QV track {key} of read {i} has {a.size} entries for {lens_l[i]} bases")
                if a is not v:
                    keep.append(a)
                ptr[i] = a.ctypes.data
            rd[field][:nr] = ptr
        chem_names = {}
        chem = np.zeros(nr, dtype=np.uint64)
        for i, r in enumerate(reads):
            c = r.get("chemistry", "*")
            if c not in chem_names:
                b = ctypes.create_string_buffer(c.encode())
                keep.append(b)
                chem_names[c] = ctypes.addressof(b)
            chem[i] = chem_names[c]
        rd["chemistry"][:nr] = chem
        rd["strand"][:nr] = [r.get("strand", 0) for r in reads]
        rd["tstart"][:nr] = [r.get("ts", 0) for r in reads]
        rd["tend"][:nr] = [-1 if r.get("te") is None else r["te"] for r in reads]
        rd["threshold"][:nr] = [float("nan") if r.get("threshold") is None else r["threshold"] for r in reads]
        keep.append(rd)
        # ZMWs: template, reads slice, output buffers (one consensus and one QV buffer for the batch)
        tpls = [z["tpl"].encode() for z in zmws]
        tl = np.fromiter(map(len, tpls), dtype=np.int64, count=n)
        cz = np.zeros(max(1, n), dtype=_struct_dtype(_lib_mod.CQuiverZmw))
        res = np.zeros(max(1, n), dtype=_struct_dtype(_lib_mod.CQuiverResult))
        nreads = np.fromiter((len(z["reads"]) for z in zmws), dtype=np.int64, count=n)
        rstart = np.zeros(n, dtype=np.int64)
        if n > 1:
            np.cumsum(nreads[:-1], out=rstart[1:])
        cap = 2 * tl + 64
        cstart = np.zeros(n, dtype=np.int64)
        if n > 1:
            np.cumsum(cap[:-1], out=cstart[1:])
        total = int(cap.sum()) if n else 0
        cons = np.zeros(max(1, total), dtype=np.uint8)
        qvb = np.zeros(max(1, total), dtype=np.int32)
        if n:
            tbuf = np.frombuffer(b"\0".join(tpls) + b"\0", dtype=np.uint8)
            keep.append(tbuf)
            tstart = np.zeros(n, dtype=np.int64)
            if n > 1:
                np.cumsum(tl[:-1] + 1, out=tstart[1:])
            cz["tpl"][:n] = tbuf.ctypes.data + tstart
            cz["tpl_len"][:n] = tl
            cz["reads"][:n] = rd.ctypes.data + rd.dtype.itemsize * rstart
            cz["n_reads"][:n] = nreads
            res["consensus"][:n] = cons.ctypes.data + cstart
            res["consensus_cap"][:n] = cap
            res["qvs"][:n] = (qvb.ctypes.data + 4 * cstart) if qvs else 0
        self.__dict__.update(dict(keep=keep, carr=carr, names=names, nc=nc, cz=cz, res=res, n=n, cap=cap,
                                  cstart=cstart, cons=cons, qvb=qvb, qvs=qvs))

    def run(self, max_iterations=40, mutation_separation=10, mutation_neighborhood=20, engine=None):
        from . import default_engine
        eng = engine or default_engine()
        carr, names, nc, cz, res, n = self.carr, self.names, self.nc, self.cz, self.res, self.n
        cap, cstart, cons, qvb, qvs = self.cap, self.cstart, self.cons, self.qvb, self.qvs
        o = _lib_mod.CRefineOptions(max_iterations, mutation_separation, mutation_neighborhood)
        _lib_mod.check(load().pbccs_quiver_polish_batch(
            eng._h, carr, names, nc, ctypes.cast(cz.ctypes.data, ctypes.POINTER(_lib_mod.CQuiverZmw)), n,
            ctypes.byref(o), ctypes.cast(res.ctypes.data, ctypes.POINTER(_lib_mod.CQuiverResult))))
        # per-field columns as Python lists once (not one structured-record access per field per ZMW)
        lens, oks = res["consensus_len"][:n].tolist(), res["ok"][:n].tolist()
        tested, applied = res["n_tested"][:n].tolist(), res["n_applied"][:n].tolist()
        conv, active = res["converged"][:n].tolist(), res["n_active"][:n].tolist()
        caps, starts = cap.tolist(), cstart.tolist()
        cbytes = cons.tobytes()
        out = []
        for k in range(n):
            ln = lens[k]
            if ln > caps[k]:
                raise _lib_mod.PbccsError(-5, "consensus outgrew its buffer")
            c0 = starts[k]
            ok = bool(oks[k])
            out.append({"consensus": cbytes[c0:c0 + ln].decode(),
                        "qvs": qvb[c0:c0 + ln].tolist() if qvs and ok else None,
                        "n_tested": tested[k], "n_applied": applied[k],
                        "converged": bool(conv[k]), "ok": ok, "n_active": active[k]})
        return out


def polish_batch(zmws, configs, max_iterations=40, mutation_separation=10, mutation_neighborhood=20, qvs=True,
                 engine=None):
    """Many Quiver scorers at once (pbccs_quiver_polish_batch): per ZMW, create the scorer over `configs`,
    AddRead every read, RefineConsensus and (qvs) ConsensusQVs -- the per-scorer call sequence, with the
    scorers' rounds in lock-step on the device.

    zmws: [{"tpl", "reads": [{"seq", "strand", "ts", "te", "features": {ins, subs, del, del_tag, merge},
    "chemistry"?}]}].  Returns per ZMW {"consensus", "qvs", "n_tested", "n_applied", "converged", "ok",
    "n_active"}."""
    return PreparedQuiverBatch(zmws, configs, qvs).run(max_iterations, mutation_separation, mutation_neighborhood,
                                                        engine)
