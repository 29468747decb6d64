"""Batched ccs polish driver: pbccs' Consensus<>() from the scorer setup on (Consensus.h:436-552).

The POA draft, FilterReads and ExtractMappedRead (Consensus.h:223-325, 352-390) run before the boundary
(pbccs_amd.driver): it takes a draft plus mapped, extent-clipped reads per ZMW, exactly what Consensus.h
hands to ArrowMultiReadMutationScorer.  Thousands of ZMWs go to the GPU per call; results come back in input order.
"""
import ctypes
import math

from . import lib as L


class ConsensusSettings:
    """ConsensusSettings (include/pacbio/ccs/Consensus.h:86-111, defaults src/Consensus.cpp:46-54)."""

    def __init__(self, min_passes=3, min_length=10, min_zscore=-5.0, max_drop_fraction=0.34,
                 min_predicted_accuracy=0.90, score_diff=12.5, max_iterations=40, mutation_separation=10,
                 mutation_neighborhood=20, zmws_per_batch=0):
        self.min_passes = min_passes
        self.min_length = min_length
        self.min_zscore = min_zscore
        self.max_drop_fraction = max_drop_fraction
        self.min_predicted_accuracy = min_predicted_accuracy
        self.score_diff = score_diff
        self.max_iterations = max_iterations
        self.mutation_separation = mutation_separation
        self.mutation_neighborhood = mutation_neighborhood
        self.zmws_per_batch = zmws_per_batch

    def _c(self):
        o = L.CPolishOptions()
        o.min_passes = self.min_passes
        o.min_length = self.min_length
        o.min_zscore = self.min_zscore
        o.max_drop_fraction = self.max_drop_fraction
        o.min_predicted_accuracy = self.min_predicted_accuracy
        o.score_diff = self.score_diff
        o.refine = L.CRefineOptions(self.max_iterations, self.mutation_separation, self.mutation_neighborhood)
        o.zmws_per_batch = self.zmws_per_batch
        return o


class _Marshalled:
    """pbccs_zmw_input / pbccs_zmw_output arrays for a list of ZMW dicts; the output buffers stay owned here."""

    def __init__(self, zmws):
        n = len(zmws)
        self.zmws = zmws
        self._ins = (L.CZmwInput * max(1, n))()
        self._outs = (L.CZmwOutput * max(1, n))()
        self._keep = []
        for i, z in enumerate(zmws):
            reads = z["reads"]
            nr = len(reads)
            draft = z["draft"].encode()
            # a read with no sequence is a placeholder the driver skipped (pbccs_amd.driver): not added, counted
            # in the drop fraction's denominator only
            seqs = (ctypes.c_char_p * max(1, nr))(*[None if r["seq"] is None else r["seq"].encode() for r in reads])
            lens = (ctypes.c_int * max(1, nr))(*[0 if r["seq"] is None else len(r["seq"]) for r in reads])
            strands = (ctypes.c_int * max(1, nr))(*[int(r.get("strand", 0)) for r in reads])
            ts = (ctypes.c_int * max(1, nr))(*[int(r.get("ts", 0)) for r in reads])
            te = (ctypes.c_int * max(1, nr))(*[int(r.get("te", len(z["draft"]))) for r in reads])
            fp = (ctypes.c_ubyte * max(1, nr))(*[1 if r.get("full_pass", True) else 0 for r in reads])
            cap = 2 * len(draft) + 64
            cons = ctypes.create_string_buffer(cap)
            qv = (ctypes.c_int * cap)()
            arr = (ctypes.c_int * max(1, nr))()
            zs = (ctypes.c_double * max(1, nr))()
            self._keep.append((draft, seqs, lens, strands, ts, te, fp, cons, qv, arr, zs))
            self._ins[i].draft = draft
            self._ins[i].draft_len = len(draft)
            for k in range(4):
                self._ins[i].snr[k] = float(z["snr"][k])
            self._ins[i].n_reads = nr
            self._ins[i].seqs = seqs
            self._ins[i].lens = lens
            self._ins[i].strands = strands
            self._ins[i].tstarts = ts
            self._ins[i].tends = te
            self._ins[i].full_pass = fp
            self._outs[i].consensus = ctypes.cast(cons, ctypes.c_char_p)
            self._outs[i].consensus_cap = cap
            self._outs[i].qvs = qv
            self._outs[i].add_read_results = arr
            self._outs[i].zscores = zs

    def results(self):
        from . import ZMW_STATUS
        res = []
        for i, z in enumerate(self.zmws):
            o = self._outs[i]
            nr = len(z["reads"])
            keep = self._keep[i]
            ln = max(0, o.consensus_len)
            ok = o.status in (0, 6)
            res.append({
                "status": ZMW_STATUS[o.status], "status_code": o.status,
                "consensus": keep[7].raw[:ln].decode() if ok else "",
                "qvs": list(keep[8][:ln]) if ok else [],
                "add_read_results": list(keep[9][:nr]), "zscores": list(keep[10][:nr]),
                "zg": o.zg, "za": o.za, "predicted_accuracy": o.predicted_accuracy, "n_tested": o.n_tested,
                "n_applied": o.n_applied, "n_passes": o.n_passes, "status_counts": list(o.status_counts),
            })
        return res


class PreparedBatch(_Marshalled):
    """ZMWs copied to HBM (pbccs_batch_create); polish() runs the hot path once (pbccs_batch_polish)."""

    def __init__(self, zmws, settings=None, engine=None):
        from . import default_engine
        import time
        self._lib = L.load()
        self.engine = engine or default_engine()
        self.settings = settings or ConsensusSettings()
        t0 = time.perf_counter()
        super().__init__(zmws)
        t1 = time.perf_counter()
        n = len(zmws)
        self._opts = self.settings._c()
        h = ctypes.c_void_p()
        L.check(L.load().pbccs_batch_create(self.engine._h, self._ins, n, ctypes.byref(self._opts), ctypes.byref(h)))
        self._h = h
        self.marshal_s = t1 - t0                     # Python dicts -> the boundary's C structs
        self.create_s = time.perf_counter() - t1     # pbccs_batch_create (per-ZMW setup + upload)

    def polish(self):
        L.check(L.load().pbccs_batch_polish(self._h, self._outs))

    def close(self):
        if getattr(self, "_h", None):
            self._lib.pbccs_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def polish_many(batches):
    """Polish several PreparedBatches of one engine concurrently (pbccs_batch_polish_many)."""
    if not batches:
        return
    n = len(batches)
    hs = (ctypes.c_void_p * n)(*[b._h.value for b in batches])
    outs = (ctypes.POINTER(L.CZmwOutput) * n)(*[ctypes.cast(b._outs, ctypes.POINTER(L.CZmwOutput)) for b in batches])
    L.check(batches[0]._lib.pbccs_batch_polish_many(hs, n, outs))


def polish_zmws(zmws, settings=None, engine=None):
    """Polish ZMWs on the GPU (upload, hot path, download).

    zmws: list of dicts {draft, snr (4), reads: [{seq, strand, ts, te, full_pass?}]}.
    Returns one dict per ZMW: status, consensus, qvs, add_read_results, zscores, zg, za, predicted_accuracy,
    n_tested, n_applied, n_passes, status_counts.
    """
    b = PreparedBatch(zmws, settings, engine)
    try:
        b.polish()
        return b.results()
    finally:
        b.close()


def plan_batches(zmws, budget_bytes, max_per_batch=2000, max_len_ratio=1.5):
    """The work queue's batch plan (pbccs_plan_batches; host only, no device).

    Returns (batches, est): batches = lists of ZMW indices, largest estimated band footprint first;
    est = per-ZMW estimated FP64 band bytes.
    """
    m = _Marshalled(zmws)
    n = len(zmws)
    order = (ctypes.c_int * max(1, n))()
    start = (ctypes.c_int * (n + 1))()
    est = (ctypes.c_double * max(1, n))()
    nb = ctypes.c_int()
    L.check(L.load().pbccs_plan_batches(m._ins, n, float(budget_bytes), int(max_per_batch), float(max_len_ratio),
                                        order, start, est, ctypes.byref(nb)))
    return [list(order[start[b]:start[b + 1]]) for b in range(nb.value)], list(est[:n])


def polish_stream(zmws, settings=None, engine=None):
    """Polish a stream of heterogeneous ZMWs (pbccs_polish_batch): bucketed by length and pass count into
    memory-sized device batches that the engine's workspace slots pull largest-first from one queue, like
    ccs's ZMW work queue (src/main/ccs.cpp:222-262).  Results in input order, as polish_zmws()."""
    from . import default_engine
    engine = engine or default_engine()
    settings = settings or ConsensusSettings()
    m = _Marshalled(zmws)
    opts = settings._c()
    L.check(L.load().pbccs_polish_batch(engine._h, m._ins, len(zmws), ctypes.byref(opts), m._outs))
    return m.results()
