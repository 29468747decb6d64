"""POA draft step on the GPU: the Python mirror of pbccs's SparsePoa
(include/pacbio/ccs/SparsePoa.h:94-131, src/SparsePoa.cpp) and ConsensusCore's PoaConsensus::FindConsensus,
over the C ABI's pbccs_sparse_poa_* / pbccs_poa_* calls, plus the batched form ccs needs
(pbccs_poa_batch: every ZMW of a batch adds its next read in the same device round).

The read-vs-graph DP and its traceback run in HIP (k_poa_fill / k_poa_trace); the graph is host state.
There is no CPU fallback: without the library these raise."""
import ctypes

from . import lib as _L
from .lib import load

GLOBAL, SEMIGLOBAL, LOCAL = 0, 1, 2
COLOR_NODES, VERBOSE_NODES = 1, 2
INT_MAX = 2**31 - 1


def _engine(engine):
    if engine is None:
        from . import default_engine
        engine = default_engine()
    return engine


def _text(fn, first=1 << 16):
    """Call fn(buf, cap, &len) and grow the buffer once on ERANGE."""
    cap = first
    for _ in range(2):
        buf = ctypes.create_string_buffer(cap + 1)
        n = ctypes.c_int()
        rc = fn(buf, cap, ctypes.byref(n))
        if rc == -5 and n.value > cap:
            cap = n.value
            continue
        _L.check(rc)
        return buf.raw[:n.value].decode()
    raise _L.PbccsError(-5, "buffer too small")


class SparsePoa:
    """PacBio::CCS::SparsePoa: OrientAndAddRead and FindConsensus with PoaAlignmentSummary extents."""

    def __init__(self, engine=None):
        self._eng = _engine(engine)
        h = ctypes.c_void_p()
        _L.check(load().pbccs_sparse_poa_create(self._eng._h, ctypes.byref(h)))
        self._h = h
        self._lib = load()
        self._n = 0

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.pbccs_sparse_poa_destroy(self._h)
            self._h = None

    def OrientAndAddRead(self, seq, min_score_to_add=0.0):
        key = ctypes.c_int()
        b = seq.encode()
        _L.check(load().pbccs_sparse_poa_orient_and_add_read(self._h, b, len(b), min_score_to_add, ctypes.byref(key)))
        if key.value >= 0:
            self._n += 1
        return key.value

    # the Consensus.h / driver.py surface
    orient_and_add_read = OrientAndAddRead

    def FindConsensus(self, min_coverage):
        """(consensus, [{"rc", "read": (b, e), "tpl": (b, e)} per key])"""
        n = max(1, self._n)
        rc = (ctypes.c_int * n)()
        ext = (ctypes.c_int * (4 * n))()
        nk = ctypes.c_int()
        css = _text(lambda buf, cap, ln: load().pbccs_sparse_poa_find_consensus(
            self._h, min_coverage, buf, cap, ln, rc, ext, ctypes.byref(nk)))
        return css, [{"rc": bool(rc[k]), "read": (ext[4 * k], ext[4 * k + 1]), "tpl": (ext[4 * k + 2], ext[4 * k + 3])}
                     for k in range(nk.value)]

    def find_consensus(self, min_coverage):
        css, summ = self.FindConsensus(min_coverage)
        return css, {k: s for k, s in enumerate(summ)}

    def ToGraphViz(self, flags=0, min_coverage=-INT_MAX):
        return _text(lambda buf, cap, ln: load().pbccs_sparse_poa_graphviz(self._h, flags, min_coverage, buf, cap, ln))


def poa_consensus(reads, mode=GLOBAL, min_coverage=-INT_MAX, graphviz_flags=None, engine=None):
    """PoaConsensus::FindConsensus(reads, mode, minCoverage): the consensus sequence, and with
    graphviz_flags also pc->Graph.ToGraphViz(flags, pc)."""
    eng = _engine(engine)
    enc = [r.encode() for r in reads]
    arr = (ctypes.c_char_p * max(1, len(enc)))(*enc)
    lens = (ctypes.c_int * max(1, len(enc)))(*[len(r) for r in enc])
    cap = sum(len(r) for r in enc) + 16
    dcap = 256 * cap + 4096 if graphviz_flags is not None else 0
    out = ctypes.create_string_buffer(cap)
    dot = ctypes.create_string_buffer(dcap) if graphviz_flags is not None else None
    n, dn = ctypes.c_int(), ctypes.c_int()
    _L.check(load().pbccs_poa_consensus(eng._h, arr, lens, len(enc), mode, min_coverage, out, cap, ctypes.byref(n),
                                        graphviz_flags or 0, dot, dcap, ctypes.byref(dn)))
    seq = out.raw[:n.value].decode()
    return (seq, dot.raw[:dn.value].decode()) if dot is not None else seq


def poa_batch(zmw_reads, max_coverage=None, min_coverage=-1, engine=None):
    """Consensus.h's PoaConsensus for many ZMWs at once.  zmw_reads: per ZMW, the subreads in FilterReads
    order (None = dropped).  Returns per ZMW {"consensus", "keys" (per read: key, -1, or -2 past
    maxPoaCov), "summaries" (per key: rc, read, tpl extents)}.

    Marshalling is flat: all reads in one buffer with a pointer table, all outputs in shared arrays, so
    the per-ZMW Python work is a few struct-field stores."""
    import numpy as np
    eng = _engine(engine)
    n = len(zmw_reads)
    counts = np.fromiter((len(r) for r in zmw_reads), dtype=np.int64, count=n)
    flat = [r for reads in zmw_reads for r in reads]
    enc = [b"" if r is None else r.encode() for r in flat]
    lens = np.fromiter((len(e) for e in enc), dtype=np.int32, count=len(enc))
    blob = ctypes.create_string_buffer(b"".join(enc), max(1, int(lens.sum())))
    starts = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=starts[1:])
    ptrs = (ctypes.addressof(blob) + starts[:-1]).astype(np.uint64)
    ptrs[lens == 0] = 0                                  # NULL: a read FilterReads dropped
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=first[1:])
    # per-ZMW consensus capacity: its read bases + 16; per-read outputs shared
    zbases = starts[first[1:]] - starts[first[:-1]] + 16   # (reduceat would fail on a trailing read-less ZMW)
    cstart = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(zbases, out=cstart[1:])
    cbuf = ctypes.create_string_buffer(max(1, int(cstart[-1])))
    keys = np.zeros(max(1, len(enc)), dtype=np.int32)
    rc = np.zeros(max(1, len(enc)), dtype=np.int32)
    ext = np.zeros(max(4, 4 * len(enc)), dtype=np.int32)
    # the per-ZMW structs filled column-wise through numpy views of their memory (one ctypes attribute store per
    # field per ZMW was most of the marshalling time at thousands of ZMWs)
    from .quiver import _struct_dtype
    ins = np.zeros(max(1, n), dtype=_struct_dtype(_L.CPoaInput))
    outs = np.zeros(max(1, n), dtype=_struct_dtype(_L.CPoaOutput))
    if n:
        f0 = first[:-1]
        ins["seqs"][:n] = ptrs.ctypes.data + 8 * f0
        ins["lens"][:n] = lens.ctypes.data + 4 * f0
        ins["n_reads"][:n] = counts
        outs["consensus"][:n] = ctypes.addressof(cbuf) + cstart[:-1]
        outs["cap"][:n] = zbases
        outs["keys"][:n] = keys.ctypes.data + 4 * f0
        outs["rc"][:n] = rc.ctypes.data + 4 * f0
        outs["extents"][:n] = ext.ctypes.data + 16 * f0
    mc = 2**62 if max_coverage is None else int(max_coverage)
    _L.check(load().pbccs_poa_batch(eng._h, ctypes.cast(ins.ctypes.data, ctypes.POINTER(_L.CPoaInput)), n, mc,
                                    int(min_coverage), ctypes.cast(outs.ctypes.data, ctypes.POINTER(_L.CPoaOutput))))
    raw = cbuf.raw
    firsts, cnts, nks = first.tolist(), counts.tolist(), outs["n_keys"][:n].tolist()
    cs, lns = cstart.tolist(), outs["len"][:n].tolist()
    keys_l, rc_l, ext_l = keys.tolist(), rc.tolist(), ext.tolist()
    res = []
    for z in range(n):
        f, nr, nk = firsts[z], cnts[z], nks[z]
        e0 = 4 * f
        res.append({"consensus": raw[cs[z]:cs[z] + lns[z]].decode(),
                    "keys": keys_l[f:f + nr],
                    "summaries": [{"rc": bool(rc_l[f + k]), "read": (ext_l[e0 + 4 * k], ext_l[e0 + 4 * k + 1]),
                                   "tpl": (ext_l[e0 + 4 * k + 2], ext_l[e0 + 4 * k + 3])} for k in range(nk)]})
    return res


def poa_stats(engine=None, reset=False):
    eng = _engine(engine)
    s = _L.CPoaStats()
    _L.check(load().pbccs_poa_stats_get(eng._h, ctypes.byref(s), 1 if reset else 0))
    return {k: getattr(s, k) for k, _ in _L.CPoaStats._fields_}
