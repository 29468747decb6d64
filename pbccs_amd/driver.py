"""Per-ZMW driver steps on the host side of the boundary: FilterReads, the POA
step's bookkeeping and ExtractMappedRead of include/pacbio/ccs/Consensus.h, turning one ZMW's raw
subreads into the pbccs_zmw_input the GPU polish takes.

    chunk (subreads + SNR) --FilterReads--> ordered reads --POA--> draft + per-read extents
        --ExtractMappedRead--> mapped, extent-clipped reads --> polish boundary (pbccs_batch_*)

The POA itself is pluggable (`poa`: a callable with the SparsePoa contract, below).  The boundary keeps
the reference's bookkeeping: reads the POA did not take and reads ExtractMappedRead rejected are passed as
placeholders (no sequence), so they count in the drop fraction's denominator exactly as Consensus.h's
`nReads = readKeys.size()` does (:441-482).

Parity: no reference test exercises FilterReads / ExtractMappedRead directly; this restatement follows
the cited lines (float32 arithmetic where the reference uses float) and is checked by tests/test_driver.py
against hand-derived expectations -- parity unpinned by reference fixtures.
"""
import numpy as np

ADAPTER_BEFORE = 1
ADAPTER_AFTER = 2
FULL_PASS = ADAPTER_BEFORE | ADAPTER_AFTER


def _full(read):
    f = read.get("flags", FULL_PASS)
    return bool(f & ADAPTER_BEFORE) and bool(f & ADAPTER_AFTER)


def _median(lengths):
    """Median<size_t> (Consensus.h:213-221): the middle element, or 0.5 * (sum of the two middle ones) as
    double, returned as float."""
    v = sorted(lengths)
    n = len(v)
    if n % 2 == 1:
        return np.float32(v[n // 2])
    return np.float32(0.5 * (v[n // 2 - 1] + v[n // 2]))


def filter_reads(reads, min_length):
    """FilterReads (include/pacbio/ccs/Consensus.h:223-292).

    reads: dicts with "seq" and "flags" (LocalContextFlags; default a full pass).  Returns the reads in the
    reference's priority order -- full passes first by closeness of their length to the median full-pass
    length, then the others by the same closeness -- with None for reads of at least twice the median
    length, which sort last.  An empty list when no read can be used (median shorter than min_length)."""
    if not reads:
        return []
    longest = 0
    lengths = []
    for r in reads:
        longest = max(longest, len(r["seq"]))
        if _full(r):
            lengths.append(len(r["seq"]))
    median = np.float32(longest) if not lengths else _median(lengths)
    max_len = 2 * int(median)                 # 2 * static_cast<size_t>(median)
    if median < np.float32(min_length):
        return []
    results = [r if len(r["seq"]) < max_len else None for r in reads]

    def lex(r):
        with np.errstate(divide="ignore", invalid="ignore"):
            l = np.float32(len(r["seq"]))
            v = min(l / median, median / l)   # float arithmetic (:271-272)
        return (v, np.float32(0.0)) if _full(r) else (np.float32(0.0), v)

    # std::stable_sort with "lhs > rhs", nullptr last (:281-289): non-null reads by descending key, ties
    # in input order; Python's sort is stable, so sort on the negated key
    kept = [r for r in results if r is not None]
    kept.sort(key=lambda r: tuple(-x for x in lex(r)))
    return kept + [None] * (len(results) - len(kept))


def extract_mapped_read(read, summary, min_length):
    """ExtractMappedRead (Consensus.h:294-325).  summary: {"rc": bool, "read": (l, r), "tpl": (l, r)}
    (PoaAlignmentSummary: ReverseComplementedRead, ExtentOnRead, ExtentOnConsensus).  Returns the mapped
    read as the polish boundary takes it, or None when the extent on the read is shorter than min_length.
    Quirk: the substring is taken from the read as given, even when the POA
    added it reverse-complemented and the extent is in the reverse complement's coordinates."""
    rs, re_ = summary["read"]
    ts, te = summary["tpl"]
    if rs > re_ or re_ - rs < min_length:
        return None
    return {"seq": read["seq"][rs:re_], "strand": 1 if summary["rc"] else 0, "ts": int(ts), "te": int(te),
            "full_pass": _full(read)}


def poa_inputs(reads, poa, max_poa_coverage=None):
    """PoaConsensus (Consensus.h:352-390): feed the filtered reads to the POA in order (None -> key -1) until
    max_poa_coverage reads were added, then take the consensus with minCoverage = 1 below 5 reads, else
    (cov + 1) / 2 - 1.

    poa: an object with the SparsePoa surface -- orient_and_add_read(seq) -> key (>= 0, or -1 when the read
    could not be added) and find_consensus(min_coverage) -> (sequence, summaries by key).
    Returns (draft, read_keys, summaries)."""
    keys = []
    cov = 0
    for r in reads:
        key = -1 if r is None else poa.orient_and_add_read(r["seq"])
        keys.append(key)
        if key >= 0:
            cov += 1
            if max_poa_coverage is not None and cov >= max_poa_coverage:
                break
    min_cov = 1 if cov < 5 else (cov + 1) // 2 - 1
    draft, summaries = poa.find_consensus(min_cov)
    return draft, keys, summaries


def zmw_input(chunk, poa, min_length=10, max_poa_coverage=None):
    """One ZMW's subreads -> the polish boundary's ZMW dict, or (status, None) when the ZMW ends before the
    scorer: NoSubreads (Consensus.h:414-420) or TooShort (:427-434).

    chunk: {"snr": 4 floats, "reads": [{"seq", "flags"}]}.  Returns (None, zmw) on success, where zmw is
    {"draft", "snr", "reads"} and reads holds one entry per POA key in order: the mapped read, or a
    placeholder {"seq": None} for a read the POA or ExtractMappedRead skipped."""
    reads = filter_reads(chunk["reads"], min_length)
    if not reads or all(r is None for r in reads):
        return "NoSubreads", None
    draft, keys, summaries = poa_inputs(reads, poa, max_poa_coverage)
    if len(draft) < min_length:
        return "TooShort", None
    out = []
    for i, key in enumerate(keys):
        mr = extract_mapped_read(reads[i], summaries[key], min_length) if key >= 0 else None
        out.append(mr if mr is not None else {"seq": None, "strand": 0, "ts": 0, "te": 0, "full_pass": False})
    return None, {"draft": draft, "snr": list(chunk["snr"]), "reads": out}


def zmw_inputs_batch(chunks, min_length=10, max_poa_coverage=None, engine=None):
    """zmw_input for many ZMWs at once, with the POA of all of them on the GPU in one pbccs_poa_batch
    (every ZMW adds its next subread in the same device round).  Returns [(status, zmw)] as zmw_input."""
    from . import poa as _poa
    filtered = [filter_reads(c["reads"], min_length) for c in chunks]
    idx = [z for z, rs in enumerate(filtered) if rs and not all(r is None for r in rs)]
    out = [("NoSubreads", None)] * len(chunks)
    res = _poa.poa_batch([[None if r is None else r["seq"] for r in filtered[z]] for z in idx],
                         max_coverage=max_poa_coverage, engine=engine)
    for z, r in zip(idx, res):
        draft = r["consensus"]
        if len(draft) < min_length:
            out[z] = ("TooShort", None)
            continue
        reads = []
        for i, key in enumerate(r["keys"]):
            if key == -2:
                break   # past maxPoaCov: Consensus.h's loop stopped before this read
            mr = extract_mapped_read(filtered[z][i], r["summaries"][key], min_length) if key >= 0 else None
            reads.append(mr if mr is not None else {"seq": None, "strand": 0, "ts": 0, "te": 0, "full_pass": False})
        out[z] = (None, {"draft": draft, "snr": list(chunks[z]["snr"]), "reads": reads})
    return out


def ccs_batch(chunks, settings=None, engine=None, max_poa_coverage=None):
    """Consensus.h's per-ZMW driver for many ZMWs in one native call (pbccs_ccs_batch): FilterReads,
    the GPU POA, TooShort, ExtractMappedRead and the GPU polish, with no Python between the stages.
    chunks: [{"snr", "reads": [{"seq", "flags"?}]}].  Returns per ZMW the polish result dict (as
    polish_zmws) plus "draft"; add_read_results / zscores hold one entry per input subread, in the
    chunk's read order: -1 / NaN for a read that never reached AddRead (dropped by FilterReads, not added
    by the POA, rejected by ExtractMappedRead, past the maxPoaCov stop, or the ZMW ended earlier).
    "add_order" lists the subread indices in AddRead order (FilterReads' stable order, Consensus.h:281):
    the order of ZScores() and of the ccs.bam zs tag.
    Raises on a draft longer than its buffer (PBCCS_ERANGE).

    Marshalling is flat, as poa.poa_batch's: every subread in one buffer behind one pointer table, every
    output in shared arrays, the per-ZMW structs written column-wise through numpy views (per-ZMW ctypes
    arrays were ~3 s of Python per 10,000 ZMWs, half the ccs stage's wall time)."""
    import ctypes
    from . import ZMW_STATUS, default_engine
    from . import lib as L
    from .polish import ConsensusSettings
    from .quiver import _struct_dtype
    eng = engine or default_engine()
    settings = settings or ConsensusSettings()
    n = len(chunks)
    counts = np.fromiter((len(c["reads"]) for c in chunks), dtype=np.int64, count=n)
    flat = [r for c in chunks for r in c["reads"]]
    nr_all = len(flat)
    seqs = [r["seq"] for r in flat]
    joined = "".join(seqs).encode()   # one encode: per-read lengths in characters are bytes for ACGT text
    lens = np.fromiter(map(len, seqs), dtype=np.int32, count=nr_all)
    if len(joined) != int(lens.sum()):   # non-ASCII text: lengths in bytes, read by read
        enc = [s.encode() for s in seqs]
        joined = b"".join(enc)
        lens = np.fromiter(map(len, enc), dtype=np.int32, count=nr_all)
    flags = np.fromiter((int(r.get("flags", FULL_PASS)) for r in flat), dtype=np.uint8, count=nr_all)
    bases = np.zeros(nr_all + 1, dtype=np.int64)
    np.cumsum(lens, out=bases[1:])
    blob = np.frombuffer(joined, dtype=np.uint8) if joined else np.zeros(1, dtype=np.uint8)   # read-only view
    ptrs = (blob.ctypes.data + bases[:-1]).astype(np.uint64)
    first = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=first[1:])
    f0 = first[:-1]
    # a POA consensus never exceeds the bases of the reads it was built from: per-ZMW capacity read bases + 64
    caps = bases[first[1:]] - bases[f0] + 64
    cstart = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(caps, out=cstart[1:])
    cons = np.zeros(max(1, int(cstart[-1])), dtype=np.uint8)     # calloc'd: pages past a draft's length untouched
    draft = np.zeros(max(1, int(cstart[-1])), dtype=np.uint8)
    qv = np.zeros(max(1, int(cstart[-1])), dtype=np.int32)
    arr = np.zeros(max(1, nr_all), dtype=np.int32)
    zs = np.zeros(max(1, nr_all), dtype=np.float64)
    order = np.zeros(max(1, nr_all), dtype=np.int32)
    ins = np.zeros(max(1, n), dtype=_struct_dtype(L.CCcsInput))
    outs = np.zeros(max(1, n), dtype=_struct_dtype(L.CCcsOutput))
    if n:
        ins["snr"][:n] = np.array([[float(v) for v in c["snr"][:4]] for c in chunks], dtype=np.float64)
        ins["n_subreads"][:n] = counts
        ins["seqs"][:n] = ptrs.ctypes.data + 8 * f0
        ins["lens"][:n] = lens.ctypes.data + 4 * f0
        ins["flags"][:n] = flags.ctypes.data + f0
        pol = outs["polish"]
        pol["consensus"][:n] = cons.ctypes.data + cstart[:-1]
        pol["consensus_cap"][:n] = caps
        pol["qvs"][:n] = qv.ctypes.data + 4 * cstart[:-1]
        pol["add_read_results"][:n] = arr.ctypes.data + 4 * f0
        pol["zscores"][:n] = zs.ctypes.data + 8 * f0
        outs["draft"][:n] = draft.ctypes.data + cstart[:-1]
        outs["draft_cap"][:n] = caps
        outs["add_order"][:n] = order.ctypes.data + 4 * f0
    opts = settings._c()
    mc = 2**62 if max_poa_coverage is None else int(max_poa_coverage)
    L.check(L.load().pbccs_ccs_batch(eng._h, ctypes.cast(ins.ctypes.data, ctypes.POINTER(L.CCcsInput)), n, mc,
                                     ctypes.byref(opts), ctypes.cast(outs.ctypes.data, ctypes.POINTER(L.CCcsOutput))))
    del blob, joined, ptrs, lens, flags   # the inputs lived until the call returned
    pol = outs["polish"]
    status, clen = pol["status"][:n].tolist(), pol["consensus_len"][:n].tolist()
    zg, za, pacc = pol["zg"][:n].tolist(), pol["za"][:n].tolist(), pol["predicted_accuracy"][:n].tolist()
    ntest, nappl, npass = pol["n_tested"][:n].tolist(), pol["n_applied"][:n].tolist(), pol["n_passes"][:n].tolist()
    scounts, dlen = pol["status_counts"][:n].tolist(), outs["draft_len"][:n].tolist()
    cs, fs, cnt = cstart.tolist(), first.tolist(), counts.tolist()
    arr_l, zs_l, order_l = arr.tolist(), zs.tolist(), order.tolist()
    res = []
    for z in range(n):
        st, c, f, nr = status[z], cs[z], fs[z], cnt[z]
        ok = st in (0, 6)
        ln = max(0, clen[z]) if ok else 0
        res.append({"status": ZMW_STATUS[st], "status_code": st,
                    "consensus": cons[c:c + ln].tobytes().decode() if ok else "",
                    "qvs": qv[c:c + ln].tolist() if ok else [],
                    "draft": draft[c:c + max(0, dlen[z])].tobytes().decode(),
                    "add_read_results": arr_l[f:f + nr], "zscores": zs_l[f:f + nr],
                    "polished": st not in (1, 2),   # NoSubreads / TooShort end before the polish
                    "add_order": [k for k in order_l[f:f + nr] if k >= 0],
                    "zg": zg[z], "za": za[z], "predicted_accuracy": pacc[z], "n_tested": ntest[z],
                    "n_applied": nappl[z], "n_passes": npass[z], "status_counts": scounts[z]})
    return res
