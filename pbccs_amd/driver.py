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
    Raises on a draft longer than its buffer (PBCCS_ERANGE)."""
    import ctypes
    from . import ZMW_STATUS, default_engine
    from . import lib as L
    from .polish import ConsensusSettings
    eng = engine or default_engine()
    settings = settings or ConsensusSettings()
    n = len(chunks)
    ins = (L.CCcsInput * max(1, n))()
    outs = (L.CCcsOutput * max(1, n))()
    keep = []
    for z, c in enumerate(chunks):
        reads = c["reads"]
        nr = len(reads)
        enc = [r["seq"].encode() for r in reads]
        seqs = (ctypes.c_char_p * max(1, nr))(*enc)
        lens = (ctypes.c_int * max(1, nr))(*[len(e) for e in enc])
        flags = (ctypes.c_ubyte * max(1, nr))(*[int(r.get("flags", FULL_PASS)) for r in reads])
        # a POA consensus never exceeds the bases of the reads it was built from
        cap = sum(len(e) for e in enc) + 64
        cons, draft = ctypes.create_string_buffer(cap), ctypes.create_string_buffer(cap)
        qv = (ctypes.c_int * cap)()
        arr = (ctypes.c_int * max(1, nr))()
        zs = (ctypes.c_double * max(1, nr))()
        order = (ctypes.c_int * max(1, nr))()
        for k in range(4):
            ins[z].snr[k] = float(c["snr"][k])
        ins[z].n_subreads, ins[z].seqs, ins[z].lens, ins[z].flags = nr, seqs, lens, flags
        o = outs[z]
        o.polish.consensus = ctypes.cast(cons, ctypes.c_char_p)
        o.polish.consensus_cap = cap
        o.polish.qvs, o.polish.add_read_results, o.polish.zscores = qv, arr, zs
        o.draft = ctypes.cast(draft, ctypes.c_char_p)
        o.draft_cap = cap
        o.add_order = order
        keep.append((seqs, lens, flags, cons, draft, qv, arr, zs, order, nr))
    opts = settings._c()
    mc = 2**62 if max_poa_coverage is None else int(max_poa_coverage)
    L.check(L.load().pbccs_ccs_batch(eng._h, ins, n, mc, ctypes.byref(opts), outs))
    res = []
    for z, (_, _, _, cons, draft, qv, arr, zs, order, nr) in enumerate(keep):
        p = outs[z].polish
        ok = p.status in (0, 6)
        ln = max(0, p.consensus_len) if ok else 0
        polished = p.status not in (1, 2)   # NoSubreads / TooShort end before the polish
        res.append({"status": ZMW_STATUS[p.status], "status_code": p.status,
                    "consensus": cons.raw[:ln].decode() if ok else "", "qvs": list(qv[:ln]) if ok else [],
                    "draft": draft.raw[:max(0, outs[z].draft_len)].decode(),
                    "add_read_results": list(arr[:nr]), "zscores": list(zs[:nr]), "polished": polished,
                    "add_order": [k for k in order[:nr] if k >= 0],
                    "zg": p.zg, "za": p.za, "predicted_accuracy": p.predicted_accuracy, "n_tested": p.n_tested,
                    "n_applied": p.n_applied, "n_passes": p.n_passes, "status_counts": list(p.status_counts)})
    return res
