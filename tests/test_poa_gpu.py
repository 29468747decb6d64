"""POA draft step on the GPU (pbccs_amd.poa over pbccs_poa_* / pbccs_sparse_poa_*) against the reference's own
POA tests (tests/golden/poa_kats.json, parsed from ConsensusCore/src/Tests/TestPoaConsensus.cpp and
tests/TestSparsePoa.cpp) and against the CPU restatement (oracle/poa_oracle.cpp) on seeded synthetic ZMWs.
Bar: bit-exact (consensus strings, read keys, orientations, extents, graph dumps)."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "poa_kats.json")))


@pytest.fixture(scope="module")
def P():
    import pbccs_amd
    from pbccs_amd import poa
    eng = pbccs_amd.Engine(0)
    poa.poa_stats(eng, reset=True)
    return poa, eng


def _rc(s):
    return s[::-1].translate(str.maketrans("ACGT", "TGCA"))


@pytest.mark.parametrize("case", GOLD["poa_consensus"], ids=lambda c: c["test"])
def test_poa_consensus_kats(P, case):
    poa, eng = P
    mc = case["min_coverage"] if case["min_coverage"] is not None else -poa.INT_MAX
    seq, dot = poa.poa_consensus(case["reads"], case["mode"], mc, graphviz_flags=case["graphviz_flags"], engine=eng)
    if case["expected"] is not None:
        assert seq == case["expected"]
    if case["expected_dot"]:
        assert dot.replace("\n", "") == case["expected_dot"]
    exp_seq, exp_dot = O.poa_consensus(case["reads"], case["mode"], mc, graphviz_flags=case["graphviz_flags"])
    assert (seq, dot) == (exp_seq, exp_dot)


def _sparse(name):
    return next(c for c in GOLD["sparse_poa"] if c["test"] == name)


@pytest.mark.parametrize("name", ["SparsePoaTest.TestLocalStaggered", "SparsePoaTest.TestOrientation"])
def test_sparse_poa_kats(P, name):
    poa, eng = P
    case = _sparse(name)
    sp = poa.SparsePoa(eng)
    keys = [sp.OrientAndAddRead(r) for r in case["reads"]]
    assert all(k >= 0 for k in keys)
    css, summ = sp.FindConsensus(case["min_coverage"])
    assert css == case["expected"]
    for k, exp in case["summaries"].items():
        s = summ[int(k)]
        if "rc" in exp:
            assert s["rc"] == exp["rc"]
        if "read" in exp:
            assert list(s["read"]) == exp["read"] and list(s["tpl"]) == exp["tpl"]
    # the batched form agrees
    b = poa.poa_batch([case["reads"]], min_coverage=case["min_coverage"], engine=eng)[0]
    assert b["consensus"] == css and b["summaries"] == summ


def test_sparse_poa_zmw6251(P):
    poa, eng = P
    case = _sparse("SparsePoaTest.TestZmw6251")
    sp = poa.SparsePoa(eng)
    assert all(sp.OrientAndAddRead(r) >= 0 for r in case["reads"])
    css, summ = sp.FindConsensus(case["min_coverage"])
    assert len(summ) == case["num_reads"]
    for k, exp in case["summaries"].items():
        assert summ[int(k)]["rc"] == exp["rc"]
    for k, (lo, hi) in case["covers"].items():
        b, e = summ[int(k)]["tpl"]
        assert b <= lo and hi <= e
    exp = O.sparse_poa(case["reads"], case["min_coverage"])
    assert css == exp["consensus"] and summ == exp["summaries"]
    dot = sp.ToGraphViz(3, case["min_coverage"])
    assert dot.startswith("digraph G {") and dot.count("->") > 1000


def test_sparse_poa_single_read_x100(P):
    """SparsePoaTest.SingleReadx100: 100 seeded 2-20 kb reads, one per graph (batched as 100 ZMWs)."""
    poa, eng = P
    seqs = O.poa_kat_reads(0)
    res = poa.poa_batch([[s] for s in seqs], min_coverage=1, engine=eng)
    for s, r in zip(seqs, res):
        assert r["consensus"] == s and r["keys"] == [0]
        assert r["summaries"] == [{"rc": False, "read": (0, len(s)), "tpl": (0, len(s))}]


def test_sparse_poa_single_and_half_x100(P):
    """SparsePoaTest.SingleAndHalfx100: a 1-5 kb read and the first third of its reverse complement."""
    poa, eng = P
    seqs = O.poa_kat_reads(1)
    res = poa.poa_batch([[s, _rc(s)[:len(s) // 3]] for s in seqs], min_coverage=1, engine=eng)
    for s, r in zip(seqs, res):
        L = len(s)
        assert r["consensus"] == s and r["keys"] == [0, 1]
        assert r["summaries"][0] == {"rc": False, "read": (0, L), "tpl": (0, L)}
        assert r["summaries"][1] == {"rc": True, "read": (0, L // 3), "tpl": (L - L // 3, L)}


def _synthetic_subreads(n, length_range, passes_range, seed):
    from pbccs_amd import synth
    zs = synth.make_zmws(n, None, None, seed=seed, length_range=length_range, passes_range=passes_range)
    return [[r["seq"] for r in z["reads"]] for z in zs]


def test_poa_batch_matches_oracle_synthetic(P):
    """Seeded ZMWs of 200-1500 bp with 2-12 passes; dropped reads (None) and a maxPoaCov stop included."""
    poa, eng = P
    zr = _synthetic_subreads(24, (200, 1500), (2, 12), seed=71)
    rng = np.random.default_rng(5)
    for reads in zr[:6]:
        reads[int(rng.integers(0, len(reads)))] = None
    res = poa.poa_batch(zr, max_coverage=None, engine=eng)
    for reads, got in zip(zr, res):
        exp = O.sparse_poa(reads)
        assert got["consensus"] == exp["consensus"]
        assert got["keys"] == exp["keys"] and got["summaries"] == exp["summaries"]
    res = poa.poa_batch(zr[:8], max_coverage=3, engine=eng)
    for reads, got in zip(zr[:8], res):
        exp = O.sparse_poa(reads, max_coverage=3)
        assert got["consensus"] == exp["consensus"] and got["keys"] == exp["keys"]
        assert got["summaries"] == exp["summaries"]


def test_poa_batch_matches_oracle_2kb(P):
    """configs[1] shape: 2 kb insert, 10 passes (alternate passes reverse-complemented)."""
    poa, eng = P
    zr = _synthetic_subreads(4, (2000, 2000), (10, 10), seed=1)
    res = poa.poa_batch(zr, engine=eng)
    for reads, got in zip(zr, res):
        exp = O.sparse_poa(reads)
        assert got["consensus"] == exp["consensus"] and got["summaries"] == exp["summaries"]
        assert [s["rc"] for s in got["summaries"]] == [False, True] * 5


def test_poa_wide_scores_long_reads(P):
    """Reads past 21.5 kb store int32 scores (3 * rows no longer fits uint16): a 21.6 kb, 2-pass ZMW, and
    GLOBAL / SEMIGLOBAL graphs (always int32) over several 1024-row chunks."""
    poa, eng = P
    zr = _synthetic_subreads(1, (21600, 21600), (2, 2), seed=9)
    got = poa.poa_batch(zr, engine=eng)[0]
    exp = O.sparse_poa(zr[0])
    assert got["consensus"] == exp["consensus"] and got["summaries"] == exp["summaries"]
    reads = _synthetic_subreads(1, (1500, 1500), (4, 4), seed=10)[0]
    reads = [r if k % 2 == 0 else _rc(r) for k, r in enumerate(reads)]   # one orientation for GLOBAL
    for mode in (O.POA_GLOBAL, O.POA_SEMIGLOBAL, O.POA_LOCAL):
        assert poa.poa_consensus(reads, mode, 2, graphviz_flags=3, engine=eng) == \
            O.poa_consensus(reads, mode, 2, graphviz_flags=3)


class _OraclePoa:
    """The oracle's SparsePoa behind driver.zmw_input's POA interface (reads added one at a time)."""
    def __init__(self):
        self.reads = []

    def orient_and_add_read(self, seq):
        self.reads.append(seq)
        return O.sparse_poa(self.reads)["keys"][-1]

    def find_consensus(self, min_cov):
        r = O.sparse_poa(self.reads, min_cov)
        return r["consensus"], dict(enumerate(r["summaries"]))


def test_driver_zmw_input_with_gpu_poa(P):
    """driver.zmw_input (FilterReads -> POA -> ExtractMappedRead) with the GPU SparsePoa equals the same
    driver with the oracle's POA."""
    poa, eng = P
    from pbccs_amd import driver

    for reads in _synthetic_subreads(3, (400, 900), (5, 9), seed=33):
        chunk = {"snr": [10.0, 7.0, 5.0, 11.0], "reads": [{"seq": s} for s in reads]}
        st_g, z_g = driver.zmw_input(chunk, poa.SparsePoa(eng))
        st_o, z_o = driver.zmw_input(chunk, _OraclePoa())
        assert st_g == st_o and z_g == z_o


def test_driver_batch_matches_per_zmw_driver(P):
    """driver.zmw_inputs_batch (one pbccs_poa_batch for all ZMWs) equals zmw_input per ZMW with the oracle's
    POA, with and without a maxPoaCov stop; a ZMW whose reads all fail FilterReads is NoSubreads."""
    poa, eng = P
    from pbccs_amd import driver

    chunks = [{"snr": [10.0, 7.0, 5.0, 11.0], "reads": [{"seq": s} for s in reads]}
              for reads in _synthetic_subreads(5, (300, 700), (3, 8), seed=44)]
    chunks.append({"snr": [8.0, 8.0, 8.0, 8.0], "reads": [{"seq": "ACGT"}]})   # median below min_length
    for cov in (None, 3):
        got = driver.zmw_inputs_batch(chunks, max_poa_coverage=cov, engine=eng)
        for c, g in zip(chunks, got):
            assert g == driver.zmw_input(c, _OraclePoa(), max_poa_coverage=cov)
    assert got[-1] == ("NoSubreads", None)


def _ccs_chunks():
    """Six synthetic ZMWs with partial passes (flags), zero-length subreads and a ZMW with no usable subread."""
    rng = np.random.default_rng(8)
    chunks = []
    for reads in _synthetic_subreads(6, (300, 900), (3, 9), seed=55):
        chunks.append({"snr": [10.0, 7.0, 5.0, 11.0],
                       "reads": [{"seq": s, "flags": int(rng.choice([3, 3, 3, 1, 2]))} for s in reads]})
    chunks.append({"snr": [9.0, 9.0, 9.0, 9.0], "reads": [{"seq": "ACGTA"}]})
    # zero-length subreads, first and later in the input: they count in FilterReads but the POA never adds them
    chunks[0]["reads"].insert(0, {"seq": ""})
    chunks[1]["reads"].insert(2, {"seq": "", "flags": 3})
    return chunks


def test_native_ccs_batch_matches_python_driver(P):
    """pbccs_ccs_batch (FilterReads, POA, ExtractMappedRead, polish in one native call) equals the Python
    driver (zmw_inputs_batch) followed by polish_zmws: statuses, drafts, consensus, QVs, per-key AddRead
    results and counts.  Includes partial passes (flags) and a ZMW with no usable subread."""
    poa, eng = P
    chunks = _ccs_chunks()
    for cov in (None, 3):
        _check_native_ccs(chunks, cov, eng)


def test_poa_drafts_after_pool_release_match_oracle(P):
    """pbccs_ccs_batch unmaps the POA score pools when it ends; the next POA maps them again.  Mapping new
    memory at the addresses just unmapped gave wrong drafts in later POA calls (VmPool::unmap_all now moves
    to a fresh address range).  Drafts from zmw_inputs_batch after each of several ccs calls equal the
    oracle's SparsePoa."""
    poa, eng = P
    from pbccs_amd import driver
    chunks = _ccs_chunks()
    want = {cov: [driver.zmw_input(c, _OraclePoa(), max_poa_coverage=cov) for c in chunks] for cov in (None, 3)}
    for _ in range(2):
        for cov in (None, 3):
            driver.ccs_batch(chunks, engine=eng, max_poa_coverage=cov)
            assert driver.zmw_inputs_batch(chunks, max_poa_coverage=cov, engine=eng) == want[cov]


def _check_native_ccs(chunks, cov, eng):
    """pbccs_ccs_batch against the Python driver + polish_zmws, per-read outputs in subread order."""
    import math
    import pbccs_amd
    from pbccs_amd import ccsio, driver
    native = driver.ccs_batch(chunks, engine=eng, max_poa_coverage=cov)
    ins = driver.zmw_inputs_batch(chunks, max_poa_coverage=cov, engine=eng)
    pol = iter(pbccs_amd.polish_zmws([z for st, z in ins if st is None], engine=eng))
    for c, (st, z), got in zip(chunks, ins, native):
        nr = len(c["reads"])
        assert len(got["add_read_results"]) == nr and len(got["zscores"]) == nr
        if st is not None:
            assert got["status"] == st
            assert got["add_read_results"] == [-1] * nr and all(math.isnan(v) for v in got["zscores"])
            continue
        exp = next(pol)
        assert got["draft"] == z["draft"]
        for k in ("status", "consensus", "qvs", "n_tested", "n_applied", "n_passes", "status_counts"):
            assert got[k] == exp[k], k
        # polish input position i is FilterReads' i-th read; map it back to the subread's input index
        order = [next(j for j, x in enumerate(c["reads"]) if x is r)
                 for r in driver.filter_reads(c["reads"], 10) if r is not None]
        want_arr, want_z = [-1] * nr, [float("nan")] * nr
        for i, (a, zz) in enumerate(zip(exp["add_read_results"], exp["zscores"])):
            want_arr[order[i]], want_z[order[i]] = a, zz
        assert got["add_read_results"] == want_arr
        for a, b in zip(got["zscores"], want_z):
            assert (math.isnan(a) and math.isnan(b)) or a == b
        # AddRead order (FilterReads' stable order): the ccs.bam zs tag of the native record equals the one of
        # the polish_zmws record, whose per-read arrays are in AddRead order already
        assert got["add_order"] == [order[i] for i, a in enumerate(exp["add_read_results"]) if a >= 0]
        if got["status"] == "Success":
            tag = lambda rec: [t for t in rec.split("\t") if t.startswith("zs:")]
            assert tag(ccsio.ccs_sam_record("m", 1, got, c["snr"])) == tag(ccsio.ccs_sam_record("m", 1, exp, c["snr"]))
        if cov is not None:
            assert sum(1 for a in got["add_read_results"] if a >= 0) <= cov
    assert native[-1]["status"] == "NoSubreads"


def test_native_ccs_batch_pipelined_chunks(P):
    """The pipelined form: ZMWs drafted in chunks of 3 (zmws_per_batch) while earlier chunks polish on the
    workspace slots; the results equal the one-chunk call's, ZMW for ZMW."""
    poa, eng = P
    from pbccs_amd import driver
    from pbccs_amd.polish import ConsensusSettings
    chunks = [{"snr": [10.0, 7.0, 5.0, 11.0], "reads": [{"seq": s} for s in reads]}
              for reads in _synthetic_subreads(11, (200, 600), (3, 7), seed=66)]
    chunks.insert(4, {"snr": [9.0, 9.0, 9.0, 9.0], "reads": [{"seq": "ACG"}]})
    one = driver.ccs_batch(chunks, engine=eng)
    many = driver.ccs_batch(chunks, ConsensusSettings(zmws_per_batch=3), engine=eng)
    assert json.dumps(many) == json.dumps(one)   # NaN z-scores (reads never added) compare equal as text
    assert one[4]["status"] == "NoSubreads"
    # the last chunk's polish cut into one piece per slot (PBCCS_CCS_TAIL_PIECE: pieces of 2 ZMWs here)
    import pbccs_amd
    os.environ["PBCCS_CCS_TAIL_PIECE"] = "2"
    try:
        e3 = pbccs_amd.Engine(0)
        e3.set_concurrency(3)
        pieces = driver.ccs_batch(chunks, ConsensusSettings(zmws_per_batch=5), engine=e3)
    finally:
        del os.environ["PBCCS_CCS_TAIL_PIECE"]
    assert json.dumps(pieces) == json.dumps(one)


def test_poa_stats_counted(P):
    poa, eng = P
    s = poa.poa_stats(eng)
    assert s["alignments"] > 0 and s["cells"] > 0 and s["trace_steps"] > 0
