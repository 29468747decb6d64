"""GPU parity of the Quiver family (HIP engine through the C ABI) against the reference's Quiver gtest
known answers and against the CPU restatement (oracle/quiver_oracle.cpp) on seeded synthetic reads with
random QV features.  Tolerance: bit-exact FP32 (every score, baseline, flip-flop count and refine outcome), since
the engine repeats the SSE recursor's single-precision operations in order; ConsensusQVs equal to the
restatement's (see _qvs_exact) and equal between the batch and the per-scorer calls."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.test_quiver_oracle_pins import run_kat

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
KATS = json.load(open(os.path.join(GOLD, "quiver_kats.json")))


class GpuQuiver:
    """Adapter with the oracle's QuiverScorer call shape over pbccs_amd's QuiverMultiReadMutationScorer."""

    def __init__(self, tpl, params, moves=15, score_diff=12.5, fast_threshold=-12.5, add_threshold=1.0,
                 sum_product=False, recursor="SparseSse"):
        import pbccs_amd as P
        self.P = P
        qp = P.QvModelParams(**params)
        cfg = P.QuiverConfig(qp, moves=moves, score_diff=score_diff, fast_score_threshold=fast_threshold,
                             add_threshold=add_threshold, sum_product=sum_product, recursor=recursor)
        self.s = P.QuiverMultiReadMutationScorer(cfg, tpl)

    def add_read(self, seq, strand=0, ts=0, te=None, features=None, threshold=None):
        f = features or {}
        return self.s.AddRead(seq, strand, ts, te, ins_qv=f.get("ins"), subs_qv=f.get("subs"), del_qv=f.get("del"),
                              del_tag=f.get("del_tag"), merge_qv=f.get("merge"), threshold=threshold)

    def score(self, t, p, b="-", fast=False):
        return self.s.ScoreMany([self.P.Mutation(t, p, b)], fast=fast)[0]

    def read_score_mutation(self, r, t, p, b="-"):
        return self.s.ReadScoreMutation(r, self.P.Mutation(t, p, b))

    def baseline(self):
        return self.s.BaselineScore()

    def apply(self, muts):
        self.s.ApplyMutations([self.P.Mutation(t, p, b) for (t, p, b) in muts])

    def template(self):
        return self.s.Template()

    def alignment(self, r):
        return self.s.Alignment(r)


@pytest.mark.parametrize("idx", range(len(KATS["kats"])))
def test_quiver_kats_on_gpu(idx):
    run_kat(GpuQuiver, KATS["kats"][idx], KATS["params"])


PARAMS2 = dict(Match=-0.2, Mismatch=-8.0, MismatchS=-0.15, Branch=-3.5, BranchS=-0.12, DeletionN=-7.5,
               DeletionWithTag=-4.5, DeletionWithTagS=-0.2, Nce=-6.0, NceS=-0.1, Merge=[-3.0, -3.2, -2.9, -3.1],
               MergeS=[-0.1, -0.12, -0.09, -0.11])


def _features(rng, seq):
    n = len(seq)
    tags = rng.choice(list("ACGTN"), size=n)
    return {"ins": rng.integers(0, 25, n).tolist(), "subs": rng.integers(0, 25, n).tolist(),
            "del": rng.integers(0, 25, n).tolist(), "del_tag": tags.tolist(), "merge": rng.integers(0, 25, n).tolist()}


def _pair(tpl, reads, sum_product, score_diff=12.5, params=None):
    params = params or PARAMS2
    g = GpuQuiver(tpl, params, score_diff=score_diff, sum_product=sum_product)
    o = O.QuiverScorer(tpl, params, score_diff=score_diff, sum_product=sum_product)
    for r in reads:
        a = g.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"])
        b = o.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"])
        assert bool(a) == bool(b)
    return g, o


def _zmw(seed, length, passes):
    from pbccs_amd import synth
    z = synth.make_zmws(1, length, passes, seed=seed)[0]
    rng = np.random.default_rng(seed)
    reads = [dict(r, features=_features(rng, r["seq"])) for r in z["reads"]]
    return z["draft"], reads


def _qvs_exact(got, exp):
    """ConsensusQVs against the restatement, exactly (tighter than the north_star's +-1): the scores are
    bit-exact floats and k_qqv sums exp(score) per position with the device libm.  An ulp of exp / log10 moves
    prob = 1 - 1/(1 + sum) by at most err = 4 eps + 16 eps sum, so k_qqv leaves to the host (QuiverBatch::QVsMany,
    the host libm on the same float scores) every position whose -10 log10(prob) lies within 4.35 err / prob + 1e-6
    of a .5 rounding boundary, and every position where 1 + sum rounded to 1.0 although sum > 0.4 eps."""
    return list(got) == list(exp)


@pytest.mark.parametrize("sum_product", [False, True])
@pytest.mark.parametrize("seed,length,passes", [(101, 80, 3), (102, 200, 5)])
def test_quiver_scores_match_oracle(sum_product, seed, length, passes):
    tpl, reads = _zmw(seed, length, passes)
    g, o = _pair(tpl, reads, sum_product)
    assert g.s.BaselineScores() == [o.read_info(k)["score"] for k in range(len(reads)) if o.read_info(k)["active"]]
    # NumFlipFlops of a read whose scorer construction threw is undefined in the reference (null scorer)
    active = [k for k in range(len(reads)) if o.read_info(k)["active"]]
    assert [g.s.NumFlipFlops()[k] for k in active] == [o.read_info(k)["flipflops"] for k in active]
    assert [g.s.ReadInfo(k)["active"] for k in range(len(reads))] == [o.read_info(k)["active"] for k in range(len(reads))]
    muts = O.unique_mutations(tpl)
    vals = g.s.ScoreMany([g.P.Mutation(t, s, b) for (t, s, b) in muts])
    fast = g.s.ScoreMany([g.P.Mutation(t, s, b) for (t, s, b) in muts], fast=True)
    for (t, s, b), v, f in zip(muts, vals, fast):
        assert v == o.score(t, s, b), (t, s, b)
        assert f == o.score(t, s, b, fast=True), (t, s, b)


@pytest.mark.parametrize("sum_product", [False, True])
def test_quiver_refine_and_qvs_match_oracle(sum_product):
    tpl, reads = _zmw(111, 150, 5)
    g, o = _pair(tpl, reads, sum_product)
    import pbccs_amd as P
    conv, nt, na = P.RefineConsensus(g.s)
    ref = o.refine()
    assert (conv, nt, na) == (ref["converged"], ref["n_tested"], ref["n_applied"])
    assert g.template() == o.template()
    assert _qvs_exact(P.ConsensusQVs(g.s), o.qvs())


def test_quiver_qvs_host_path_matches_device_path(monkeypatch):
    """k_qqv leaves positions whose rounding could depend on the libm to the host; PBCCS_QQV_HOST=1 sends every
    position there: the QVs equal the device path's and the restatement's."""
    tpl, reads = _zmw(112, 160, 5)
    g, o = _pair(tpl, reads, True)
    import pbccs_amd as P
    dev = P.ConsensusQVs(g.s)
    monkeypatch.setenv("PBCCS_QQV_HOST", "1")
    host = P.ConsensusQVs(g.s)
    assert host == dev and _qvs_exact(host, o.qvs())


def test_quiver_add_threshold_memory_gate():
    """AddRead's AllocatedEntries gate (MultiReadMutationScorer.cpp:263-276) reproduces the oracle's
    libstdc++ capacity accounting."""
    tpl, reads = _zmw(121, 120, 4)
    g = GpuQuiver(tpl, PARAMS2, score_diff=12.5)
    o = O.QuiverScorer(tpl, PARAMS2, score_diff=12.5)
    for r in reads:
        for thr in (0.05, 0.2):
            a = g.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"], threshold=thr)
            b = o.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"], threshold=thr)
            assert bool(a) == bool(b), (thr, a, b)
    for k in range(g.s.NumReads()):
        info = o.read_info(k)
        if info["active"]:
            assert g.s.AllocatedEntries(k) == info["allocated"]


@pytest.mark.parametrize("seed,length,passes,moves", [(111, 60, 3, 15), (112, 300, 4, 15), (113, 500, 3, 7)])
def test_quiver_alignment_matches_oracle(seed, length, passes, moves):
    """RecursorFuzzTest.Alignment (TestRecursors.cpp:351-366) against the restatement: the Viterbi traceback
    of every read (both strands, banded, merges on/off) is the same gapped Target / Query pair."""
    tpl, reads = _zmw(seed, length, passes)
    g = GpuQuiver(tpl, PARAMS2, moves=moves)
    o = O.QuiverScorer(tpl, PARAMS2, moves=moves)
    for k, r in enumerate(reads):
        a = g.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"])
        b = o.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"])
        assert bool(a) == bool(b)
        if a:
            t, q = g.alignment(k)
            assert (t, q) == o.alignment(k)
            L = len(tpl)
            window = tpl[r["ts"]:r["te"]] if r["strand"] == 0 else \
                tpl[::-1].translate(str.maketrans("ACGT", "TGCA"))[L - r["te"]:L - r["ts"]]
            assert len(t) == len(q) and t.replace("-", "") == window and q.replace("-", "") == r["seq"]


def test_quiver_alignment_sum_product_refused():
    """Alignment is Viterbi-only (RecursorBase.cpp:128-131 ShouldNotReachHere): the ABI refuses it."""
    from pbccs_amd.lib import PbccsError
    tpl, reads = _zmw(114, 60, 2)
    g = GpuQuiver(tpl, PARAMS2, sum_product=True)
    g.add_read(reads[0]["seq"], reads[0]["strand"], reads[0]["ts"], reads[0]["te"], reads[0]["features"])
    with pytest.raises(PbccsError):
        g.alignment(0)


@pytest.mark.parametrize("recursor", ["SparseSimple", "DenseSse", "DenseSimple"])
def test_quiver_kats_all_recursor_types(recursor):
    """ConsensusCore's typed Quiver tests run every recursor type (TestRecursors.cpp:63-66,
    TestMutationScorer.cpp:59-62) against the same expectations: replay every KAT with each."""
    for k in KATS["kats"]:
        run_kat(lambda tpl, params, **kw: GpuQuiver(tpl, params, recursor=recursor, **kw), k, KATS["params"])


@pytest.mark.parametrize("recursor", ["SparseSimple", "DenseSse", "DenseSimple"])
@pytest.mark.parametrize("sum_product", [False, True])
def test_quiver_recursor_types_match_oracle(recursor, sum_product):
    """Simple / dense recursors against the restatement: baseline scores, flip-flops, every unique mutation's
    score, AllocatedEntries (dense: Rows * Columns) and -- Viterbi -- every read's alignment."""
    tpl, reads = _zmw(121, 150, 4)
    g = GpuQuiver(tpl, PARAMS2, sum_product=sum_product, recursor=recursor)
    o = O.QuiverScorer(tpl, PARAMS2, sum_product=sum_product, recursor=recursor)
    for r in reads:
        assert bool(g.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"])) == \
            bool(o.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"]))
    active = [k for k in range(len(reads)) if o.read_info(k)["active"]]
    assert g.s.BaselineScores() == [o.read_info(k)["score"] for k in active]
    assert [g.s.NumFlipFlops()[k] for k in active] == [o.read_info(k)["flipflops"] for k in active]
    for k in active:
        ga, gb = g.s.AllocatedEntries(k)
        info = o.read_info(k)
        assert (ga, gb) == info["allocated"]
        if recursor.startswith("Dense"):
            assert ga == (len(reads[k]["seq"]) + 1) * (reads[k]["te"] - reads[k]["ts"] + 1)
        if not sum_product:
            assert g.alignment(k) == o.alignment(k)
    muts = O.unique_mutations(tpl)
    vals = g.s.ScoreMany([g.P.Mutation(t, s, b) for (t, s, b) in muts])
    for (t, s, b), v in zip(muts, vals):
        assert v == o.score(t, s, b), (t, s, b)


@pytest.mark.parametrize("sum_product", [False, True])
def test_quiver_polish_batch_matches_scorers(sum_product):
    """pbccs_quiver_polish_batch (every scorer's rounds in lock-step: batched fills, device Score /
    FastIsFavorable reduction and BestSubset) equals the per-scorer call sequence -- AddRead, RefineConsensus,
    ConsensusQVs -- ZMW for ZMW, and the oracle on the first ZMWs; one ZMW has a read AddRead drops."""
    import pbccs_amd as P
    from pbccs_amd import quiver
    zs = []
    for k, (length, passes) in enumerate([(120, 4), (200, 5), (90, 3), (160, 6), (60, 2)]):
        tpl, reads = _zmw(200 + k, length, passes)
        zs.append({"tpl": tpl, "reads": reads})
    zs[2]["reads"][0] = dict(zs[2]["reads"][0], threshold=0.001)   # the memory gate drops it
    cfg = P.QuiverConfig(P.QvModelParams(**PARAMS2), sum_product=sum_product)
    got = quiver.polish_batch(zs, cfg)
    for z, g in zip(zs, got):
        s = P.QuiverMultiReadMutationScorer(cfg, z["tpl"])
        na = 0
        for r in z["reads"]:
            f = r["features"]
            na += s.AddRead(r["seq"], r["strand"], r["ts"], r["te"], ins_qv=f["ins"], subs_qv=f["subs"],
                            del_qv=f["del"], del_tag=f["del_tag"], merge_qv=f["merge"], threshold=r.get("threshold"))
        conv, nt, nap = P.RefineConsensus(s)
        assert g["ok"] and g["n_active"] == na
        assert (g["converged"], g["n_tested"], g["n_applied"]) == (conv, nt, nap)
        assert g["consensus"] == s.Template()
        assert g["qvs"] == P.ConsensusQVs(s)
    for z, g in list(zip(zs, got))[:2]:
        tpl, reads = z["tpl"], z["reads"]
        o = O.QuiverScorer(tpl, PARAMS2, sum_product=sum_product)
        for r in reads:
            o.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"])
        ref = o.refine()
        assert (g["converged"], g["n_tested"], g["n_applied"]) == (ref["converged"], ref["n_tested"], ref["n_applied"])
        assert g["consensus"] == o.template()
        assert _qvs_exact(g["qvs"], o.qvs())


def test_quiver_coop_fill_long_reads_match_oracle():
    """k_qfill_coop (one wavefront per read) at configs[1]-like sizes: 1.5 kb reads whose bands span several
    64-row chunks, ScoreDiff 18 -- active flags, baseline scores, flip-flop counts and AllocatedEntries
    equal the oracle's; then the batch polish of those ZMWs equals the oracle's refine and QVs."""
    import pbccs_amd as P
    from pbccs_amd import quiver, synth
    zs = synth.make_quiver_zmws(2, 1500, 6, seed=7)
    cfg = P.QuiverConfig(P.QvModelParams(**synth.QUIVER_PARAMS), score_diff=synth.QUIVER_SCORE_DIFF)
    for z in zs:
        g = P.QuiverMultiReadMutationScorer(cfg, z["tpl"])
        o = O.QuiverScorer(z["tpl"], synth.QUIVER_PARAMS, score_diff=synth.QUIVER_SCORE_DIFF)
        for r in z["reads"]:
            f = r["features"]
            a = g.AddRead(r["seq"], r["strand"], r["ts"], r["te"], ins_qv=f["ins"], subs_qv=f["subs"], del_qv=f["del"],
                          del_tag=f["del_tag"], merge_qv=f["merge"])
            b = o.add_read(r["seq"], r["strand"], r["ts"], r["te"], f)
            assert bool(a) == bool(b)
        act = [k for k in range(len(z["reads"])) if o.read_info(k)["active"]]
        assert len(act) >= 4
        assert g.BaselineScores() == [o.read_info(k)["score"] for k in act]
        assert [g.NumFlipFlops()[k] for k in act] == [o.read_info(k)["flipflops"] for k in act]
        assert [g.AllocatedEntries(k) for k in act] == [tuple(o.read_info(k)["allocated"]) for k in act]
    got = quiver.polish_batch(zs, cfg)
    for z, r in zip(zs, got):
        o = O.QuiverScorer(z["tpl"], synth.QUIVER_PARAMS, score_diff=synth.QUIVER_SCORE_DIFF)
        for rd in z["reads"]:
            o.add_read(rd["seq"], rd["strand"], rd["ts"], rd["te"], rd["features"])
        ref = o.refine()
        assert (r["converged"], r["n_tested"], r["n_applied"]) == (ref["converged"], ref["n_tested"], ref["n_applied"])
        assert r["consensus"] == o.template()
        assert _qvs_exact(r["qvs"], o.qvs())


@pytest.mark.parametrize("score_diff,sum_product", [(60.0, False), (60.0, True), (400.0, False)])
def test_quiver_tall_band_fill_paths_match_oracle(score_diff, sum_product):
    """Wide bands send reads down every SparseSse fill path: at ScoreDiff 60 (~26 rows per column) some columns
    outgrow k_qfill_grp's 64-row ring (kQTall -> k_qfill_coop), at ScoreDiff 400 (~137 rows) most outgrow the
    coop kernel's 128-row ring too (-> its full-height ring).  Active flags, baselines, flip-flops,
    AllocatedEntries and every unique mutation's score equal the oracle's."""
    tpl, reads = _zmw(321, 300, 3)
    g, o = _pair(tpl, reads, sum_product, score_diff=score_diff)
    act = [k for k in range(len(reads)) if o.read_info(k)["active"]]
    assert len(act) == len(reads)
    assert g.s.BaselineScores() == [o.read_info(k)["score"] for k in act]
    assert [g.s.NumFlipFlops()[k] for k in act] == [o.read_info(k)["flipflops"] for k in act]
    assert [g.s.AllocatedEntries(k) for k in act] == [tuple(o.read_info(k)["allocated"]) for k in act]
    muts = O.unique_mutations(tpl)
    vals = g.s.ScoreMany([g.P.Mutation(t, s, b) for (t, s, b) in muts])
    for (t, s, b), v in zip(muts, vals):
        assert v == o.score(t, s, b), (t, s, b)


@pytest.mark.parametrize("pins", [(True, True), (False, False)])
def test_qv_evaluator_python_mirror_matches_oracle(pins):
    """pbccs_amd.QvEvaluator (the Python mirror of QvEvaluator.hpp:90-317 over pbccs_qv_evaluator_moves): every
    cell's Inc / Del / Extra / Merge equals the oracle's evaluator, NaN outside each move's domain."""
    import math
    import pbccs_amd as P
    rng = np.random.default_rng(5)
    tpl = "".join(rng.choice(list("ACGT"), size=30)) + "CCCAAA"
    seq = tpl[2:20] + "AAA" + tpl[21:34]
    f = _features(rng, seq)
    feats = P.QvSequenceFeatures(seq, f["ins"], f["subs"], f["del"], f["del_tag"], f["merge"])
    ev = P.QvEvaluator(feats, tpl, P.QvModelParams(**PARAMS2), pin_start=pins[0], pin_end=pins[1])
    cells = [(i, j) for i in range(-1, len(seq) + 2) for j in range(-1, len(tpl) + 2)]
    got = ev.Moves(cells)
    exp = O.qv_eval_moves(seq, tpl, PARAMS2, cells, f, pin_start=pins[0], pin_end=pins[1])
    for k in range(4):
        for a, b in zip(got[k], exp[k]):
            assert (math.isnan(a) and math.isnan(b)) or a == b
    assert ev.Inc(0, 0) == exp[0][cells.index((0, 0))] and ev.ReadLength() == len(seq)


def test_quiver_alignment_leaves_the_bands_intact():
    """RecursorBase::Alignment is a read-only walk of the alpha band: asking twice gives the same alignment, and
    the scores after it are unchanged (the move count once landed in the bands' column-offset array)."""
    k = KATS["kats"][0]
    g = GpuQuiver(k["tpl"], KATS["params"], moves=k["moves"], score_diff=k["score_diff"],
                  fast_threshold=k["fast_threshold"])
    g.add_read(k["reads"][0]["seq"], 0, 0, len(k["tpl"]))
    first = g.alignment(0)
    assert first == ("GATG", "GATG")
    assert g.alignment(0) == first and g.alignment(0) == first
    tpl, reads = _zmw(131, 120, 4)
    g, o = _pair(tpl, reads, False)
    muts = O.unique_mutations(tpl)[:200]
    before = g.s.ScoreMany([g.P.Mutation(t, s, b) for (t, s, b) in muts])
    for r in range(g.s.NumReads()):
        if g.s.ReadInfo(r)["active"]:
            assert g.alignment(r) == g.alignment(r) == o.alignment(r)
    assert g.s.ScoreMany([g.P.Mutation(t, s, b) for (t, s, b) in muts]) == before
