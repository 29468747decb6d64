"""GPU parity: the HIP engine (through the C ABI) against the CPU restatement (oracle/) and the
reference's own known answers.

Tolerances (north_star): consensus / applied mutations / nTested / nApplied / AddReadResult bit-exact;
per-mutation and per-read log-likelihoods within 1e-9 relative here (the engine repeats the reference's
FP64 operation order; only device `log` may differ by an ulp); QVs within +-1.
"""
import json
import math
import os

import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
SNR = [10.0, 7.0, 5.0, 11.0]


def _close(a, b, rel=1e-9, abs_=1e-9):
    if math.isinf(a) or math.isinf(b) or math.isnan(a) or math.isnan(b):
        return (math.isnan(a) and math.isnan(b)) or a == b
    return abs(a - b) <= abs_ + rel * max(abs(a), abs(b))


@pytest.fixture(scope="module")
def P():
    import pbccs_amd
    return pbccs_amd


def _scorers(P, tpl, reads, snr=SNR, threshold=float("nan")):
    g = P.ArrowMultiReadMutationScorer(P.ArrowConfig(snr), tpl)
    o = O.Scorer(tpl, snr)
    rg, ro = [], []
    for r in reads:
        seq, strand, ts, te = r["seq"], r.get("strand", 0), r.get("ts", 0), r.get("te", len(tpl))
        rg.append(g.AddRead(seq, strand, ts, te, threshold))
        ro.append(o.add_read(seq, strand, ts, te, threshold))
    return g, o, rg, ro


def test_matrixtester_kats_on_gpu(P):
    k = json.load(open(os.path.join(GOLD, "arrow_kats.json")))
    for b in k["baseline"]:
        g = P.ArrowMultiReadMutationScorer(P.ArrowConfig(k["snr"]), b["tpl"])
        for r in b["reads"]:
            g.AddRead(r)
        assert abs(1 - g.BaselineScore() / b["expected"]) < k["tolerance_rel"]
    for m in k["mutations"]:
        g = P.ArrowMultiReadMutationScorer(P.ArrowConfig(k["snr"]), m["tpl"])
        for r in m["reads"] * m.get("copies", 1):
            g.AddRead(r)
        v = g.Score(P.Mutation(m["type"], m["start"], m["base"])) / m.get("divide_by", 1)
        assert abs(1 - v / m["expected"]) < k["tolerance_rel"], (m["line"], v)
    se = k["short_equalities"]
    a = P.ArrowMultiReadMutationScorer(P.ArrowConfig(k["snr"]), se["tpl_short"])
    a.AddRead(se["read"])
    b = P.ArrowMultiReadMutationScorer(P.ArrowConfig(k["snr"]), se["tpl_long"])
    b.AddRead(se["read"])
    mL = P.Mutation(se["type"], se["start"])
    assert abs(1 - a.BaselineScore() / (b.BaselineScore() + b.Score(mL))) < 1e-5
    b.ApplyMutations([mL])
    assert b.Template() == se["tpl_short"]
    assert abs(1 - a.BaselineScore() / b.BaselineScore()) < 1e-5


@pytest.mark.parametrize("seed,length,passes", [(11, 60, 3), (12, 150, 4), (13, 400, 6)])
def test_every_mutation_score_matches_oracle(P, seed, length, passes):
    from pbccs_amd import synth
    z = synth.make_zmws(1, length, passes, seed=seed)[0]
    g, o, rg, ro = _scorers(P, z["draft"], z["reads"])
    assert rg == ro
    ll_g = g.BaselineScores()
    for r in range(len(z["reads"])):
        assert _close(ll_g[r], o.read_info(r)["ll"]), r   # per-read LL (north_star: 1e-4 relative; asserted tighter)
    assert _close(g.BaselineScore(), o.baseline())
    muts = O.unique_mutations(z["draft"])
    gm = [P.Mutation(t, s, b) for (t, s, b) in muts]
    full = g.ScoreMany(gm)
    fast = g.ScoreMany(gm, -12.5)
    for (t, s, b), vf, vq in zip(muts, full, fast):
        assert _close(vf, o.score(t, s, b)), (t, s, b)
        assert _close(vq, o.score(t, s, b, -12.5)), (t, s, b)


@pytest.mark.parametrize("threshold", [1.0, float("nan")])
def test_matrixtester_multiread_zmw_matches_oracle(P, threshold):
    """MatrixTester.cpp:212-384 -- the reference's only real multi-read ZMW (54 subreads, real SNRs, non-spanning
    windows on both strands; tests/golden/matrixtester_multiread.json).  At the demo's AddRead threshold 1.0 (the
    z-score gate keeps 5 reads; the refine ends NonConvergent on an end-of-template oscillation) and with the gate off
    (all 54 reads): AddRead results, per-read LLs, z-scores, every unique mutation's full and fast score, the demo's
    Score(INSERTION 202 'C'), RefineConsensus (converged, nTested, nApplied, template) and ConsensusQVs."""
    d = json.load(open(os.path.join(GOLD, "matrixtester_multiread.json")))
    tpl, snr = d["tpl"], d["snr"]
    g = P.ArrowMultiReadMutationScorer(P.ArrowConfig(snr), tpl)
    o = O.Scorer(tpl, snr)
    rg = [g.AddRead(r["seq"], r["strand"], r["ts"], r["te"], threshold) for r in d["reads"]]
    ro = [o.add_read(r["seq"], r["strand"], r["ts"], r["te"], threshold) for r in d["reads"]]
    assert rg == ro
    ll = g.BaselineScores()   # the active reads' LLs, in AddRead order (MultiReadMutationScorer.cpp:508-516)
    oll = [o.read_info(r)["ll"] for r in range(o.num_reads()) if o.read_info(r)["active"]]
    assert len(ll) == len(oll) == rg.count(0)
    for a, b in zip(ll, oll):
        assert _close(a, b)
    assert _close(g.BaselineScore(), o.baseline())
    if math.isnan(threshold):   # every read added: the z-scores over real error profiles
        (zg, za), zs = g.ZScores()
        ozg, oza, ozs = o.zscores()
        assert _close(zg, ozg) and _close(za, oza)
        assert all(_close(a, b) for a, b in zip(zs, ozs))
    m = d["mutation"]
    mt = {"INSERTION": P.INSERTION, "DELETION": P.DELETION, "SUBSTITUTION": P.SUBSTITUTION}[m["type"]]
    assert _close(g.Score(P.Mutation(mt, m["start"], m["base"])), o.score(mt, m["start"], m["base"]))
    muts = O.unique_mutations(tpl)
    gm = [P.Mutation(t, s, b) for (t, s, b) in muts]
    for (t, s, b), vf, vq in zip(muts, g.ScoreMany(gm), g.ScoreMany(gm, -12.5)):
        assert _close(vf, o.score(t, s, b)), (t, s, b)
        assert _close(vq, o.score(t, s, b, -12.5)), (t, s, b)
    conv, nt, na = P.RefineConsensus(g)
    ref = o.refine()
    assert (conv, nt, na) == (ref["converged"], ref["n_tested"], ref["n_applied"])
    assert g.Template() == o.template()
    qg, qo = P.ConsensusQVs(g), o.qvs()
    assert len(qg) == len(qo) and max(abs(a - b) for a, b in zip(qg, qo)) <= 1


def test_partial_windows_and_strands(P):
    from pbccs_amd import synth
    import numpy as np
    z = synth.make_zmws(1, 300, 4, seed=21)[0]
    L = len(z["draft"])
    reads = []
    rng = np.random.default_rng(5)
    for k, r in enumerate(z["reads"]):
        ts, te = int(rng.integers(0, 40)), L - int(rng.integers(0, 40))
        # clip the read sequence roughly to the window (non-spanning reads, MultiReadMutationScorer.hpp:112-114)
        frac0, frac1 = ts / L, te / L
        s = r["seq"][int(frac0 * len(r["seq"])):int(frac1 * len(r["seq"]))]
        reads.append({"seq": s, "strand": r["strand"], "ts": ts, "te": te})
    g, o, rg, ro = _scorers(P, z["draft"], reads)
    assert rg == ro
    muts = O.unique_mutations(z["draft"])
    for (t, s, b) in muts[::3]:
        m = P.Mutation(t, s, b)
        assert _close(g.Score(m), o.score(t, s, b)), (t, s, b)
        sg = g.Scores(m, -1e300)
        so = o.scores(t, s, b, -1e300)
        assert len(sg) == len(so)
        for x, y in zip(sg, so):
            assert _close(x, y)


def test_zscore_gate_and_zscores(P):
    from pbccs_amd import synth
    z = synth.make_zmws(1, 300, 5, seed=31)[0]
    reads = list(z["reads"])
    reads.append({"seq": "ACGT" * 75, "strand": 0, "ts": 0, "te": len(z["draft"])})   # junk read -> POOR_ZSCORE
    g, o, rg, ro = _scorers(P, z["draft"], reads, threshold=-5.0)
    assert rg == ro
    (zg, za), zs = g.ZScores()
    ozg, oza, ozs = o.zscores()
    assert _close(zg, ozg, 1e-9) and _close(za, oza, 1e-9)
    for a, b in zip(zs, ozs):
        assert _close(a, b, 1e-9)


@pytest.mark.parametrize("seed,length,passes", [(41, 200, 5), (42, 500, 8), (43, 800, 10)])
def test_refine_and_qvs_match_oracle(P, seed, length, passes):
    from pbccs_amd import synth
    z = synth.make_zmws(1, length, passes, seed=seed)[0]
    g, o, rg, ro = _scorers(P, z["draft"], z["reads"], threshold=-5.0)
    assert rg == ro
    conv, nt, na = P.RefineConsensus(g)
    ref = o.refine()
    assert conv == ref["converged"]
    assert (nt, na) == (ref["n_tested"], ref["n_applied"])
    assert g.Template() == o.template()
    assert _close(g.BaselineScore(), o.baseline(), 1e-9)
    qg = P.ConsensusQVs(g)
    qo = o.qvs()
    assert len(qg) == len(qo)
    assert max(abs(a - b) for a, b in zip(qg, qo)) <= 1
    assert sum(a != b for a, b in zip(qg, qo)) <= max(1, len(qo) // 1000)


def test_polish_batch_matches_oracle(P):
    from pbccs_amd import synth
    zs = synth.make_zmws(6, 400, 7, seed=51)
    res = P.polish_zmws(zs)
    for z, r in zip(zs, res):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert r["add_read_results"] == e["add_read_results"]
        assert r["n_tested"] == e["n_tested"] and r["n_applied"] == e["n_applied"]
        if e["converged"]:
            assert r["consensus"] == e["template"]
            assert abs(r["predicted_accuracy"] - e["pred_acc"]) < 1e-3
            assert max(abs(a - b) for a, b in zip(r["qvs"], e["qvs"])) <= 1
        assert _close(r["zg"], e["zg"], 1e-9) and _close(r["za"], e["za"], 1e-9)


@pytest.mark.parametrize("sep,lds_cap", [(10, None), (10, "5"), (3, "0"), (0, None)])
def test_device_best_subset_matches_host(P, monkeypatch, sep, lds_cap):
    """k_best_subset (BestSubset, Consensus-inl.hpp:98-118, on the device) against the host restatement on
    every refine round of a batch (PBCCS_CHECK_BEST_SUBSET=1 makes any difference fatal), with the LDS
    stage, the HBM path of lists longer than the LDS cap (PBCCS_BEST_LDS), another separation and
    separation 0 (the whole list, in order); the batch then matches the oracle bit-exactly.  Separation 0
    is checked device-against-host only: it applies overlapping mutations, whose transcript runs past the
    template (Mutation.cpp:131-170), so the window remap leaves the reference's contract there."""
    from pbccs_amd import synth
    from pbccs_amd.polish import ConsensusSettings
    monkeypatch.setenv("PBCCS_CHECK_BEST_SUBSET", "1")
    if lds_cap is not None:
        monkeypatch.setenv("PBCCS_BEST_LDS", lds_cap)
    zs = synth.make_zmws(5, 500, 6, seed=52 + sep)
    res = P.polish_zmws(zs, ConsensusSettings(mutation_separation=sep))
    if sep == 0:
        return
    for z, r in zip(zs, res):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"], separation=sep)
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]


def test_zmw6251_survey_probe_record_on_gpu(P):
    """ZMW 6251 against SURVEY.md §0 item 4's survey-probe record (boost-shim build, a cross-check only) and,
    bit for bit, against the oracle."""
    z = json.load(open(os.path.join(GOLD, "zmw6251.json")))
    r = P.polish_zmws([{"draft": z["draft"], "snr": z["snr"], "reads": z["reads"]}])[0]
    e = z["expected"]
    tol = e["tolerance_abs"]
    assert r["status"] == "Success"
    assert r["add_read_results"] == e["add_read_results"]
    assert abs(r["zg"] - e["zg"]) < tol["zg"] and abs(r["za"] - e["za"]) < tol["za"]
    assert r["n_tested"] == e["n_tested"] and r["n_applied"] == e["n_applied"]
    assert len(r["consensus"]) == e["final_length"]
    assert abs(r["predicted_accuracy"] - e["pred_acc"]) < tol["pred_acc"]
    o = O.polish_zmw(z["draft"], z["reads"], z["snr"], z["min_zscore"])
    assert r["consensus"] == o["template"]


def test_fills_with_threshold_division_path_match_oracle(P, monkeypatch):
    """The fill's row-threshold test (x >= pm / sdn) runs as two products with a division only in a 2^-49 band
    around the quotient; PBCCS_FILL_THR_MARGIN widens that band to 2^-4 so the division path decides most rows:
    per-read LL and flip-flop counts stay equal to the oracle, tall reads included."""
    from pbccs_amd import synth
    monkeypatch.setenv("PBCCS_FILL_THR_MARGIN", "0.0625")
    for z in synth.make_zmws(2, 2000, 10, seed=62):
        g, o, rg, ro = _scorers(P, z["draft"], z["reads"])
        assert rg == ro
        assert g.NumFlipFlops() == [o.read_info(k)["flipflops"] for k in range(len(z["reads"]))]
        for x, y in zip(g.BaselineScores(), [o.read_info(k)["ll"] for k in range(len(z["reads"]))]):
            assert _close(x, y, 1e-12, 1e-12)


def test_fills_2kb_match_oracle(P):
    """Full-size (configs[1]) fills: per-read LL and flip-flop counts, including the reads whose first
    band explodes past 4% of the matrix (the 5-pass reband path, ~one read per ZMW at 2 kb) and the
    6-flip-flop reads whose trailing passes the engine skips at the band fixed point."""
    from pbccs_amd import synth
    zs = synth.make_zmws(3, 2000, 10, seed=61)
    for z in zs:
        g, o, rg, ro = _scorers(P, z["draft"], z["reads"])
        assert rg == ro
        assert g.NumFlipFlops() == [o.read_info(k)["flipflops"] for k in range(len(z["reads"]))]
        for x, y in zip(g.BaselineScores(), [o.read_info(k)["ll"] for k in range(len(z["reads"]))]):
            assert _close(x, y, 1e-12, 1e-12)


def test_polish_2kb_batch_matches_oracle(P):
    """configs[1] ZMWs (2 kb insert, 10 passes) through the batch entry point: bit-exact consensus,
    nTested/nApplied and AddRead results; QVs within +-1."""
    from pbccs_amd import synth
    zs = synth.make_zmws(6, 2000, 10, seed=71)
    res = P.polish_zmws(zs)
    for z, r in zip(zs, res):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        assert r["consensus"] == e["template"]
        assert max(abs(a - b) for a, b in zip(r["qvs"], e["qvs"])) <= 1


def test_fills_10kb_match_oracle(P):
    """configs[2] reads (10 kb insert, 8 passes): wide bands and long windows, including reads whose
    columns outgrow the 1024-row LDS buffer (the all-rows 64-lane path) -- per-read LL and flip-flops."""
    from pbccs_amd import synth
    zs = synth.make_zmws(2, 10000, 8, seed=81)
    for z in zs:
        g, o, rg, ro = _scorers(P, z["draft"], z["reads"])
        assert rg == ro
        assert g.NumFlipFlops() == [o.read_info(k)["flipflops"] for k in range(len(z["reads"]))]
        for x, y in zip(g.BaselineScores(), [o.read_info(k)["ll"] for k in range(len(z["reads"]))]):
            assert _close(x, y, 1e-12, 1e-12)


def test_polish_mixed_batch_matches_oracle(P):
    """configs[3]-style batch (divergence stress): per-ZMW insert length, pass count and SNR all differ
    within one batch (lengths scaled down to 0.3-1.5 kb so the oracle stays fast)."""
    from pbccs_amd import synth
    zs = synth.make_zmws(8, None, None, seed=91, length_range=(300, 1500), passes_range=(3, 30), random_snr=True)
    res = P.polish_zmws(zs)
    for z, r in zip(zs, res):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]
            assert max(abs(a - b) for a, b in zip(r["qvs"], e["qvs"])) <= 1


def test_band_growth_in_kernel_matches_oracle(P, monkeypatch):
    """Every read starts with a 2-row-per-column value region, so nearly every fill outgrows it and moves
    to a larger region inside the kernel (CoopFill::valBump) -- results must not change."""
    from pbccs_amd import synth
    monkeypatch.setenv("PBCCS_INITIAL_BAND_HEIGHT", "2")
    zs = synth.make_zmws(4, 600, 6, seed=95)
    res = P.polish_zmws(zs)
    for z, r in zip(zs, res):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]


def test_band_reclaim_matches_oracle(P, monkeypatch):
    """PBCCS_RECLAIM=1: the refills relay the band pool out afresh (ArrowBatch::Relayout), ConsensusQVs run
    in the round each ZMW converges, and gated / NonConvergent ZMWs are retired -- with 2-row first regions,
    so every fill also re-runs passes into exact regions (regrow_bands).  Results must not change."""
    from pbccs_amd import synth
    monkeypatch.setenv("PBCCS_RECLAIM", "1")
    monkeypatch.setenv("PBCCS_INITIAL_BAND_HEIGHT", "2")
    seed, idx = NONCONVERGENT_2KB
    allz = synth.make_zmws(max(idx) + 1, 2000, 10, seed=seed)
    zs = synth.make_zmws(4, 2000, 10, seed=73) + [allz[idx[0]]]
    zs += synth.make_zmws(2, 600, 2, seed=74)   # too few passes: gated, retired after AddRead
    res = P.polish_zmws(zs)
    for k, (z, r) in enumerate(zip(zs, res)):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert r["add_read_results"] == e["add_read_results"]
        if k >= 5:
            assert r["status"] == "TooFewPasses"
            continue
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]
            assert max(abs(a - b) for a, b in zip(r["qvs"], e["qvs"])) <= 1
        else:
            assert r["status"] == "NonConvergent"


# configs[1] ZMWs (seed 1, the bench's first step) that the reference loop leaves NonConvergent: their
# templates oscillate until MaximumIterations, which the engine replays instead of re-running
# (engine.hip, Refine: cycle replay).  Found with tools/find_nonconvergent.py 2000 2000 10 1.
NONCONVERGENT_2KB = (1, (820, 880, 1324, 1962))


def test_nonconvergent_cycles_batch_match_oracle(P):
    from pbccs_amd import synth
    seed, idx = NONCONVERGENT_2KB
    allz = synth.make_zmws(max(idx) + 1, 2000, 10, seed=seed)
    zs = [allz[i] for i in idx]
    res = P.polish_zmws(zs)
    for z, r in zip(zs, res):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert not e["converged"]
        assert r["status"] == "NonConvergent"
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])


def test_nonconvergent_cycle_final_state_matches_oracle(P):
    """Through the scorer API the state after RefineConsensus is observable: the replayed cycle must end
    on the reference's final template (MaximumIterations - i mod period real iterations are run)."""
    from pbccs_amd import synth
    seed, idx = NONCONVERGENT_2KB
    z = synth.make_zmws(idx[0] + 1, 2000, 10, seed=seed)[idx[0]]
    g, o, rg, ro = _scorers(P, z["draft"], z["reads"], threshold=-5.0)
    assert rg == ro
    conv, nt, na = P.RefineConsensus(g)
    ref = o.refine()
    assert (conv, nt, na) == (ref["converged"], ref["n_tested"], ref["n_applied"])
    assert g.Template() == o.template()
    assert _close(g.BaselineScore(), o.baseline(), 1e-9)
    for odd in (39, 38):   # both parities of the iterations left after the cycle is detected
        g, o, _, _ = _scorers(P, z["draft"], z["reads"], threshold=-5.0)
        conv, nt, na = P.RefineConsensus(g, max_iterations=odd)
        ref = o.refine(max_iter=odd)
        assert (conv, nt, na) == (ref["converged"], ref["n_tested"], ref["n_applied"])
        assert g.Template() == o.template()


def test_phased_scoring_matches_oracle(P, monkeypatch):
    """Every refine round scored in phases (reads [0,3), then [3,5) and [5,n) of the mutations whose ordered
    fast-score prefix has not broken yet; engine.hip RunRound): consensus, nTested/nApplied, AddRead results
    and QVs as the oracle -- including a mixed batch where some ZMWs have fewer reads than a phase boundary
    and the NonConvergent 2 kb ZMWs (their replayed iterations consume the phased rounds' favourable lists)."""
    from pbccs_amd import synth
    monkeypatch.setenv("PBCCS_PHASED_MIN_TASKS", "0")
    seed, idx = NONCONVERGENT_2KB
    allz = synth.make_zmws(max(idx) + 1, 2000, 10, seed=seed)
    zs = [allz[i] for i in idx[:2]] + synth.make_zmws(2, 2000, 10, seed=72)
    zs += synth.make_zmws(6, None, None, seed=93, length_range=(300, 1200), passes_range=(3, 12), random_snr=True)
    res = P.polish_zmws(zs)
    for z, r in zip(zs, res):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]
            assert max(abs(a - b) for a, b in zip(r["qvs"], e["qvs"])) <= 1


def test_polish_10kb_batch_matches_oracle(P):
    """configs[2] ZMWs (10 kb insert, 8 passes) through the batch entry point: wide bands and long windows
    (reads on the all-rows global-column fill path included) -- bit-exact consensus, nTested/nApplied and
    AddRead results; QVs within +-1.  The oracle needs ~2.5 CPU-minutes for these two ZMWs, so its outputs
    are a committed fixture (tests/golden/make_polish_fixtures.py); the inputs are regenerated and checked
    against the fixture's digest."""
    import sys
    from pbccs_amd import synth
    sys.path.insert(0, GOLD)
    from make_polish_fixtures import digest
    fx = json.load(open(os.path.join(GOLD, "polish_10kb.json")))
    zs = synth.make_zmws(2, 10000, 8, seed=82)
    res = P.polish_zmws(zs)
    for z, r, e in zip(zs, res, fx["zmws"]):
        assert digest(z) == e["digest"]
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        assert e["converged"]
        assert r["consensus"] == e["consensus"]
        got = [min(max(q, 0), 93) for q in r["qvs"]]
        exp = [ord(c) - 33 for c in e["qvs"]]
        assert len(got) == len(exp) and max(abs(a - b) for a, b in zip(got, exp)) <= 1


def test_polish_mixed_long_matches_fixture(P):
    """configs[3] shapes at full size: a 15.2 kb insert with 21 passes beside a 0.7 kb / 3-pass and a
    4.8 kb / 14-pass ZMW at random SNRs, through the work queue (polish_stream: length buckets, memory-sized
    batches).  The oracle needs ~10 CPU-minutes for the long ZMW, so its records are a committed fixture
    (tests/golden/make_polish_fixtures.py mixed_long); inputs are regenerated and checked by digest."""
    import sys
    sys.path.insert(0, GOLD)
    from make_polish_fixtures import digest, mixed_long_zmws
    fx = json.load(open(os.path.join(GOLD, "polish_mixed_long.json")))
    zs = mixed_long_zmws()
    assert len(zs[0]["draft"]) >= 15000 and len(zs[0]["reads"]) >= 20
    res = P.polish_stream(zs)
    for z, r, e in zip(zs, res, fx["zmws"]):
        assert digest(z) == e["digest"]
        assert r["add_read_results"] == e["add_read_results"]
        # the oracle record is the scorer's polish; the batch applies Consensus.h's gates first (:473-490)
        st = e["add_read_results"]
        if sum(1 for s in st if s == 0) < 3:
            assert r["status"] == "TooFewPasses"
            continue
        if sum(1 for s in st if s != 0) / len(st) > 0.34:
            assert r["status"] == "TooManyUnusable"
            continue
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["consensus"]
            got = [min(max(q, 0), 93) for q in r["qvs"]]
            exp = [ord(c) - 33 for c in e["qvs"]]
            assert len(got) == len(exp) and max(abs(a - b) for a, b in zip(got, exp)) <= 1


def test_polish_20kb_matches_fixture(P):
    """configs[3]'s top length: a 20 kb insert with 24 passes -- the widest bands of the mixed workload, where
    the 4%-of-matrix reband (SimpleRecursor.cpp:642-691) explodes furthest and the bands are checkpointed --
    through the work queue against the oracle's committed record (tests/golden/make_polish_fixtures.py 20kb,
    ~30 CPU-minutes); the input is regenerated and checked by digest."""
    import sys
    sys.path.insert(0, GOLD)
    from make_polish_fixtures import digest, long20_zmws
    fx = json.load(open(os.path.join(GOLD, "polish_20kb.json")))
    zs = long20_zmws()
    assert len(zs[0]["draft"]) >= 19000 and len(zs[0]["reads"]) >= 24
    res = P.polish_stream(zs)
    for z, r, e in zip(zs, res, fx["zmws"]):
        assert digest(z) == e["digest"]
        assert r["add_read_results"] == e["add_read_results"]
        assert sum(1 for s in e["add_read_results"] if s == 0) >= 3   # a polished ZMW, not a gated one
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        assert e["converged"] and r["status"] in ("Success", "PoorQuality")
        assert r["consensus"] == e["consensus"]
        got = [min(max(q, 0), 93) for q in r["qvs"]]
        exp = [ord(c) - 33 for c in e["qvs"]]
        assert len(got) == len(exp) and max(abs(a - b) for a, b in zip(got, exp)) <= 1
