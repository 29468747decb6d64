"""Pin the CPU restatement (oracle/) against the reference's own known answers.

* ConsensusCore/src/Demos/MatrixTester.cpp:74-204 -- 12 Arrow KATs, 1e-5 relative (the demo's ASSERT_EQ).
* src/Tests/TestMutations.cpp, TestMutationEnumerator.cpp -- ApplyMutations / transcripts / enumerators.
* SURVEY.md §0 item 4 -- the survey's probe record of tests/data ZMW 6251 (the reference built against a
  boost shim in the survey container: a cross-check of the restatement, not a parity pin by this tier's rules).
"""
import json
import math
import os

import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kats():
    return json.load(open(os.path.join(GOLD, "arrow_kats.json")))


def test_matrixtester_baselines():
    k = _kats()
    for b in k["baseline"]:
        s = O.Scorer(b["tpl"], k["snr"])
        for r in b["reads"]:
            s.add_read(r)
        v = s.baseline()
        assert abs(1 - v / b["expected"]) < k["tolerance_rel"], (b, v)


@pytest.mark.parametrize("idx", range(8))
def test_matrixtester_mutation_scores(idx):
    k = _kats()
    m = k["mutations"][idx]
    s = O.Scorer(m["tpl"], k["snr"])
    for r in m["reads"] * m.get("copies", 1):
        s.add_read(r)
    v = s.score(m["type"], m["start"], m["base"]) / m.get("divide_by", 1)
    assert abs(1 - v / m["expected"]) < k["tolerance_rel"], (m["line"], v)


def test_matrixtester_short_equalities():
    k = _kats()
    se = k["short_equalities"]
    a = O.Scorer(se["tpl_short"], k["snr"])
    a.add_read(se["read"])
    b = O.Scorer(se["tpl_long"], k["snr"])
    b.add_read(se["read"])
    assert abs(1 - a.baseline() / (b.baseline() + b.score(se["type"], se["start"]))) < 1e-5
    b.apply([(se["type"], se["start"], "-")])
    assert b.template() == se["tpl_short"]
    assert abs(1 - a.baseline() / b.baseline()) < 1e-5


def test_enumerators_match_gtests():
    # TestMutationEnumerator.cpp:73-104
    assert len(O.unique_mutations("GAATC")) == 7 * 5 + 1 - 1
    assert len(O.nearby_mutations("GAATC", [1], 1)) == 8 + 7
    assert len(O.nearby_mutations("GAATC", [1], 2)) == 8 + 7 + 6
    assert sorted(O.nearby_mutations("GAATC", [1, 3], 2)) == sorted(O.unique_mutations("GAATC"))


def test_apply_mutations_match_gtests():
    # TestMutations.cpp:64-181
    I, D, S = O.INSERTION, O.DELETION, O.SUBSTITUTION
    assert O.apply_mutations("ACGTACGTACGT", [(S, 0, "C")])[0] == "CCGTACGTACGT"
    assert O.apply_mutations("ACGTACGTACGT", [(D, 4, "-")])[0] == "ACGTCGTACGT"
    assert O.apply_mutations("ACGTACGTACGT", [(I, 0, "C")])[0] == "CACGTACGTACGT"
    muts = [(I, 3, "C"), (I, 2, "T"), (I, 0, "G"), (S, 6, "T"), (D, 4, "-")]
    assert O.apply_mutations("GATTACA", muts)[0] == "GGATTCTCT"
    assert O.apply_mutations("GATTACA", [(S, 2, "A"), (I, 2, "T")])[0] == "GATATACA"
    assert O.apply_mutations("GATTACA", [(D, 2, "-"), (I, 5, "C"), (S, 4, "G")])[1] == [0, 1, 2, 2, 3, 5, 6, 7]
    assert O.apply_mutations("GG", [(I, 0, "A")])[1] == [1, 2, 3]
    assert O.apply_mutations("AGG", [(D, 0, "-")])[1] == [0, 0, 1, 2]


def test_zmw6251_polish_matches_survey_probe_record():
    """Cross-check against SURVEY.md §0 item 4's record (a boost-shim build of the reference in the survey
    container).  A shim build pins nothing by this tier's rules; the pins are the KATs above."""
    z = json.load(open(os.path.join(GOLD, "zmw6251.json")))
    r = O.polish_zmw(z["draft"], z["reads"], z["snr"], z["min_zscore"])
    e = z["expected"]
    tol = e["tolerance_abs"]
    assert r["add_read_results"] == e["add_read_results"]
    assert abs(r["zg"] - e["zg"]) < tol["zg"]
    assert abs(r["za"] - e["za"]) < tol["za"]
    assert r["converged"] == e["converged"]
    assert r["n_tested"] == e["n_tested"]
    assert r["n_applied"] == e["n_applied"]
    assert len(r["template"]) == e["final_length"]
    assert abs(r["pred_acc"] - e["pred_acc"]) < tol["pred_acc"]


def test_polish_fixture_inputs_regenerate():
    """tests/golden/polish_10kb.json was made from synth.make_zmws(2, 10000, 8, seed=82): the inputs the GPU
    test regenerates must still hash to the fixture's digests (guards synth drift)."""
    import json
    import os
    import sys
    from pbccs_amd import synth
    gold = os.path.join(os.path.dirname(__file__), "golden")
    sys.path.insert(0, gold)
    from make_polish_fixtures import digest
    fx = json.load(open(os.path.join(gold, "polish_10kb.json")))
    zs = synth.make_zmws(2, 10000, 8, seed=82)
    assert [digest(z) for z in zs] == [e["digest"] for e in fx["zmws"]]


def test_matrixtester_multiread_fixture_runs_on_the_restatement():
    """MatrixTester.cpp:212-384 (TestMultiReadScorer): the reference's only real multi-read ZMW -- 54 subreads,
    real SNRs, non-spanning windows on both strands.  The demo asserts nothing, so this pins the fixture's shape
    and that the restatement takes every read (the GPU comparison is test_gpu_parity's)."""
    d = json.load(open(os.path.join(GOLD, "matrixtester_multiread.json")))
    assert len(d["tpl"]) == 223 and len(d["reads"]) == 54
    assert {r["strand"] for r in d["reads"]} == {0, 1}
    assert sum(1 for r in d["reads"] if r["ts"] > 0 or r["te"] < len(d["tpl"])) >= 20   # non-spanning windows
    o = O.Scorer(d["tpl"], d["snr"])
    res = [o.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["threshold"]) for r in d["reads"]]
    assert set(res) <= {0, 1, 3}   # SUCCESS / ALPHABETAMISMATCH / POOR_ZSCORE at the demo's threshold 1.0
    assert res.count(0) > 0
    m = d["mutation"]
    v = o.score(O.INSERTION if m["type"] == "INSERTION" else O.SUBSTITUTION, m["start"], m["base"])
    assert math.isfinite(v)
