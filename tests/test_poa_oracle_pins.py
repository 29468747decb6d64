"""Pins the POA CPU restatement (oracle/poa_oracle.cpp) to the reference's own POA tests: every case of
ConsensusCore/src/Tests/TestPoaConsensus.cpp and tests/TestSparsePoa.cpp, as tests/golden/poa_kats.json
holds them (inputs and expected outputs parsed out of those files by tests/golden/make_golden.py).
CPU only."""
import json
import os

import pytest

from oracle import oracle as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "poa_kats.json")))


def _rc(s):
    return s[::-1].translate(str.maketrans("ACGT", "TGCA"))


@pytest.mark.parametrize("case", GOLD["poa_consensus"], ids=lambda c: c["test"])
def test_poa_consensus_kats(case):
    mc = case["min_coverage"] if case["min_coverage"] is not None else -O.INT_MAX
    seq, dot = O.poa_consensus(case["reads"], case["mode"], mc, graphviz_flags=case["graphviz_flags"])
    if case["expected"] is not None:
        assert seq == case["expected"]
    if case["expected_dot"]:
        assert dot.replace("\n", "") == case["expected_dot"]
    if case.get("deterministic_only"):
        # NondeterminismRegressionTest: 100 runs give one answer
        assert {O.poa_consensus(case["reads"], case["mode"], mc) for _ in range(5)} == {seq}


def _sparse_case(name):
    return next(c for c in GOLD["sparse_poa"] if c["test"] == name)


@pytest.mark.parametrize("name", ["SparsePoaTest.TestLocalStaggered", "SparsePoaTest.TestOrientation"])
def test_sparse_poa_extents(name):
    case = _sparse_case(name)
    got = O.sparse_poa(case["reads"], case["min_coverage"])
    assert all(k >= 0 for k in got["keys"])
    assert got["consensus"] == case["expected"]
    for k, exp in case["summaries"].items():
        s = got["summaries"][int(k)]
        if "rc" in exp:
            assert s["rc"] == exp["rc"]
        if "read" in exp:
            assert list(s["read"]) == exp["read"] and list(s["tpl"]) == exp["tpl"]


def test_sparse_poa_zmw6251():
    case = _sparse_case("SparsePoaTest.TestZmw6251")
    got = O.sparse_poa(case["reads"], case["min_coverage"])
    assert all(k >= 0 for k in got["keys"]) and len(got["summaries"]) == case["num_reads"]
    for k, exp in case["summaries"].items():
        assert got["summaries"][int(k)]["rc"] == exp["rc"]
    for k, (lo, hi) in case["covers"].items():
        b, e = got["summaries"][int(k)]["tpl"]
        assert b <= lo and hi <= e


def test_sparse_poa_single_read_x100():
    for seq in O.poa_kat_reads(0)[:25]:   # the first 25 of the 100 (2-20 kb each); all run in the GPU test
        got = O.sparse_poa([seq], 1)
        assert got["consensus"] == seq
        s = got["summaries"][0]
        assert s["read"] == (0, len(seq)) and s["tpl"] == (0, len(seq)) and not s["rc"]


def test_sparse_poa_single_and_half_x100():
    for seq1 in O.poa_kat_reads(1)[:20]:
        L = len(seq1)
        seq2 = _rc(seq1)[:L // 3]
        got = O.sparse_poa([seq1, seq2], 1)
        assert got["consensus"] == seq1
        a, b = got["summaries"]
        assert a["read"] == (0, L) and a["tpl"] == (0, L) and not a["rc"]
        assert b["read"] == (0, L // 3) and b["tpl"] == (L - L // 3, L) and b["rc"]
