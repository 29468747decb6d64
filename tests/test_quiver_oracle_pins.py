"""Pin the Quiver CPU restatement (oracle/quiver_oracle.cpp) to the reference's own Quiver gtest
known answers (tests/golden/quiver_kats.json, transcribed by tests/golden/make_golden.py from
ConsensusCore/src/Tests/{TestRecursors,TestMutationScorer,TestMultiReadMutationScorer}.cpp with
TestingParams from ParameterSettings.cpp).  Exact float equality, as the gtests' EXPECT_EQ / FLOAT_EQ."""
import json
import math
import os

import pytest

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kats():
    return json.load(open(os.path.join(GOLD, "quiver_kats.json")))


def run_kat(make_scorer, k, params):
    """Drive one KAT through a scorer factory (shared with the GPU parity test)."""
    s = make_scorer(k["tpl"], params, moves=k["moves"], score_diff=k["score_diff"], fast_threshold=k["fast_threshold"])
    for r in k["reads"]:
        s.add_read(r["seq"], r["strand"], r["ts"], r["te"] if r["te"] is not None else len(k["tpl"]))
    for c in k["checks"]:
        kind = c["kind"]
        if kind == "baseline":
            assert s.baseline() == c["expected"], (k["name"], s.baseline())
        elif kind == "score":
            t, p, b = c["mut"]
            v = s.score(t, p, b)
            assert v == pytest.approx(c["expected"], abs=1e-5), (k["name"], c, v)
        elif kind == "read_score_mutation":
            t, p, b = c["mut"]
            v = s.read_score_mutation(0, t, p, b)
            assert v == pytest.approx(c["expected"], abs=1e-5), (k["name"], c, v)
        elif kind == "add_read":
            r = c["read"]
            s.add_read(r["seq"], r["strand"], r["ts"], r["te"] if r["te"] is not None else len(s.template()))
        elif kind == "alignment":
            assert s.alignment(c["read"]) == (c["target"], c["query"]), (k["name"], s.alignment(c["read"]))
        elif kind == "apply":
            s.apply([tuple(m) for m in c["muts"]])
            assert s.template() == c["template"]
        else:
            raise AssertionError(kind)
    return s


@pytest.mark.parametrize("idx", range(len(_kats()["kats"])))
def test_quiver_kats(idx):
    d = _kats()
    run_kat(O.QuiverScorer, d["kats"][idx], d["params"])


def test_cephes_log_add_close_to_libm():
    """logAdd (detail/SseMath.hpp:66-88) with the Cephes polynomials: ~1e-7 relative of the exact value."""
    for a, b in [(-1.0, -2.0), (0.0, 0.0), (-30.0, -0.5), (-100.0, -100.0), (5.0, -3.0)]:
        exact = max(a, b) + math.log1p(math.exp(min(a, b) - max(a, b)))
        assert O.quiver_log_add(a, b) == pytest.approx(exact, rel=1e-6, abs=1e-6)
    assert O.quiver_log_add(-3.4028234663852886e38, -1.0) == -1.0   # -FLT_MAX is the empty-cell value


def test_sum_product_and_viterbi_agree_on_exact_reads():
    """With one dominant path (read == template) both combiners give the same baseline up to the mass of
    the alternative paths (sum-product >= Viterbi)."""
    P = _kats()["params"]
    tpl = "GATTACAGATTACAGGCT"
    v = O.QuiverScorer(tpl, P)
    v.add_read(tpl)
    sp = O.QuiverScorer(tpl, P, sum_product=True)
    sp.add_read(tpl)
    assert v.baseline() == 0.0
    assert 0.0 <= sp.baseline() < 0.1
