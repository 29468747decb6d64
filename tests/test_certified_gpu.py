"""The certified fast path against the restatement and against the exact path.

The batch polish fills the LDS-only tall reads with the reassociated chain (scan_chain64): their band values are not
the reference's bit for bit, so every decision taken on them is certified against a tracked deviation bound -- each
band end, begin hint and flip-flop test in the fill (an uncertain read re-runs on the exact path), the AddRead z-score
gate, and each round's favourable test, fast-score break and BestSubset float-cast order (an uncertain ZMW round is
scored again on exact bands).  So the records must equal the reference's: consensus, nTested / nApplied and AddRead
results bit-exact, z-scores within 1e-9 relative (north_star: LLs within 1e-4), QVs within +-1.
"""
import math
from concurrent.futures import ThreadPoolExecutor

import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _close(a, b, rel=1e-9):
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b)
    return abs(a - b) <= 1e-9 + rel * max(abs(a), abs(b))


def _polish(zs, monkeypatch, **env):
    import pbccs_amd
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    eng = pbccs_amd.Engine(0)
    res = pbccs_amd.polish_zmws(zs, engine=eng)
    c = eng.counters()
    for k in env:
        monkeypatch.delenv(k)
    return res, c


def _oracle(zs):
    with ThreadPoolExecutor(max_workers=8) as ex:   # ctypes releases the GIL
        return list(ex.map(lambda z: O.polish_zmw(z["draft"], z["reads"], z["snr"]), zs))


def _check_against_oracle(zs, res, ref):
    for z, r, e in zip(zs, res, ref):
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]
            assert max(abs(a - b) for a, b in zip(r["qvs"], e["qvs"])) <= 1
        assert _close(r["zg"], e["zg"]) and _close(r["za"], e["za"])


@pytest.fixture(scope="module")
def batch2kb():
    from pbccs_amd import synth
    zs = synth.make_zmws(16, 2000, 10, seed=61)   # about one read per ZMW takes the tall path
    return zs, _oracle(zs)


def test_certified_scan_matches_oracle_on_2kb(batch2kb, monkeypatch):
    zs, ref = batch2kb
    res, c = _polish(zs, monkeypatch)
    assert c["scan_reads"] > 0
    _check_against_oracle(zs, res, ref)


def test_certified_scan_fallbacks_match_oracle(batch2kb, monkeypatch):
    """Bounds inflated 1e9x (PBCCS_SCAN_DEV_SCALE): many fill decisions and score decisions become uncertain, so the
    exact re-runs of reads and the exact re-scoring of ZMW rounds carry the batch -- and it still equals the reference."""
    zs, ref = batch2kb
    res, c = _polish(zs, monkeypatch, PBCCS_SCAN_DEV_SCALE="1e9")
    assert c["scan_reads"] > 0 and c["uncertain_reads"] > 0
    _check_against_oracle(zs, res, ref)


def test_certified_scan_equals_exact_path(batch2kb, monkeypatch):
    zs, _ = batch2kb
    fast, cf = _polish(zs, monkeypatch)
    exact, ce = _polish(zs, monkeypatch, PBCCS_CERTIFIED_SCAN="0")
    assert cf["scan_reads"] > 0 and ce["scan_reads"] == 0
    for a, b in zip(fast, exact):
        for k in ("status", "consensus", "n_tested", "n_applied", "add_read_results", "n_passes"):
            assert a[k] == b[k], k
        assert len(a["qvs"]) == len(b["qvs"]) and all(abs(x - y) <= 1 for x, y in zip(a["qvs"], b["qvs"]))
        assert all(_close(x, y) for x, y in zip(a["zscores"], b["zscores"]))


@pytest.mark.parametrize("ckpt_k", ["8", "0"])
def test_certified_scan_equals_exact_path_on_10kb_hybrid(ckpt_k, monkeypatch):
    """10 kb reads: their columns overflow the LDS buffers, so they fill on the hybrid path (rows past the LDS buffer in
    global scratch), checkpointed (PBCCS_CKPT_K=8: every 8th column kept, the rest replayed by k_score_ckpt) or with full
    bands (0).  The certified fast path -- on the hybrid path too (PBCCS_SCAN_PATHS=3; off by default) -- must give the
    exact path's records."""
    from pbccs_amd import synth
    zs = synth.make_zmws(3, 10000, 8, seed=67)
    fast, cf = _polish(zs, monkeypatch, PBCCS_CKPT_K=ckpt_k, PBCCS_SCAN_PATHS="3")
    exact, ce = _polish(zs, monkeypatch, PBCCS_CKPT_K=ckpt_k, PBCCS_CERTIFIED_SCAN="0")
    assert cf["scan_reads"] > 0 and ce["scan_reads"] == 0
    for a, b in zip(fast, exact):
        for k in ("status", "consensus", "n_tested", "n_applied", "add_read_results", "n_passes"):
            assert a[k] == b[k], k
        assert len(a["qvs"]) == len(b["qvs"]) and all(abs(x - y) <= 1 for x, y in zip(a["qvs"], b["qvs"]))
        assert all(_close(x, y) for x, y in zip(a["zscores"], b["zscores"]))

