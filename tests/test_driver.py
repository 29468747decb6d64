"""Per-ZMW driver steps before the boundary (pbccs_amd/driver.py): FilterReads, the POA bookkeeping and
ExtractMappedRead of include/pacbio/ccs/Consensus.h:223-390, and their effect on the gates inside the
batched polish (nPasses over full-pass SUCCESS reads, the drop fraction over every POA key).

The reference has no test of these functions; the expectations below are derived by hand from the cited
lines (parity unpinned by reference fixtures).  The GPU test polishes a driver-built ZMW and checks the
engine against the oracle on the reads the driver added, and the gates against a Python restatement of
Consensus.h:441-490."""
import pytest

from pbccs_amd import driver, synth

FULL, PARTIAL = driver.FULL_PASS, driver.ADAPTER_BEFORE


def _r(n, flags=FULL, tag="A"):
    return {"seq": tag * n, "flags": flags}


def test_filter_reads_orders_by_closeness_to_the_median_full_pass():
    reads = [_r(100, tag="a"), _r(90, tag="b"), _r(250, tag="c"), _r(120, PARTIAL, "d"), _r(100, tag="e"),
             _r(40, PARTIAL, "f"), _r(60, tag="g")]
    # full passes 100, 90, 250, 100, 60 -> median 100, maxLen 200: read c (250) is dropped (None, last)
    out = driver.filter_reads(reads, 10)
    assert out[-1] is None and len(out) == len(reads)
    tags = [r["seq"][0] for r in out[:-1]]
    # full passes by min(l/m, m/l) descending (a, e tie at 1.0 in input order; b 0.9; g 0.6), then partials
    # (d: 100/120 = 0.833; f: 0.4)
    assert tags == ["a", "e", "b", "g", "d", "f"]


def test_filter_reads_even_median_and_no_full_passes():
    reads = [_r(10, tag="a"), _r(21, tag="b"), _r(30, PARTIAL, "c")]
    # median of (10, 21) = 0.5 * 31 = 15.5 -> maxLen = 2 * 15 = 30: read c (30) is dropped
    out = driver.filter_reads(reads, 5)
    assert out[-1] is None and [r["seq"][0] for r in out[:2]] == ["b", "a"]   # 15.5/21=0.738 > 10/15.5=0.645
    # no full pass: median = longest (40), maxLen 80, every read kept, ordered by (0, v) descending
    reads = [_r(20, PARTIAL, "a"), _r(40, PARTIAL, "b"), _r(30, PARTIAL, "c")]
    assert [r["seq"][0] for r in driver.filter_reads(reads, 5)] == ["b", "c", "a"]
    # median below MinLength -> nothing
    assert driver.filter_reads([_r(8), _r(9)], 10) == []
    assert driver.filter_reads([], 10) == []


def test_extract_mapped_read_uses_rc_extents_on_the_given_read():
    read = {"seq": "AACCGGTTAC", "flags": FULL}
    s = {"rc": True, "read": (2, 8), "tpl": (5, 11)}
    mr = driver.extract_mapped_read(read, s, 3)
    # Appendix A.15: substr of the read as given (not of its reverse complement), strand REVERSE
    assert mr == {"seq": "CCGGTT", "strand": 1, "ts": 5, "te": 11, "full_pass": True}
    assert driver.extract_mapped_read(read, {"rc": False, "read": (2, 4), "tpl": (0, 2)}, 3) is None
    assert driver.extract_mapped_read(read, {"rc": False, "read": (5, 4), "tpl": (0, 2)}, 0) is None


class StubPoa:
    """SparsePoa surface over fixed answers: reads in `reject` cannot be added (key -1); the consensus and
    each added read's summary come from the constructor."""

    def __init__(self, draft, summary_of, reject=()):
        self.draft, self.summary_of, self.reject = draft, summary_of, set(reject)
        self.keys, self.min_cov = [], None

    def orient_and_add_read(self, seq):
        if seq in self.reject:
            return -1
        self.keys.append(seq)
        return len(self.keys) - 1

    def find_consensus(self, min_coverage):
        self.min_cov = min_coverage
        return self.draft, [self.summary_of(s) for s in self.keys]


def test_poa_bookkeeping_min_coverage_and_max_coverage():
    reads = [{"seq": s, "flags": FULL} for s in ("AAAA", "CCCC", "GGGG", "TTTT", "ACAC", "GTGT", "CACA")]
    poa = StubPoa("ACGT", lambda s: {"rc": False, "read": (0, 4), "tpl": (0, 4)}, reject={"GGGG"})
    draft, keys, _ = driver.poa_inputs(reads + [None], poa)
    assert keys == [0, 1, -1, 2, 3, 4, 5, -1] and poa.min_cov == (6 + 1) // 2 - 1
    poa = StubPoa("ACGT", lambda s: {"rc": False, "read": (0, 4), "tpl": (0, 4)})
    _, keys, _ = driver.poa_inputs(reads, poa, max_poa_coverage=3)
    assert keys == [0, 1, 2] and poa.min_cov == 1


def _driver_zmw(seed):
    """A synthetic ZMW as raw subreads: full passes plus one partial pass, one read the stub POA rejects and
    one whose POA extent is too short to extract."""
    z = synth.make_zmws(1, 400, 8, seed=seed)[0]
    reads = [{"seq": r["seq"], "flags": FULL} for r in z["reads"]]
    reads[3]["flags"] = PARTIAL
    strand = {r["seq"]: r["strand"] for r in z["reads"]}
    reject = {reads[5]["seq"]}
    short = reads[6]["seq"]

    def summary(seq):
        if seq == short:
            return {"rc": False, "read": (0, 5), "tpl": (0, 5)}
        return {"rc": strand[seq] == 1, "read": (0, len(seq)), "tpl": (0, len(z["draft"]))}
    return {"snr": z["snr"], "reads": reads}, StubPoa(z["draft"], summary, reject)


def test_zmw_input_placeholders_and_statuses():
    chunk, poa = _driver_zmw(11)
    status, zmw = driver.zmw_input(chunk, poa)
    assert status is None and len(zmw["reads"]) == len(chunk["reads"])
    assert sum(1 for r in zmw["reads"] if r["seq"] is None) == 2      # the rejected and the too-short read
    assert driver.zmw_input({"snr": [10] * 4, "reads": []}, poa) == ("NoSubreads", None)
    tiny = StubPoa("ACG", lambda s: {"rc": False, "read": (0, 3), "tpl": (0, 3)})
    assert driver.zmw_input({"snr": [10] * 4, "reads": [_r(40)] * 3}, tiny)[0] == "TooShort"


@pytest.mark.gpu
def test_driver_zmw_polishes_like_the_oracle_with_reference_gates():
    import pbccs_amd
    from oracle import oracle as O
    for seed in (11, 12):
        chunk, poa = _driver_zmw(seed)
        _, zmw = driver.zmw_input(chunk, poa)
        got = pbccs_amd.polish_zmws([zmw], engine=pbccs_amd.Engine(0))[0]
        added = [r for r in zmw["reads"] if r["seq"] is not None]
        e = O.polish_zmw(zmw["draft"], added, zmw["snr"])
        # AddRead results: the added reads in order, -1 at the placeholders
        it = iter(e["add_read_results"])
        assert got["add_read_results"] == [-1 if r["seq"] is None else next(it) for r in zmw["reads"]]
        # Consensus.h:441-490: passes = full-pass SUCCESS reads; dropped / nReads over every POA key
        n_pass = sum(1 for r, s in zip(added, e["add_read_results"]) if s == 0 and r["full_pass"])
        n_drop = sum(1 for s in e["add_read_results"] if s != 0)
        assert got["n_passes"] == n_pass
        if n_pass < 3:
            assert got["status"] == "TooFewPasses"
        elif n_drop / len(zmw["reads"]) > 0.34:
            assert got["status"] == "TooManyUnusable"
        else:
            assert (got["n_tested"], got["n_applied"]) == (e["n_tested"], e["n_applied"])
            if e["converged"]:
                assert got["consensus"] == e["template"]
