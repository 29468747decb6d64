"""ZMW work queue (pbccs_polish_batch / pbccs_plan_batches): the host-side batch plan on CPU, and on the
GPU the queue's results against the oracle and against one-batch polish (a ZMW's result must not depend on
which batch, slot or bucket it lands in)."""
import math

import pytest

from pbccs_amd import synth


def _mixed(n, seed, lo=500, hi=20000):
    return synth.make_zmws(n, None, None, seed=seed, length_range=(lo, hi), passes_range=(3, 30), random_snr=True)


@pytest.mark.parametrize("budget,cap,ratio", [(30e9, 2000, 1.5), (2e9, 3, 1.5), (1e12, 2000, 1e9), (1.0, 5, 1.0)])
def test_plan_is_a_bucketed_partition(budget, cap, ratio):
    import pbccs_amd
    zs = _mixed(60, seed=5)
    batches, est = pbccs_amd.plan_batches(zs, budget, cap, ratio)
    flat = [i for b in batches for i in b]
    assert sorted(flat) == list(range(len(zs)))
    sizes = []
    for b in batches:
        assert 1 <= len(b) <= cap
        lens = [len(zs[i]["draft"]) for i in b]
        assert lens == sorted(lens)
        assert max(lens) <= ratio * min(lens) + 1e-9
        bytes_ = sum(est[i] for i in b)
        assert len(b) == 1 or bytes_ <= budget
        sizes.append(bytes_)
    # longest templates first (a batch's time follows its rounds' latency), then largest
    keys = [(max(len(zs[i]["draft"]) for i in b), est_b) for b, est_b in zip(batches, sizes)]
    assert keys == sorted(keys, reverse=True)
    assert (batches, est) == pbccs_amd.plan_batches(zs, budget, cap, ratio)   # deterministic


def test_plan_estimates_grow_with_length_and_passes():
    import pbccs_amd
    a = synth.make_zmws(1, 2000, 10, seed=1)[0]
    b = synth.make_zmws(1, 10000, 8, seed=1)[0]
    c = synth.make_zmws(1, 2000, 20, seed=1)[0]
    _, est = pbccs_amd.plan_batches([a, b, c], 1e12)
    # 10 kb windows keep checkpointed tall bands (every K-th column), so they grow by less
    # than the full (I+1)(J+1) matrix would, but still well above linear in the window
    assert est[1] > 6 * est[0] and 1.8 * est[0] < est[2] < 2.2 * est[0]
    # the one-batch budget of a 2 kb / 10-pass ZMW is within ~2x of the measured 13.5 MB
    assert 13.5e6 <= est[0] <= 30e6


def test_plan_rejects_bad_arguments():
    import pbccs_amd
    zs = _mixed(3, seed=1)
    for args in [(0.0, 10, 1.5), (1e9, 0, 1.5), (1e9, 10, 0.5)]:
        with pytest.raises(pbccs_amd.PbccsError):
            pbccs_amd.plan_batches(zs, *args)
    assert pbccs_amd.plan_batches([], 1e9) == ([], [])


@pytest.mark.gpu
@pytest.mark.parametrize("per_batch", [0, 2])
def test_work_queue_matches_oracle_and_single_batch(per_batch):
    """Mixed lengths (0.3-1.5 kb so the oracle stays fast), passes and SNRs through the queue: buckets of
    different sizes on different workspace slots; zmws_per_batch=2 exercises the caller-sized chunks."""
    import pbccs_amd
    from oracle import oracle as O
    zs = _mixed(10, seed=97, lo=300, hi=1500)
    eng = pbccs_amd.Engine(0)
    eng.set_concurrency(3)
    got = pbccs_amd.polish_stream(zs, pbccs_amd.ConsensusSettings(zmws_per_batch=per_batch), eng)
    one = pbccs_amd.polish_zmws(zs, engine=eng)
    def same(a, b):   # NaN z-scores (ZMWs gated before ZScores) compare equal
        return a == b or (isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b))

    for z, r, s in zip(zs, got, one):
        assert r.keys() == s.keys()
        for k in r:
            if isinstance(r[k], list):
                assert len(r[k]) == len(s[k]) and all(same(x, y) for x, y in zip(r[k], s[k])), k
            else:
                assert same(r[k], s[k]), k
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]
            assert max(abs(a - b) for a, b in zip(r["qvs"], e["qvs"])) <= 1


def test_queue_fails_loudly_without_engine():
    """pbccs_polish_batch never throws across the ABI: a null engine is EINVAL, not a crash or a CPU fallback."""
    import ctypes
    from pbccs_amd import lib as L
    n = 2
    ins = (L.CZmwInput * n)()
    outs = (L.CZmwOutput * n)()
    opts = L.CPolishOptions()
    L.load().pbccs_polish_options_default(ctypes.byref(opts))
    rc = L.load().pbccs_polish_batch(None, ins, n, ctypes.byref(opts), outs)
    assert L.ERRORS[rc] == "EINVAL"


@pytest.mark.gpu
def test_work_queue_gated_zmws_keep_input_order():
    """ZMWs rejected before the device (no subreads, draft shorter than MinLength) mixed into the queue, one
    of them alone in its length bucket: statuses land at their input positions and the rest still polish."""
    import pbccs_amd
    from oracle import oracle as O
    zs = _mixed(4, seed=98, lo=300, hi=600)
    empty = {"draft": "ACGTACGTACGTACGT", "snr": [10.0, 7.0, 5.0, 11.0], "reads": []}
    short = {"draft": "ACGTAC", "snr": [10.0, 7.0, 5.0, 11.0], "reads": [{"seq": "ACGTAC", "strand": 0}] * 3}
    batch = [zs[0], empty, zs[1], short, zs[2], zs[3]]
    got = pbccs_amd.polish_stream(batch, engine=pbccs_amd.Engine(0))
    assert got[1]["status"] == "NoSubreads" and got[3]["status"] == "TooShort"
    for z, r in zip(zs, [got[0], got[2], got[4], got[5]]):
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]


def _same_records(got, ref):
    def same(a, b):   # NaN z-scores (ZMWs gated before ZScores) compare equal
        return a == b or (isinstance(a, float) and isinstance(b, float) and math.isnan(a) and math.isnan(b))
    for r, s in zip(got, ref):
        assert r.keys() == s.keys()
        for k in r:
            if isinstance(r[k], list):
                assert len(r[k]) == len(s[k]) and all(same(x, y) for x, y in zip(r[k], s[k])), k
            else:
                assert same(r[k], s[k]), k


@pytest.mark.gpu
def test_out_of_memory_batches_are_rerun_with_identical_results(monkeypatch):
    """PBCCS_POOL_CAP_MB caps every band pool, so a 24-ZMW 2 kb batch (~340 MB of bands at its high-water
    mark) runs the pool out of memory mid-polish
    (PBCCS_EOOM inside the engine).  Each entry point rebuilds the batch from its inputs and reruns it,
    halved until it fits -- pbccs_batch_polish, pbccs_batch_polish_many beside a batch that fits, and the
    work queue -- and every ZMW's record equals the uncapped polish."""
    import pbccs_amd
    zs = synth.make_zmws(24, 2000, 10, seed=31)
    small = synth.make_zmws(2, 600, 6, seed=32)
    ref = pbccs_amd.polish_zmws(zs, engine=pbccs_amd.Engine(0))
    ref_small = pbccs_amd.polish_zmws(small, engine=pbccs_amd.Engine(0))

    # the cap is set before the batches are created: a pool maps in granules of min(1 GB, cap), and an
    # uncapped creation would map a whole 1 GB granule that the 24 ZMWs then fit in
    monkeypatch.setenv("PBCCS_POOL_CAP_MB", "200")
    eng = pbccs_amd.Engine(0)
    eng.set_concurrency(2)
    batch = pbccs_amd.PreparedBatch(zs, engine=eng)    # its initial band regions (~160 MB) fit the cap
    batch.polish()
    _same_records(batch.results(), ref)
    assert eng.counters()["oom_retries"] >= 2          # the whole batch, then its halves
    batch.close()

    eng = pbccs_amd.Engine(0)
    eng.set_concurrency(2)
    b1 = pbccs_amd.PreparedBatch(zs, engine=eng)
    b2 = pbccs_amd.PreparedBatch(small, engine=eng)
    pbccs_amd.polish_many([b1, b2])
    _same_records(b1.results(), ref)
    _same_records(b2.results(), ref_small)
    assert eng.counters()["oom_retries"] >= 1
    b1.close()
    b2.close()

    eng = pbccs_amd.Engine(0)
    eng.set_concurrency(2)
    got = pbccs_amd.polish_stream(zs + small, pbccs_amd.ConsensusSettings(zmws_per_batch=24), eng)
    _same_records(got, ref + ref_small)
    assert eng.counters()["oom_retries"] >= 1


@pytest.mark.gpu
def test_out_of_memory_rerun_on_slot_streams_after_same_va_remap(monkeypatch):
    """The round-5 failure (same-VA remap): the work queue's out-of-memory rerun on the slots' persistent
    streams (PBCCS_SLOT_STREAMS=1) returned unpolished drafts for 22-23 of 24 ZMWs, with most of the device held
    elsewhere (as earlier tests' engines hold it in a full GPU run).  Its pool had been handed back the address range
    it had mapped and unmapped two reservations before; pools now keep such ranges reserved, so the rerun maps fresh
    addresses and every record equals the uncapped polish."""
    import ctypes
    import pbccs_amd
    zs = synth.make_zmws(24, 2000, 10, seed=31)
    small = synth.make_zmws(2, 600, 6, seed=32)
    ref = pbccs_amd.polish_zmws(zs + small, engine=pbccs_amd.Engine(0))
    # the HIP runtime the engine library uses (torch bundles another one, which need not see the device here)
    hip = ctypes.CDLL("libamdhip64.so")
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
    hold = max(0, free.value - (20 << 30))   # leave 20 GB: the fills take no in-kernel growth headroom
    blocks = []
    try:
        while hold > (1 << 30):
            n = min(hold, 16 << 30)
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) == 0
            blocks.append(p)
            hold -= n
        monkeypatch.setenv("PBCCS_POOL_CAP_MB", "200")
        monkeypatch.setenv("PBCCS_SLOT_STREAMS", "1")
        eng = pbccs_amd.Engine(0)
        eng.set_concurrency(2)
        got = pbccs_amd.polish_stream(zs + small, pbccs_amd.ConsensusSettings(zmws_per_batch=24), eng)
        assert eng.counters()["oom_retries"] >= 2
        _same_records(got, ref)
    finally:
        for p in blocks:
            hip.hipFree(p)


@pytest.mark.gpu
def test_device_memory_does_not_grow_across_calls(monkeypatch):
    """buffers that stream-ordered growth retires are freed at quiescent points (Workspace::TrimRetired),
    so repeating the same work on one engine -- growing batches, and an out-of-memory rerun with its pool unmaps --
    leaves the device's free memory where the previous repetition left it."""
    import ctypes
    import pbccs_amd
    hip = ctypes.CDLL("libamdhip64.so")

    def free_bytes():
        f, t = ctypes.c_size_t(), ctypes.c_size_t()
        assert hip.hipDeviceSynchronize() == 0 and hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)) == 0
        return f.value

    # a 24-ZMW 2 kb batch (its pool runs out under the cap: a rerun, halved) beside a batch of 16 small ZMWs
    zs = synth.make_zmws(24, 2000, 10, seed=31) + synth.make_zmws(16, 600, 6, seed=41)
    eng = pbccs_amd.Engine(0)
    eng.set_concurrency(2)
    settings = pbccs_amd.ConsensusSettings(zmws_per_batch=24)
    monkeypatch.setenv("PBCCS_POOL_CAP_MB", "200")
    frees = []
    for _ in range(3):   # the first repetition sizes everything; the next two must not take more
        pbccs_amd.polish_stream(zs, settings, eng)
        frees.append(free_bytes())
    assert eng.counters()["oom_retries"] >= 2
    assert frees[1] - frees[2] < (64 << 20), frees
