"""Checkpointed bands: reads whose bands keep every K-th column's values only, scored by
k_score_ckpt, which replays the other columns from the kept ones.  The replay must reproduce the fill's
values bit for bit, so every result is compared with the oracle (oracle/arrow_oracle.cpp) exactly as the
full-band tests do.  PBCCS_CKPT_ALL=K puts every cooperative fill on checkpoints (the default policy only
takes the tall bands of windows >= 4 kb, which tests/test_gpu_parity.py's 10 kb and 15 kb fixtures cover);
K = 3 exercises an interval that divides nothing, K = 8 the default."""
import math
import os

import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
SNR = [10.0, 7.0, 5.0, 11.0]


def _close(a, b, rel=1e-9, abs_=1e-9):
    if math.isinf(a) or math.isinf(b) or math.isnan(a) or math.isnan(b):
        return (math.isnan(a) and math.isnan(b)) or a == b
    return abs(a - b) <= abs_ + rel * max(abs(a), abs(b))


@pytest.fixture
def ckpt_env(monkeypatch):
    def set_(k, phased_min=None):
        monkeypatch.setenv("PBCCS_CKPT_ALL", str(k))
        if phased_min is not None:
            monkeypatch.setenv("PBCCS_PHASED_MIN_TASKS", str(phased_min))
    return set_


@pytest.mark.parametrize("K,seed,length,passes", [(3, 12, 150, 4), (8, 13, 400, 6), (4, 14, 900, 5)])
def test_every_mutation_score_checkpointed(ckpt_env, K, seed, length, passes):
    import pbccs_amd as P
    from pbccs_amd import synth
    ckpt_env(K)
    z = synth.make_zmws(1, length, passes, seed=seed)[0]
    g = P.ArrowMultiReadMutationScorer(P.ArrowConfig(SNR), z["draft"])
    o = O.Scorer(z["draft"], SNR)
    for r in z["reads"]:
        assert g.AddRead(r["seq"], r["strand"], 0, len(z["draft"])) == \
            o.add_read(r["seq"], r["strand"], 0, len(z["draft"]))
    assert _close(g.BaselineScore(), o.baseline())
    muts = O.unique_mutations(z["draft"])
    full = g.ScoreMany([P.Mutation(t, s, b) for (t, s, b) in muts])
    for (t, s, b), v in zip(muts, full):
        assert _close(v, o.score(t, s, b)), (t, s, b)
    # per-read scores of a spread of mutations (Scores(): every read, no early break)
    for (t, s, b) in muts[::17]:
        for x, y in zip(g.Scores(P.Mutation(t, s, b), -1e300), o.scores(t, s, b, -1e300)):
            assert _close(x, y), (t, s, b)


@pytest.mark.parametrize("K,phased_min", [(4, None), (5, 0)])
def test_batch_polish_checkpointed_matches_oracle(ckpt_env, K, phased_min):
    """configs[1] ZMWs through the batch polish with every band checkpointed; phased_min 0 scores every
    refine round in phases, so sparse chunks of surviving mutations reach the replay."""
    import pbccs_amd as P
    from concurrent.futures import ThreadPoolExecutor
    from pbccs_amd import synth
    ckpt_env(K, phased_min)
    zs = synth.make_zmws(6, 2000, 10, seed=606 + K)
    res = P.polish_zmws(zs)
    O.lib()
    with ThreadPoolExecutor(max_workers=min(6, os.cpu_count() or 1)) as ex:
        orc = list(ex.map(lambda z: O.polish_zmw(z["draft"], z["reads"], z["snr"]), zs))
    for r, e in zip(res, orc):
        assert r["add_read_results"] == e["add_read_results"]
        assert (r["n_tested"], r["n_applied"]) == (e["n_tested"], e["n_applied"])
        if e["converged"]:
            assert r["consensus"] == e["template"]
            assert max(abs(a - b) for a, b in zip(r["qvs"], e["qvs"])) <= 1


def test_checkpoint_policy_cuts_band_memory(monkeypatch):
    """The default policy checkpoints the tall bands of >= 4 kb windows: the same 10 kb ZMWs keep far fewer
    band values than with checkpoints off (PBCCS_CKPT_K=0), with identical results."""
    import pbccs_amd as P
    from pbccs_amd import synth
    zs = synth.make_zmws(2, 10000, 8, seed=82)   # tests/golden/polish_10kb.json's inputs
    out = {}
    for k in ("0", "8"):
        monkeypatch.setenv("PBCCS_CKPT_K", k)
        eng = P.Engine(0)
        eng.counters(reset=True)
        res = P.polish_zmws(zs, engine=eng)
        out[k] = (res, eng.counters(reset=True)["band_used_bytes"])
    (r0, b0), (r8, b8) = out["0"], out["8"]
    for a, b in zip(r0, r8):
        assert (a["consensus"], a["qvs"], a["n_tested"], a["n_applied"], a["add_read_results"]) == \
               (b["consensus"], b["qvs"], b["n_tested"], b["n_applied"], b["add_read_results"])
    assert b8 < 0.5 * b0, (b8, b0)
