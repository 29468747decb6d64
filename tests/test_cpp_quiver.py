"""The Quiver half of the C++ facade (include/pbccs_amd/Quiver.hpp): tests/cpp/quiver_driver.cpp is a ConsensusCore
Quiver caller written against the facade only -- QuiverConfigTable, MultiReadMutationScorer<R> of each recursor type,
MappedQvRead / QvSequenceFeatures, RefineConsensus / ConsensusQVs, QvEvaluator.  On the GPU it runs the reference's
12 Quiver gtest KATs (tests/golden/quiver_kats.json, through run_kat like the oracle and the Python mirror), a
RefineConsensus + ConsensusQVs polish against the oracle, and QvEvaluator's four moves over every cell of seeded
reads against the oracle's evaluator, with and without pins.  The CPU test compiles and links it."""
import json
import math
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "quiver_driver.cpp")
BIN = os.path.join(ROOT, "tests", "cpp", "_build", "quiver_driver")
LIBDIR = os.path.join(ROOT, "pbccs_amd", "_lib")
KATS = json.load(open(os.path.join(ROOT, "tests", "golden", "quiver_kats.json")))


def _build():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I" + os.path.join(ROOT, "include"), SRC, "-L" + LIBDIR,
                           "-lpbccs_amd", "-Wl,-rpath," + LIBDIR, "-o", BIN])


def test_quiver_facade_driver_compiles_and_links():
    if not os.path.exists(os.path.join(LIBDIR, "libpbccs_amd.so")):
        pytest.skip("library not built")
    _build()
    assert os.path.exists(BIN)


def _tracks(features, n):
    f = features or {}
    out = []
    for k in ("ins", "subs", "del", "del_tag", "merge"):
        v = f.get(k)
        if v is None:
            out.append("-")
        else:
            vals = [float(ord(x)) if isinstance(x, str) else float(x) for x in v]
            assert len(vals) == n
            out.append(",".join(repr(x) for x in vals))
    return out


class Driver:
    """One quiver_driver process: a command line in, an answer line out."""

    def __init__(self):
        self.p = subprocess.Popen([BIN], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)

    def ask(self, line):
        self.p.stdin.write(line + "\n")
        self.p.stdin.flush()
        out = self.p.stdout.readline().rstrip("\n")
        assert not out.startswith("error"), (line[:80], out)
        return out

    def close(self):
        self.p.stdin.write("quit\n")
        self.p.stdin.flush()
        self.p.wait(timeout=60)


def _f(x):
    return float.fromhex(x)


class CppQuiver:
    """The oracle's QuiverScorer call shape over the C++ facade driver (run_kat drives it)."""
    driver = None

    def __init__(self, tpl, params, moves=15, score_diff=12.5, fast_threshold=-12.5, add_threshold=1.0,
                 sum_product=False, recursor="SparseSse"):
        d = CppQuiver.driver
        self.d = d
        p = " ".join(repr(float(x)) for x in O.qv_params(params))
        rec = O.QUIVER_RECURSORS.index(recursor)
        assert d.ask(f"new {int(sum_product)} {rec} {moves} {score_diff!r} {fast_threshold!r} {add_threshold!r} {p} "
                     f"{tpl}") == "ok"

    def add_read(self, seq, strand=0, ts=0, te=None, features=None, threshold=None):
        te = len(self.template()) if te is None else te
        thr = "nan" if threshold is None else repr(float(threshold))
        return self.d.ask(f"add {strand} {ts} {te} {thr} {seq} {' '.join(_tracks(features, len(seq)))}") == "1"

    def score(self, t, p, b="-", fast=False):
        return _f(self.d.ask(f"score {t} {p} {b} {int(fast)}"))

    def read_score_mutation(self, r, t, p, b="-"):
        return _f(self.d.ask(f"rsm {r} {t} {p} {b}"))

    def baseline(self):
        return _f(self.d.ask("baseline"))

    def apply(self, muts):
        assert self.d.ask(f"apply {len(muts)} " + " ".join(f"{t} {p} {b}" for t, p, b in muts)) == "ok"

    def template(self):
        return self.d.ask("template")

    def alignment(self, r):
        t, q = self.d.ask(f"align {r}").split()
        return t, q

    def refine(self):
        c, nt, na = self.d.ask("refine").split()
        return {"converged": c == "1", "n_tested": int(nt), "n_applied": int(na)}

    def qvs(self):
        return [int(x) for x in self.d.ask("qvs").split()]


@pytest.fixture(scope="module")
def driver():
    _build()
    d = Driver()
    CppQuiver.driver = d
    yield d
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("idx", range(len(KATS["kats"])))
def test_quiver_kats_through_cpp_facade(driver, idx):
    from tests.test_quiver_oracle_pins import run_kat
    run_kat(CppQuiver, KATS["kats"][idx], KATS["params"])


PARAMS2 = dict(Match=-0.2, Mismatch=-8.0, MismatchS=-0.15, Branch=-3.5, BranchS=-0.12, DeletionN=-7.5,
               DeletionWithTag=-4.5, DeletionWithTagS=-0.2, Nce=-6.0, NceS=-0.1, Merge=[-3.0, -3.2, -2.9, -3.1],
               MergeS=[-0.1, -0.12, -0.09, -0.11])


def _features(rng, seq):
    n = len(seq)
    return {"ins": rng.integers(0, 25, n).tolist(), "subs": rng.integers(0, 25, n).tolist(),
            "del": rng.integers(0, 25, n).tolist(), "del_tag": rng.choice(list("ACGTN"), size=n).tolist(),
            "merge": rng.integers(0, 25, n).tolist()}


@pytest.mark.gpu
@pytest.mark.parametrize("sum_product,recursor", [(False, "SparseSse"), (True, "SparseSse"), (False, "DenseSimple")])
def test_quiver_refine_and_qvs_through_cpp_facade_match_oracle(driver, sum_product, recursor):
    """RefineConsensus + ConsensusQVs over a Quiver MultiReadMutationScorer built by the facade equal the oracle's
    (consensus, nTested, nApplied, QVs exact, per-read flip-flops)."""
    from pbccs_amd import synth
    z = synth.make_zmws(1, 160, 5, seed=512 + int(sum_product))[0]
    rng = np.random.default_rng(7)
    reads = [dict(r, features=_features(rng, r["seq"])) for r in z["reads"]]
    g = CppQuiver(z["draft"], PARAMS2, sum_product=sum_product, recursor=recursor)
    o = O.QuiverScorer(z["draft"], PARAMS2, sum_product=sum_product, recursor=recursor)
    for r in reads:
        assert g.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"]) == \
            bool(o.add_read(r["seq"], r["strand"], r["ts"], r["te"], r["features"]))
    assert g.baseline() == o.baseline()
    flips = [int(x) for x in driver.ask("flips").split()]
    active = [k for k in range(o.num_reads()) if o.read_info(k)["active"]]
    assert active and [flips[k] for k in active] == [o.read_info(k)["flipflops"] for k in active]
    eg, eo = g.refine(), o.refine()
    assert (eg["converged"], eg["n_tested"], eg["n_applied"]) == (eo["converged"], eo["n_tested"], eo["n_applied"])
    assert g.template() == o.template()
    assert g.qvs() == o.qvs()


@pytest.mark.gpu
@pytest.mark.parametrize("pins", [(True, True), (False, True), (True, False), (False, False)])
def test_qv_evaluator_moves_through_cpp_facade_match_oracle(driver, pins):
    """QvEvaluator::Inc / Del / Extra / Merge (QvEvaluator.hpp:160-207) on the device, at every cell of a seeded
    read x template (plus the edge rows and columns each move's domain admits, and cells outside them: NaN), bit for
    bit against the oracle's evaluator; Merge on homopolymer runs included."""
    rng = np.random.default_rng(31 + pins[0] + 2 * pins[1])
    tpl = "".join(rng.choice(list("ACGT"), size=40)) + "AAAGGGTTTCC"
    seq = tpl[3:30] + "GGGG" + tpl[31:48]
    f = _features(rng, seq)
    I, J = len(seq), len(tpl)
    cells = [(i, j) for i in range(-1, I + 2) for j in range(-1, J + 2)]
    p = " ".join(repr(float(x)) for x in O.qv_params(PARAMS2))
    line = (f"moves {int(pins[0])} {int(pins[1])} {tpl} {seq} {' '.join(_tracks(f, I))} {len(cells)} " +
            " ".join(f"{i} {j}" for i, j in cells) + " " + p)
    out = driver.ask(line)
    assert "single-cell-mismatch" not in out
    got = [_f(x) for x in out.split()]
    n = len(cells)
    exp = O.qv_eval_moves(seq, tpl, PARAMS2, cells, f, pin_start=pins[0], pin_end=pins[1])
    for k in range(4):
        for c, a, b in zip(cells, got[k * n:(k + 1) * n], exp[k]):
            assert (math.isnan(a) and math.isnan(b)) or a == b, (k, c, a, b)
    assert sum(1 for v in exp[3] if v > -1e30 and not math.isnan(v)) > 0   # some Merge cells are live
