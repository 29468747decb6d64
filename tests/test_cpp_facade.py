"""The C++ facade (include/pbccs_amd/ConsensusCore.hpp) compiles a Consensus.h-style driver unchanged in
shape (CPU test), and that driver reproduces ZMW 6251 on the GPU (gpu test): bit for bit
against the oracle, and against SURVEY.md §0 item 4's survey-probe record (a boost-shim build, a cross-check)."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "consensus_driver.cpp")
BIN = os.path.join(ROOT, "tests", "cpp", "_build", "consensus_driver")
LIBDIR = os.path.join(ROOT, "pbccs_amd", "_lib")


def _build():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I" + os.path.join(ROOT, "include"), SRC, "-L" + LIBDIR,
                           "-lpbccs_amd", "-Wl,-rpath," + LIBDIR, "-o", BIN])


def test_facade_driver_compiles_and_links():
    if not os.path.exists(os.path.join(LIBDIR, "libpbccs_amd.so")):
        pytest.skip("library not built")
    _build()
    assert os.path.exists(BIN)


@pytest.mark.gpu
def test_facade_driver_reproduces_zmw6251():
    _build()
    z = json.load(open(os.path.join(ROOT, "tests", "golden", "zmw6251.json")))
    lines = [f"{z['draft']} {' '.join(str(x) for x in z['snr'])} {z['min_zscore']}"]
    for r in z["reads"]:
        lines.append(f"{r['strand']} {r['ts']} {r['te']} {r['seq']}")
    out = subprocess.run([BIN], input="\n".join(lines) + "\n", capture_output=True, text=True, check=True).stdout
    kv = dict(line.split("=", 1) for line in out.strip().splitlines())
    e = z["expected"]
    assert kv["converged"] == "1"
    assert int(kv["n_tested"]) == e["n_tested"] and int(kv["n_applied"]) == e["n_applied"]
    assert abs(float(kv["zg"]) - e["zg"]) < e["tolerance_abs"]["zg"]
    assert abs(float(kv["pred_acc"]) - e["pred_acc"]) < e["tolerance_abs"]["pred_acc"]
    assert len(kv["consensus"]) == e["final_length"]
    assert int(kv["success"]) == 8


POA_SRC = os.path.join(ROOT, "tests", "cpp", "poa_driver.cpp")
POA_BIN = os.path.join(ROOT, "tests", "cpp", "_build", "poa_driver")


def _build_poa():
    os.makedirs(os.path.dirname(POA_BIN), exist_ok=True)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-I" + os.path.join(ROOT, "include"), POA_SRC, "-L" + LIBDIR,
                           "-lpbccs_amd", "-Wl,-rpath," + LIBDIR, "-o", POA_BIN])


def test_poa_facade_driver_compiles_and_links():
    if not os.path.exists(os.path.join(LIBDIR, "libpbccs_amd.so")):
        pytest.skip("library not built")
    _build_poa()
    assert os.path.exists(POA_BIN)


@pytest.mark.gpu
def test_poa_facade_driver_matches_oracle():
    """Consensus.h's PoaConsensus loop through the C++ SparsePoa facade on ZMW 6251's subreads (one read
    dropped, maxPoaCov 8) equals the oracle's SparsePoa."""
    from oracle import oracle as O
    _build_poa()
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "poa_kats.json")))
    reads = next(c for c in gold["sparse_poa"] if c["test"] == "SparsePoaTest.TestZmw6251")["reads"]
    reads = [None if k == 3 else r for k, r in enumerate(reads)]
    inp = "8\n" + "\n".join("" if r is None else r for r in reads) + "\n"
    out = subprocess.run([POA_BIN], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    exp = O.sparse_poa(reads, max_coverage=8)
    assert out[0] == exp["consensus"]
    assert [int(x) for x in out[1].split()] == [k for k in exp["keys"] if k != -2]
    summ = [tuple(int(x) for x in line.split()) for line in out[2:2 + len(exp["summaries"])]]
    assert summ == [(int(s["rc"]), *s["read"], *s["tpl"]) for s in exp["summaries"]]
    assert out[2 + len(exp["summaries"])] == "GGG"
