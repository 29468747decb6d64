"""The C++ facade (include/pbccs_amd/ConsensusCore.hpp) compiles a Consensus.h-style driver unchanged in
shape (CPU test), and that driver reproduces the reference record for ZMW 6251 on the GPU (gpu test)."""
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
