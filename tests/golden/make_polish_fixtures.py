#!/usr/bin/env python3
"""Oracle polish fixtures for inputs too slow to polish on the CPU inside a GPU test (run in the build
container; minutes of CPU).  Inputs are regenerated from pbccs_amd.synth (PCG64, seeded), so a fixture
holds only the input digest and the oracle's outputs:

  tests/golden/polish_10kb.json -- synth.make_zmws(2, 10000, 8, seed=82) (configs[2] shape), polished by
  oracle/arrow_oracle.cpp (AddRead, RefineConsensus, ConsensusQVs).
  tests/golden/polish_mixed_long.json -- mixed_long_zmws() (configs[3] shape: a 15.2 kb insert with 21
  passes beside a 0.7 kb / 3-pass and a 4.8 kb / 14-pass ZMW at random SNRs), the same records.
  tests/golden/polish_20kb.json -- long20_zmws(): configs[3]'s top length, a 20 kb insert with 24 passes (the
  widest bands of the mix, SimpleRecursor.cpp:642-691's reband at its largest), the same records.

Usage: make_polish_fixtures.py [10kb|mixed_long|20kb]  (default: all; the 15 kb ZMW takes ~10 CPU-minutes, the
20 kb one ~30)

The oracle is test infrastructure (CPU restatement of the reference path, oracle/ header); the GPU test
compares the engine's batch polish against these records.
"""
import hashlib
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from pbccs_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402


def digest(z):
    h = hashlib.sha256(z["draft"].encode())
    for r in z["reads"]:
        h.update(repr((r["seq"], r.get("strand", 0), r.get("ts", 0), r.get("te"))).encode())
    h.update(repr(tuple(z["snr"])).encode())
    return h.hexdigest()


def mixed_long_zmws():
    """configs[3] shapes for the GPU test: one ZMW of at least 15 kb with at least 20 passes (SNR as
    configs[1], so its reads pass the z-score gate), one short few-pass ZMW and one mid-size one at
    per-ZMW random SNRs."""
    rng = np.random.Generator(np.random.PCG64(303))
    return [synth.make_zmw(rng, 15200, 21),
            synth.make_zmw(rng, 700, 3, tuple(float(x) for x in rng.uniform(6.0, 14.0, size=4))),
            synth.make_zmw(rng, 4800, 14, tuple(float(x) for x in rng.uniform(6.0, 14.0, size=4)))]


def long20_zmws():
    """configs[3]'s upper end: one 20 kb ZMW with 24 passes at configs[1]'s SNR."""
    rng = np.random.Generator(np.random.PCG64(2020))
    return [synth.make_zmw(rng, 20000, 24)]


def record(z):
    e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
    return {
        "digest": digest(z),
        "converged": bool(e["converged"]),
        "n_tested": e["n_tested"],
        "n_applied": e["n_applied"],
        "add_read_results": e["add_read_results"],
        "consensus": e["template"],
        "qvs": "".join(chr(33 + min(max(q, 0), 93)) for q in e.get("qvs", [])),
        "qvs_raw_max": max(e["qvs"]) if e.get("qvs") else None,
    }


def write(name, inputs, zs):
    with ProcessPoolExecutor(max_workers=len(zs)) as ex:   # one ZMW per process: the oracle is serial
        recs = list(ex.map(record, zs))
    for r in recs:
        print(name, r["n_tested"], r["n_applied"], r["converged"], flush=True)
    json.dump({"inputs": inputs, "zmws": recs}, open(os.path.join(HERE, name), "w"))


def main():
    which = sys.argv[1:] or ["10kb", "mixed_long", "20kb"]
    if "10kb" in which:
        write("polish_10kb.json", "synth.make_zmws(2, 10000, 8, seed=82)", synth.make_zmws(2, 10000, 8, seed=82))
    if "mixed_long" in which:
        write("polish_mixed_long.json", "make_polish_fixtures.mixed_long_zmws()", mixed_long_zmws())
    if "20kb" in which:
        write("polish_20kb.json", "make_polish_fixtures.long20_zmws()", long20_zmws())


if __name__ == "__main__":
    main()
