#!/usr/bin/env python3
"""Oracle polish fixtures for inputs too slow to polish on the CPU inside a GPU test (run in the build
container; minutes of CPU).  Inputs are regenerated from pbccs_amd.synth (PCG64, seeded), so a fixture
holds only the input digest and the oracle's outputs:

  tests/golden/polish_10kb.json -- synth.make_zmws(2, 10000, 8, seed=82) (configs[2] shape), polished by
  oracle/arrow_oracle.cpp (AddRead, RefineConsensus, ConsensusQVs).

The oracle is test infrastructure (CPU restatement of the reference path, oracle/ header); the GPU test
compares the engine's batch polish against these records.
"""
import hashlib
import json
import os
import sys

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


def main():
    zs = synth.make_zmws(2, 10000, 8, seed=82)
    out = {"inputs": "synth.make_zmws(2, 10000, 8, seed=82)", "zmws": []}
    for z in zs:
        e = O.polish_zmw(z["draft"], z["reads"], z["snr"])
        out["zmws"].append({
            "digest": digest(z),
            "converged": bool(e["converged"]),
            "n_tested": e["n_tested"],
            "n_applied": e["n_applied"],
            "add_read_results": e["add_read_results"],
            "consensus": e["template"],
            "qvs": "".join(chr(33 + min(max(q, 0), 93)) for q in e["qvs"]),
            "qvs_raw_max": max(e["qvs"]),
        })
        print(len(out["zmws"]), e["n_tested"], e["n_applied"], flush=True)
    json.dump(out, open(os.path.join(HERE, "polish_10kb.json"), "w"))


if __name__ == "__main__":
    main()
