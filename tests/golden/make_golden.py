#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/ (run in the build container).

Reads data that the reference's own tests and demos hold (never its code):
  * ConsensusCore/src/Demos/MatrixTester.cpp:74-204 -- the 12 Arrow known-answer values (C#-derived,
    checked there at 1e-5 relative) and the template/read strings they are quoted on;
  * tests/data/m140905_..._X0.fasta -- the 10 subreads of ZMW 6251 (the only subread data in the tree);
  * SURVEY.md §0 item 4 / Appendix C -- the reference's recorded polish outputs on that ZMW
    (draft = subread 2, reads 1..8 mapped over the full draft, odd index REVERSE,
     SNR (10,7,5,11), MinZScore -5).
Writes:
  tests/golden/arrow_kats.json, tests/golden/zmw6251.json
Only this script touches /root/reference; the fixtures travel, the reference does not.
"""
import json
import os
import re
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _matrixtester_strings():
    src = open(os.path.join(REF, "ConsensusCore/src/Demos/MatrixTester.cpp")).read()
    long_tpl = re.search(r'std::string longTPL = "([ACGT]+)"', src).group(1)
    long_read = re.search(r'std::string long_read = "([ACGT]+)"', src).group(1)
    return long_tpl, long_read


def make_kats():
    long_tpl, long_read = _matrixtester_strings()
    snr = [10.0, 7.0, 5.0, 11.0]
    tpl, read = "ACGTCGT", "ACGTACGT"
    kats = {
        "tolerance_rel": 1e-5,
        "snr": snr,
        "source": "ConsensusCore/src/Demos/MatrixTester.cpp:74-204",
        # AddRead(mr) with the default (NaN) add threshold: no z-score gate.
        "baseline": [
            {"tpl": tpl, "reads": [read], "expected": -4.74517984808494, "line": 89},
            {"tpl": tpl, "reads": ["ACCTCGT"], "expected": -5.79237005993877, "line": 147},
        ],
        # scorer t = (tpl, [read]); Score(m) for single mutations.  type: 0 INS, 1 DEL, 2 SUB.
        "mutations": [
            {"tpl": tpl, "reads": [read], "type": 0, "start": 4, "base": "A", "expected": 4.00250386364592, "line": 155},
            {"tpl": tpl, "reads": [read], "type": 2, "start": 2, "base": "C", "expected": -5.19526526492876, "line": 161},
            {"tpl": tpl, "reads": [read], "type": 1, "start": 4, "base": "-", "expected": -4.33430539094949, "line": 166},
            {"tpl": tpl, "reads": [read], "type": 1, "start": 6, "base": "-", "expected": -9.70299447206563, "line": 171},
            {"tpl": tpl, "reads": [read], "type": 1, "start": 0, "base": "-", "expected": -10.5597017942167, "line": 182},
            {"tpl": tpl, "reads": [read], "type": 2, "start": 4, "base": "A", "expected": -0.166992912601578, "line": 196},
            {"tpl": tpl, "reads": [read], "type": 0, "start": 4, "base": "G", "expected": -1.60697112438296, "line": 201},
            # 200 copies of long_read against longTPL; Score(Del@755) / 200.
            {"tpl": long_tpl, "reads": [long_read], "copies": 200, "type": 1, "start": 755, "base": "-",
             "expected": -3.80891683862648, "divide_by": 200, "line": 140},
        ],
        # t_ = ("ACT", ["ACT"]); t0 = ("ACGT", ["ACT"]); BaselineScore(t_) == BaselineScore(t0) + Score(t0, Del@2),
        # and == BaselineScore(t0) after ApplyMutations({Del@2}).  (:117-129)
        "short_equalities": {"tpl_short": "ACT", "tpl_long": "ACGT", "read": "ACT", "type": 1, "start": 2, "line": 129},
    }
    return kats


def make_zmw6251():
    path = os.path.join(REF, "tests/data/m140905_042212_sidney_c100564852550000001823085912221377_s1_X0.fasta")
    names, seqs = [], []
    for line in open(path):
        line = line.strip()
        if line.startswith(">"):
            names.append(line[1:])
            seqs.append("")
        elif line:
            seqs[-1] += line
    draft = seqs[2]
    reads = []
    for k in range(1, 9):
        reads.append({"name": names[k], "seq": seqs[k], "strand": 1 if k % 2 else 0, "ts": 0, "te": len(draft)})
    return {
        "source": "tests/data/m140905_..._X0.fasta (ZMW 6251); recipe and outputs: SURVEY.md §0 item 4",
        "all_subreads": [{"name": n, "seq": s} for n, s in zip(names, seqs)],
        "draft": draft,
        "snr": [10.0, 7.0, 5.0, 11.0],
        "min_zscore": -5.0,
        "reads": reads,
        "expected": {
            "add_read_results": [0] * 8,
            "zg": 11.295465,
            "za": 3.993550,
            "converged": True,
            "n_tested": 11255,
            "n_applied": 37,
            "final_length": 602,
            "pred_acc": 0.999696,
            "tolerance_abs": {"zg": 5e-6, "za": 5e-6, "pred_acc": 5e-7},
        },
    }


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are committed, nothing to regenerate")
    with open(os.path.join(HERE, "arrow_kats.json"), "w") as f:
        json.dump(make_kats(), f, indent=1)
    with open(os.path.join(HERE, "zmw6251.json"), "w") as f:
        json.dump(make_zmw6251(), f, indent=1)
    print("wrote arrow_kats.json, zmw6251.json")


if __name__ == "__main__":
    main()
