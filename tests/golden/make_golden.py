#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/ (run in the build container).

Reads data that the reference's own tests and demos hold (never its code):
  * ConsensusCore/src/Demos/MatrixTester.cpp:74-204 -- the 12 Arrow known-answer values (C#-derived,
    checked there at 1e-5 relative) and the template/read strings they are quoted on;
  * tests/data/m140905_..._X0.fasta -- the 10 subreads of ZMW 6251 (the only subread data in the tree);
  * SURVEY.md §0 item 4 / Appendix C -- the survey's probe record of the polish on that ZMW (a boost-shim
    build of the reference in the survey container: a cross-check, not a parity pin)
    (draft = subread 2, reads 1..8 mapped over the full draft, odd index REVERSE,
     SNR (10,7,5,11), MinZScore -5).
  * ConsensusCore/src/Tests/TestPoaConsensus.cpp and tests/TestSparsePoa.cpp -- the POA known answers
    (read sets, alignment modes, expected graph dumps, consensus sequences and per-read extents), parsed
    out of the test sources' string literals and EXPECT lines.
Writes:
  tests/golden/arrow_kats.json, tests/golden/zmw6251.json, tests/golden/quiver_kats.json,
  tests/golden/poa_kats.json
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


def _testing_params():
    """TestingParams (ConsensusCore/src/Tests/ParameterSettings.cpp:47-63), read from the test source."""
    src = open(os.path.join(REF, "ConsensusCore/src/Tests/ParameterSettings.cpp")).read()
    body = src[src.index("QvModelParams TestingParams"):src.index("QuiverConfig TestingConfig")]
    vals = [float(v.rstrip("f")) for v in re.findall(r"(-?[0-9.]+f),\s*//|(?<=\s)(-?[0-9.]+f)\);", body) for v in v if v]
    names = ["Match", "Mismatch", "MismatchS", "Branch", "BranchS", "DeletionN", "DeletionWithTag",
             "DeletionWithTagS", "Nce", "NceS", "Merge", "MergeS"]
    assert len(vals) == len(names), vals
    return dict(zip(names, vals))


def make_quiver_kats():
    """The Quiver gtest known answers, transcribed as data (inputs + expected outputs), values from
    TestingParams.  Viterbi recursor unless noted (SparseSseQvRecursor, the MultiReadMutationScorer type
    of Quiver/MultiReadMutationScorer.hpp:242)."""
    P = _testing_params()
    INS, DEL, SUB = 0, 1, 2
    nb, std = 1e9, 200.0   # BandingOptions(0, 1e9) "noBanding", BandingOptions(4, 200) (TestRecursors.cpp:78-80)
    medium_tpl = "GATTACA" * 10
    medium_read = "GATTACA" * 3 + "GATTTTTTACA" * 4 + "GATTACA" * 3

    def case(name, source, tpl, reads, checks, moves=15, score_diff=std, fast=-12.5):
        return {"name": name, "source": source, "tpl": tpl, "moves": moves, "score_diff": score_diff,
                "fast_threshold": fast, "reads": reads, "checks": checks}

    def rd(seq, strand=0, ts=0, te=None):
        return {"seq": seq, "strand": strand, "ts": ts, "te": te}

    def sc(t, pos, base, exp):
        return {"kind": "score", "mut": [t, pos, base], "expected": exp}

    def ms(t, pos, base, exp):   # single-read MutationScorer::ScoreMutation (read 0)
        return {"kind": "read_score_mutation", "mut": [t, pos, base], "expected": exp}

    kats = [
        # + RecursorBase::Alignment's Target() / Query() (:117-119, :147-149, :172-174)
        case("SmallMatch", "src/Tests/TestRecursors.cpp:99-126", "GATG", [rd("GATG")],
             [{"kind": "baseline", "expected": 0.0},
              {"kind": "alignment", "read": 0, "target": "GATG", "query": "GATG"}], moves=7, score_diff=nb),
        case("SmallMismatch", "src/Tests/TestRecursors.cpp:128-152", "GATG", [rd("GATC")],
             [{"kind": "baseline", "expected": -10.0},
              {"kind": "alignment", "read": 0, "target": "GATG", "query": "GATC"}], moves=7, score_diff=nb),
        case("SmallMerge", "src/Tests/TestRecursors.cpp:154-182", "GATT", [rd("GAT")],
             [{"kind": "baseline", "expected": -2.0},
              {"kind": "alignment", "read": 0, "target": "GATT", "query": "GA-T"}], moves=15, score_diff=nb),
        case("MediumSized", "src/Tests/TestRecursors.cpp:184-204 (FillAlphaBeta)", medium_tpl, [rd(medium_read)],
             [{"kind": "baseline", "expected": -80.0}], moves=7, score_diff=std),
        case("MutationScorer.Basic", "src/Tests/TestMutationScorer.cpp:100-124", "GATTACA", [rd("GATTACA")],
             [{"kind": "baseline", "expected": 0.0},
              ms(INS, 4, "A", P["Merge"]), ms(INS, 4, "G", P["DeletionN"]),
              ms(SUB, 4, "T", P["Mismatch"]), ms(DEL, 4, "-", P["Nce"])]),
        case("MutationScorer.AtBeginning", "src/Tests/TestMutationScorer.cpp:138-158", "GATTACA", [rd("GATTACA")],
             [ms(INS, 0, "A", P["DeletionN"]), ms(INS, 1, "G", P["Merge"]), ms(INS, 1, "A", P["Merge"]),
              ms(INS, 1, "T", P["DeletionN"]), ms(SUB, 0, "T", P["Mismatch"]), ms(DEL, 0, "-", P["Nce"])]),
        case("MutationScorer.AtEnd", "src/Tests/TestMutationScorer.cpp:160-176", "GATTACA", [rd("GATTACA")],
             [ms(INS, 7, "A", P["Merge"]), ms(INS, 7, "G", P["DeletionN"]), ms(SUB, 6, "T", P["Mismatch"]),
              ms(DEL, 6, "-", P["Nce"])]),
        case("MutationScorer.TinyTemplate", "src/Tests/TestMutationScorer.cpp:179-202", "GTGC", [rd("GTGC")],
             [ms(DEL, 0, "-", P["Nce"]), ms(DEL, 3, "-", P["Nce"]), ms(INS, 0, "T", P["DeletionN"]),
              ms(INS, 4, "T", P["DeletionN"])] + [ms(SUB, p, "A", P["Mismatch"]) for p in range(4)]),
        case("MRMS.Basic", "src/Tests/TestMultiReadMutationScorer.cpp:275-319 (FastScoreThreshold -500)",
             "TTGATTACATT", [rd("TTGATTACATT")],
             [sc(SUB, 6, "A", 0.0), sc(INS, 6, "A", P["Merge"]), sc(SUB, 6, "T", P["Mismatch"]),
              sc(DEL, 6, "-", P["Nce"]),
              {"kind": "add_read", "read": rd("TTGATTACATT")},
              sc(SUB, 6, "A", 0.0), sc(INS, 6, "A", -4.0), sc(SUB, 6, "T", -20.0), sc(DEL, 6, "-", -16.0),
              {"kind": "apply", "muts": [[INS, 6, "A"]], "template": "TTGATTAACATT"},
              sc(SUB, 6, "A", 0.0)], fast=-500.0),
        case("MRMS.ReverseStrand", "src/Tests/TestMultiReadMutationScorer.cpp:395-437", "AATGTAATCAA",
             [rd("TTGATTACATT", 1)],
             [sc(SUB, 4, "T", 0.0), sc(INS, 5, "T", P["Merge"]), sc(SUB, 4, "A", P["Mismatch"]),
              sc(DEL, 4, "-", P["Nce"]),
              {"kind": "add_read", "read": rd("TTGATTACATT", 1)},
              sc(SUB, 4, "T", 0.0), sc(INS, 5, "T", 2 * P["Merge"]), sc(SUB, 4, "A", 2 * P["Mismatch"]),
              sc(DEL, 4, "-", 2 * P["Nce"]),
              {"kind": "apply", "muts": [[INS, 5, "T"]], "template": "AATGTTAATCAA"},
              sc(SUB, 4, "T", 0.0)], fast=-500.0),
        case("MRMS.MutationsAtBeginning", "src/Tests/TestMultiReadMutationScorer.cpp:440-460", "TTGATTACATT",
             [rd("TTGATTACATT")],
             [sc(SUB, 0, "T", 0.0), sc(INS, 0, "A", 0.0), sc(INS, 1, "A", P["DeletionN"]),
              sc(DEL, 0, "-", P["Branch"])], fast=-500.0),
        case("MRMS.MutationsAtEnd", "src/Tests/TestMultiReadMutationScorer.cpp:462-483", "TTGATTACATT",
             [rd("TTGATTACATT")],
             [sc(SUB, 10, "T", 0.0), sc(INS, 11, "A", P["DeletionN"]), sc(INS, 12, "A", 0.0),
              sc(DEL, 10, "-", P["Branch"])], fast=-500.0),
    ]
    return {"params": P, "tolerance_abs": 0.0, "kats": kats}


def _cpp_statements(body):
    """Split C++ test code into statements; each is (text with literals replaced by @k, [literals]).
    Adjacent literals are concatenated (C++ translation phase 6); comments are dropped."""
    out, text, lits, i = [], "", [], 0
    while i < len(body):
        c = body[i]
        if body.startswith("//", i):
            i = body.index("\n", i)
            continue
        if body.startswith("/*", i):
            i = body.index("*/", i) + 2
            continue
        if c == '"':
            j, buf = i + 1, ""
            while body[j] != '"':
                if body[j] == "\\":
                    buf += body[j + 1]
                    j += 2
                else:
                    buf += body[j]
                    j += 1
            i = j + 1
            if text.rstrip().endswith("@%d" % (len(lits) - 1)) and lits:
                lits[-1] += buf
            else:
                text += "@%d" % len(lits)
                lits.append(buf)
            continue
        if c in ";{}":
            if text.strip():
                out.append((" ".join(text.split()), lits))
            text, lits = "", []
            i += 1
            continue
        text += c
        i += 1
    return out


def _tests(src):
    """TEST(Suite, Name) bodies of a gtest source, skipping #if 0 regions."""
    src = re.sub(r"#if 0.*?#endif", "", src, flags=re.S)
    tests = {}
    for m in re.finditer(r"TEST\((\w+), (\w+)\)\s*\{", src):
        depth, j = 1, m.end()
        while depth:
            depth += {"{": 1, "}": -1}.get(src[j], 0)
            j += 1
        tests[m.group(1) + "." + m.group(2)] = src[m.end():j - 1]
    return tests


def make_poa_kats():
    modes = {"GLOBAL": 0, "SEMIGLOBAL": 1, "LOCAL": 2}
    path = "ConsensusCore/src/Tests/TestPoaConsensus.cpp"
    cases = []
    for name, body in _tests(open(os.path.join(REF, path)).read()).items():
        cur = None
        for text, lits in _cpp_statements(body):
            if text.startswith("vector<std::string> reads") or text.startswith("std::vector<std::string> reads"):
                cur = {"test": name, "source": path, "reads": [], "mode": 0, "min_coverage": None,
                       "expected_dot": None, "graphviz_flags": 0, "expected": None}
            elif text.startswith("reads +="):
                cur["reads"] += lits
            elif "FindConsensus(reads" in text:
                m = re.search(r"FindConsensus\(reads, (\w+)(?:, (\d+))?\)", text)
                cur["mode"] = modes[m.group(1)]
                cur["min_coverage"] = int(m.group(2)) if m.group(2) else None
            elif text.startswith("string expectedDot"):
                cur["expected_dot"] = lits[0]
            elif "ToGraphViz(PoaGraph::COLOR_NODES | PoaGraph::VERBOSE_NODES" in text:
                cur["graphviz_flags"] = 3
            elif text.startswith("EXPECT_EQ(@0, pc->Sequence"):
                cur["expected"] = lits[0]
            elif text.startswith("delete pc") and "run" not in name.lower() and cur and cur not in cases:
                cases.append(cur)
            elif text.startswith("ASSERT_EQ(1, answers.size())"):
                cur["deterministic_only"] = True
    sp_path = "tests/TestSparsePoa.cpp"
    sparse = []
    for name, body in _tests(open(os.path.join(REF, sp_path)).read()).items():
        stmts = _cpp_statements(body)
        case = {"test": name, "source": sp_path, "reads": [], "summaries": {}}
        brace_init = False
        for text, lits in stmts:
            if text.startswith("reads +=") or brace_init:
                case["reads"] += lits
            brace_init = text.startswith("vector<std::string> reads =")
            m = re.search(r"FindConsensus\((\d+), &summaries\)", text)
            if m:
                case["min_coverage"] = int(m.group(1))
            if text.startswith("EXPECT_EQ(@0, consensusSeq"):
                case["expected"] = lits[0]
            m = re.match(r"EXPECT_EQ\(Interval\( ?(\d+), ?(\d+)\), summaries\[(\d+)\]\.ExtentOn(Read|Consensus)", text)
            if m:
                d = case["summaries"].setdefault(m.group(3), {})
                d["read" if m.group(4) == "Read" else "tpl"] = [int(m.group(1)), int(m.group(2))]
            m = re.match(r"EXPECT_(TRUE|FALSE) ?\(summaries\[(\d+)\]\.ReverseComplementedRead", text)
            if m and name in ("SparsePoaTest.TestLocalStaggered", "SparsePoaTest.TestOrientation"):
                case["summaries"].setdefault(m.group(2), {})["rc"] = m.group(1) == "TRUE"
        sparse.append(case)
    fasta = open(os.path.join(REF, "tests/data/m140905_042212_sidney_c100564852550000001823085912221377_s1_X0.fasta")).read()
    zmw = [ "".join(rec.split("\n")[1:]) for rec in fasta.split(">")[1:]]
    for c in sparse:
        if c["test"] == "SparsePoaTest.TestZmw6251":
            c["reads"] = zmw
            # EXPECTs (:169-194): 10 reads in the graph; summaries[0] is forward, summaries[1] reverse;
            # extent of read 0 covers [300, 595) and read 1 covers [5, 595) on the ~600 bp consensus.
            c["num_reads"] = 10
            c["covers"] = {"0": [300, 595], "1": [5, 595]}
            c["summaries"] = {"0": {"rc": False}, "1": {"rc": True}}
        if c["test"] in ("SparsePoaTest.SingleReadx100", "SparsePoaTest.SingleAndHalfx100"):
            c["generated"] = "orc_poa_kat_reads (std::mt19937(42) stream of the test)"
    return {"poa_consensus": cases, "sparse_poa": sparse}


def make_matrixtester_multiread():
    """MatrixTester::TestMultiReadScorer (MatrixTester.cpp:212-384): the reference's one real multi-read ZMW -- a
    222 bp template, SNR (15.49, 8.79, 13.52, 14.96) and 54 subreads with their strands and (often non-spanning)
    template windows, each AddRead at threshold 1.0, then Score(INSERTION 202 'C').  The demo prints the score
    and asserts nothing, so the fixture holds inputs only (parity against the restatement, not pinned)."""
    src = open(os.path.join(REF, "ConsensusCore/src/Demos/MatrixTester.cpp")).read()
    body = src[src.index("int MatrixTester::TestMultiReadScorer()"):]
    body = body[:body.index("return 0;")]
    tpl = re.search(r'std::string temp = "([ACGT]+)"', body).group(1)
    snr = [float(x) for x in re.search(r"SNR snr\(([^)]*)\)", body).group(1).split(",")]
    seqs = {int(k): (n, s) for k, n, s in re.findall(r'ArrowRead r(\d+) = MakeRead\("([^"]*)","([ACGT]*)"\);', body)}
    mapped = re.findall(r"MappedArrowRead mr(\d+)\(r(\d+), StrandEnum::(FORWARD|REVERSE)_STRAND, (\d+), (\d+), "
                        r"(true|false), (true|false) \);", body)
    adds = re.findall(r"scorer\.AddRead\(mr(\d+), ([0-9.]+)\);", body)
    mut = re.search(r"Mutation m\(MutationType::(\w+), (\d+), '([ACGT])'\);", body)
    by_mr = {int(m[0]): m for m in mapped}
    reads = []
    for k, thr in adds:
        m = by_mr[int(k)]
        name, seq = seqs[int(m[1])]
        reads.append({"name": name, "seq": seq, "strand": 1 if m[2] == "REVERSE" else 0, "ts": int(m[3]),
                      "te": int(m[4]), "pin_start": m[5] == "true", "pin_end": m[6] == "true",
                      "threshold": float(thr)})
    assert len(reads) == 54, len(reads)
    return {"source": "ConsensusCore/src/Demos/MatrixTester.cpp:212-384 (TestMultiReadScorer)",
            "tpl": tpl, "snr": snr, "reads": reads,
            "mutation": {"type": mut.group(1), "start": int(mut.group(2)), "base": mut.group(3)},
            "note": "inputs only: the demo prints Score(m) without an expected value (parity unpinned by the "
                    "reference; the GPU test compares with oracle/arrow_oracle.cpp)"}


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are committed, nothing to regenerate")
    with open(os.path.join(HERE, "arrow_kats.json"), "w") as f:
        json.dump(make_kats(), f, indent=1)
    with open(os.path.join(HERE, "zmw6251.json"), "w") as f:
        json.dump(make_zmw6251(), f, indent=1)
    with open(os.path.join(HERE, "quiver_kats.json"), "w") as f:
        json.dump(make_quiver_kats(), f, indent=1)
    with open(os.path.join(HERE, "poa_kats.json"), "w") as f:
        json.dump(make_poa_kats(), f, indent=1)
    with open(os.path.join(HERE, "matrixtester_multiread.json"), "w") as f:
        json.dump(make_matrixtester_multiread(), f, indent=1)
    print("wrote arrow_kats.json, zmw6251.json, quiver_kats.json, poa_kats.json, matrixtester_multiread.json")


if __name__ == "__main__":
    main()
