"""ccs I/O around the polish path (pbccs_amd/ccsio.py): subread FASTA grouping with the ccs.cpp gates, the
results report, and the CCS SAM/FASTQ records.  Input data: the reference's own test subreads (ZMW 6251, kept
as a fixture in tests/golden/zmw6251.json)."""
import json
import os

import pytest

from pbccs_amd import ccsio

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def z6251():
    return json.load(open(os.path.join(GOLD, "zmw6251.json")))


def _fasta(tmp_path, recs, width=60):
    p = tmp_path / "subreads.fasta"
    with open(p, "w") as f:
        for name, seq in recs:
            f.write(f">{name}\n")
            for i in range(0, len(seq), width):
                f.write(seq[i:i + width] + "\n")
    return str(p)


def test_fasta_roundtrip_and_names(tmp_path, z6251):
    recs = [(r["name"], r["seq"]) for r in z6251["all_subreads"]]
    assert ccsio.read_fasta(_fasta(tmp_path, recs)) == recs
    movie, hole, qs, qe = ccsio.parse_subread_name(recs[1][0])
    assert (movie.endswith("_s1_X0"), hole, qs, qe) == (True, 6251, 525, 1145)


def test_grouping_gates(z6251):
    recs = [(r["name"], r["seq"]) for r in z6251["all_subreads"]]
    movie = ccsio.parse_subread_name(recs[0][0])[0]
    # ZMW 6251 as is, a second hole with only two subreads (TooFewPasses), a third below the SNR gate
    two = [(f"{movie}/7/0_100", "ACGT" * 25), (f"{movie}/7/150_250", "ACGT" * 25)]
    poor = [(f"{movie}/8/0_100", "ACGT" * 25)] * 4
    snr = {6251: z6251["snr"], 7: [8, 8, 8, 8], 8: [3.9, 8, 8, 8]}
    chunks, counts = ccsio.group_zmws(recs + two + poor, lambda m, h: snr[h])
    assert [c["hole"] for c in chunks] == [6251]
    assert [r["name"] for r in chunks[0]["reads"]] == [n for n, _ in recs]
    assert (counts.TooFewPasses, counts.PoorSNR, counts.total()) == (1, 1, 2)
    # the read-accuracy filter drops single reads, not the ZMW
    chunks, _ = ccsio.group_zmws(recs, lambda m, h: snr[h], read_score_of=lambda n: 0.5 if n == recs[3][0] else 0.9)
    assert len(chunks[0]["reads"]) == len(recs) - 1


def test_results_report_format():
    c = ccsio.ResultCounts()
    c.Success, c.PoorSNR, c.TooFewPasses, c.Other = 5, 1, 1, 1
    lines = c.report().splitlines()
    assert lines[0] == "Success -- CCS generated,5,62.50%"
    assert lines[1] == "Failed -- Below SNR threshold,1,12.50%"
    assert lines[4] == "Failed -- Not enough full passes,1,12.50%"
    assert lines[7] == "Failed -- CCS below minimum predicted accuracy,0,0.00%"
    assert len(lines) == 8
    d = ccsio.ResultCounts()
    d += c
    d += c
    assert d.total() == 16


def test_ccs_records():
    res = {"consensus": "ACGTA", "qvs": [10, 20, 93, 100, -3], "n_passes": 7, "predicted_accuracy": 0.99876,
           "za": -0.25, "zscores": [0.5, float("nan"), -1.25, float("nan")], "add_read_results": [0, 3, 0, -1],
           "status_counts": [2, 0, 0, 1, 0]}
    f = ccsio.ccs_sam_record("mov", 42, res, [10.0, 7.0, 5.0, 11.0]).split("\t")
    assert f[:11] == ["mov/42/ccs", "4", "*", "0", "255", "*", "*", "0", "0", "ACGTA", "+5~~!"]
    tags = f[11:]
    assert [t[:2] for t in tags] == ["RG", "zm", "np", "rq", "sn", "pq", "za", "zs", "rs"]
    assert tags[0] == "RG:Z:" + ccsio.read_group_id("mov") and len(tags[0]) == 13
    assert tags[1:4] == ["zm:i:42", "np:i:7", "rq:i:998"]
    assert tags[4] == "sn:B:f,10.0,7.0,5.0,11.0"
    assert tags[7] == "zs:B:f,0.5,nan,-1.25" and tags[8] == "rs:B:i,2,0,0,1,0"
    assert ccsio.ccs_fastq_record("mov", 42, res) == "@mov/42/ccs\nACGTA\n+\n+5~~!\n"
    assert ccsio.sam_header(["mov"]).startswith("@HD\tVN:1.5")
