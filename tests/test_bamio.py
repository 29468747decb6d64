"""BAM I/O without pbbam (pbccs_amd/bamio.py): BGZF framing checked against Python's own gzip decoder and
the SAMv1 layout, SAM <-> BAM record round trips of the CCS records ccs.cpp writes, and subread BAM input
through ccs.cpp's grouping gates.  BAM parity with the reference is unpinned (no reference test holds a
BAM); these are format and round-trip checks.  CPU only, except the end-to-end GPU case at the bottom."""
import gzip
import os
import random
import struct

import pytest

from pbccs_amd import bamio, ccsio


def test_bgzf_blocks_decode_with_gzip(tmp_path):
    rng = random.Random(3)
    payload = bytes(rng.getrandbits(8) for _ in range(200_000)) + b"A" * 150_000
    p = tmp_path / "x.bgzf"
    with bamio.BgzfWriter(str(p)) as w:
        w.write(payload[:1000])
        w.write(payload[1000:])
    raw = p.read_bytes()
    assert gzip.decompress(raw) == payload                      # a valid multi-member gzip stream
    assert raw.endswith(bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000"))
    r = bamio.BgzfReader(str(p))
    blocks = list(r.blocks())
    r.close()
    assert b"".join(blocks) == payload and all(len(b) <= 0xff00 for b in blocks) and blocks[-1] == b""


def _ccs_result():
    return {"status": "Success", "consensus": "ACGTTGCANACGT", "qvs": [30, 40, 93, 12, 0, 5, 60, 61, 62, 63, 70, 80, 90],
            "add_read_results": [0, 0, 3, 0], "zscores": [0.5, -1.25, float("nan"), 2.0], "za": 0.41666,
            "predicted_accuracy": 0.9987654, "n_passes": 3, "status_counts": [3, 0, 0, 1, 0]}


def test_ccs_record_round_trip_and_layout(tmp_path):
    line = ccsio.ccs_sam_record("m140905_42", 6251, _ccs_result(), [10.0, 7.0, 5.0, 11.5])
    rec = bamio.sam_to_bam_record(line, bin_=0)
    size = struct.unpack_from("<i", rec)[0]
    assert size == len(rec) - 4
    ref, pos, lname, mapq, bin_, ncig, flag, lseq, nref, npos, tlen = struct.unpack_from("<iiBBHHHIiii", rec, 4)
    assert (ref, pos, mapq, bin_, ncig, flag, lseq, nref, npos, tlen) == (-1, -1, 255, 0, 0, 4, 13, -1, -1, 0)
    assert rec[36:36 + lname] == b"m140905_42/6251/ccs\0"
    seq = rec[36 + lname:36 + lname + 7]
    assert seq[0] == (1 << 4) | 2 and seq[4] == (15 << 4) | 1          # A C ... N A (4-bit codes, high nibble first)
    assert bamio.bam_record_to_sam(rec[4:]) == line
    p = tmp_path / "ccs.bam"
    bamio.write_ccs_bam(str(p), ["m140905_42"], [line, line.replace("/6251/", "/7000/").replace("zm:i:6251", "zm:i:7000")])
    header, lines = bamio.read_bam(str(p))
    assert header == ccsio.sam_header(["m140905_42"])
    assert lines[0] == line and "zm:i:7000" in lines[1]
    assert gzip.decompress(p.read_bytes())[:4] == b"BAM\1"


def test_pbi_index_round_trip_and_offsets(tmp_path):
    """ccs.bam + .pbi (ccs.cpp --pbi): the index holds one basic-data entry per record in file order (rgId from
    the read-group hex id, qStart/qEnd -1, holeNumber = zm, readQual = rq / 1000, ctxtFlag 0), and every
    fileOffset is a BGZF virtual offset that lands on its record -- checked across block boundaries with
    records large enough to span several 64 KiB blocks."""
    import zlib
    from pbccs_amd import pbi
    rng = random.Random(11)
    lines = []
    for k in range(40):
        res = dict(_ccs_result())
        L = rng.choice([13, 500, 9000, 70000])
        res["consensus"] = "".join(rng.choice("ACGT") for _ in range(L))
        res["qvs"] = [rng.randint(0, 93) for _ in range(L)]
        res["predicted_accuracy"] = rng.uniform(0.9, 1.0)
        lines.append(ccsio.ccs_sam_record("m140905_42", 1000 + 7 * k, res, [10.0, 7.0, 5.0, 11.5]))
    p = tmp_path / "ccs.bam"
    bamio.write_ccs_bam(str(p), ["m140905_42"], lines, pbi=True)
    idx = pbi.read_pbi(str(p) + ".pbi")
    assert idx["version"] == 0x030001 and idx["flags"] == 0 and idx["n_reads"] == len(lines)
    rg = int(ccsio.read_group_id("m140905_42"), 16)
    assert idx["rg_id"] == [rg - (1 << 32) if rg >= 1 << 31 else rg] * len(lines)
    assert idx["q_start"] == [-1] * len(lines) and idx["q_end"] == [-1] * len(lines)
    assert idx["hole_number"] == [1000 + 7 * k for k in range(len(lines))]
    assert idx["ctxt_flag"] == [0] * len(lines)
    for q, line in zip(idx["read_qual"], lines):
        rq = int(line.split("rq:i:")[1].split("\t")[0])
        assert abs(q - rq / 1000.0) < 1e-6
    raw = p.read_bytes()
    offs = idx["file_offset"]
    assert offs == sorted(offs) and len(set(offs)) == len(offs)
    for off, line in zip(offs, lines):
        coff, uoff = off >> 16, off & 0xffff
        # inflate from the record's block on: enough blocks for the record's 4-byte size and body
        data, k = b"", coff
        while len(data) < uoff + 4 or len(data) < uoff + 4 + struct.unpack_from("<i", data, uoff)[0]:
            xlen = struct.unpack_from("<H", raw, k + 10)[0]
            bsize = struct.unpack_from("<H", raw, k + 12 + 4)[0] + 1
            data += zlib.decompress(raw[k + 12 + xlen:k + bsize - 8], -15)
            k += bsize
        size = struct.unpack_from("<i", data, uoff)[0]
        assert bamio.bam_record_to_sam(data[uoff + 4:uoff + 4 + size]) == line


def test_subread_bam_grouping_matches_fasta_path(tmp_path):
    """group_subread_bam applies ccs.cpp's gates (PoorSNR, read score, TooFewPasses) with the tags' values,
    exactly as group_zmws does given the same values."""
    rng = random.Random(9)
    recs, snrs, scores, flags = [], {}, {}, {}
    for hole, (snr, n) in enumerate([((10, 7, 5, 11), 5), ((3.5, 8, 8, 8), 4), ((9, 9, 9, 9), 2), ((6, 6, 6, 6), 6)]):
        snrs[hole] = snr
        for k in range(n):
            seq = "".join(rng.choice("ACGT") for _ in range(rng.randint(50, 90)))
            qs = 100 * k
            name = f"mv/{hole}/{qs}_{qs + len(seq)}"
            scores[name] = 0.7 if (hole == 3 and k == 1) else 0.9
            flags[name] = 3 if k % 3 else 1
            recs.append(bamio.subread_sam_line("mv", hole, qs, qs + len(seq), seq, snr, flags[name], scores[name]))
    p = tmp_path / "subreads.bam"
    bamio.write_bam(str(p), "@HD\tVN:1.5\tSO:unknown\n", recs)
    chunks, counts = bamio.group_subread_bam(str(p))
    names = [r.split("\t")[0] for r in recs]
    seqs = [r.split("\t")[9] for r in recs]
    import numpy as np
    exp_chunks, exp_counts = ccsio.group_zmws(
        list(zip(names, seqs)), lambda m, h: [float(np.float32(x)) for x in snrs[h]],
        read_score_of=lambda n: float(np.float32(scores[n])), flags_of=lambda n: flags[n])
    assert chunks == exp_chunks
    assert (counts.PoorSNR, counts.TooFewPasses) == (exp_counts.PoorSNR, exp_counts.TooFewPasses) == (1, 1)
    assert [c["hole"] for c in chunks] == [0, 3] and len(chunks[1]["reads"]) == 5


@pytest.mark.gpu
def test_subread_bam_to_ccs_bam_on_gpu(tmp_path):
    """subreads.bam -> grouping gates -> FilterReads + POA + ExtractMappedRead (GPU) -> polish (GPU) ->
    ccs.bam; the BAM's records equal the SAM text records of the same results."""
    import pbccs_amd
    from pbccs_amd import driver, synth
    zs = synth.make_zmws(4, 400, 6, seed=77)
    lines = []
    for hole, z in enumerate(zs):
        qs = 0
        for r in z["reads"]:
            lines.append(bamio.subread_sam_line("mvB", hole, qs, qs + len(r["seq"]), r["seq"], z["snr"]))
            qs += len(r["seq"]) + 40
    p = tmp_path / "subreads.bam"
    bamio.write_bam(str(p), "@HD\tVN:1.5\tSO:unknown\n", lines)
    chunks, counts = bamio.group_subread_bam(str(p))
    assert len(chunks) == 4 and counts.PoorSNR == 0
    ins = driver.zmw_inputs_batch(chunks)
    zmws = [z for st, z in ins if st is None]
    res = pbccs_amd.polish_zmws(zmws)
    sam = [ccsio.ccs_sam_record("mvB", c["hole"], r, c["snr"]) for c, r in zip(chunks, res) if r["status"] == "Success"]
    assert sam
    out = tmp_path / "ccs.bam"
    bamio.write_ccs_bam(str(out), ["mvB"], sam)
    header, back = bamio.read_bam(str(out))
    assert back == sam
