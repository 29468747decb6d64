"""BAM input/output around the polish path, without pbbam or htslib.

The reference reads subreads.bam and writes ccs.bam through pbbam (src/main/ccs.cpp:105-172, 393-480),
which is not vendored.  This module implements the two formats it needs from their
published specifications (SAMv1 §4: BGZF blocks, the BAM header and alignment records, typed aux tags)
with zlib:

- `BgzfWriter` / `BgzfReader`: gzip members of at most 64 KiB carrying the `BC` extra field, and the
  28-byte end-of-file block;
- `write_bam(path, header_text, records)` / `read_bam(path)`: the BAM header (no reference sequences:
  PacBio subread and CCS BAMs are unaligned) and records, each record given as a SAM text line
  (`sam_to_bam_record` / `bam_record_to_sam` convert both ways, tags with their SAM types);
- `read_subread_bam(path)` -> the subread records ccs.cpp's loop consumes (name movie/hole/qs_qe,
  sequence, `zm`, `qs`, `qe`, `sn`, `cx`, `rq`), and `group_subread_bam` feeds them to
  ccsio.group_zmws with the per-ZMW SNR, read accuracy and context flags taken from the tags, as
  ccs.cpp:402-475 takes them from pbbam's BamRecord;
- `write_ccs_bam(path, movies, records)`: ccsio.ccs_sam_record lines (ccs.cpp:105-172's fields and tag
  order, Bin 0, MAPQ 255, flag 4) as BAM.

BAM parity is unpinned: no reference test holds a BAM file.  The tests check round trips and the byte
layout against the specification (tests/test_bamio.py).
"""
import struct
import zlib

_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
_MAX_BLOCK = 0xff00          # uncompressed bytes per BGZF block (htslib's BGZF_BLOCK_SIZE)
_SEQ_CODES = "=ACMGRSVTWYHKDBN"
_SEQ_INDEX = {c: i for i, c in enumerate(_SEQ_CODES)}
_B_TYPES = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}


class BgzfWriter:
    """BGZF stream (SAMv1 §4.1): deflate members with the BC extra subfield holding the block size - 1."""

    def __init__(self, path, level=6):
        self._f = open(path, "wb")
        self._buf = bytearray()
        self._level = level

    def tell(self):
        """BGZF virtual offset of the next byte written: compressed offset of its block << 16 | offset inside it."""
        return (self._f.tell() << 16) | len(self._buf)

    def write(self, data):
        self._buf += data
        while len(self._buf) >= _MAX_BLOCK:
            self._block(bytes(self._buf[:_MAX_BLOCK]))
            del self._buf[:_MAX_BLOCK]

    def _block(self, raw):
        c = zlib.compressobj(self._level, zlib.DEFLATED, -15)
        cdata = c.compress(raw) + c.flush()
        bsize = 18 + len(cdata) + 8   # header (12 + 6 extra) + data + CRC32/ISIZE
        hdr = struct.pack("<BBBBIBBHBBHH", 0x1f, 0x8b, 8, 4, 0, 0, 0xff, 6, ord("B"), ord("C"), 2, bsize - 1)
        self._f.write(hdr + cdata + struct.pack("<II", zlib.crc32(raw) & 0xffffffff, len(raw)))

    def close(self):
        if self._buf:
            self._block(bytes(self._buf))
            self._buf = bytearray()
        self._f.write(_BGZF_EOF)
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class BgzfReader:
    """The concatenated payload of a BGZF file, block by block (checks each block's CRC and size)."""

    def __init__(self, path):
        self._f = open(path, "rb")

    def blocks(self):
        while True:
            hdr = self._f.read(12)
            if not hdr:
                return
            if len(hdr) < 12 or hdr[:4] != b"\x1f\x8b\x08\x04":
                raise ValueError("not a BGZF block")
            xlen = struct.unpack("<H", hdr[10:12])[0]
            extra = self._f.read(xlen)
            bsize = None
            k = 0
            while k < xlen:
                si1, si2, slen = extra[k], extra[k + 1], struct.unpack("<H", extra[k + 2:k + 4])[0]
                if si1 == ord("B") and si2 == ord("C"):
                    bsize = struct.unpack("<H", extra[k + 4:k + 6])[0] + 1
                k += 4 + slen
            if bsize is None:
                raise ValueError("BGZF block without a BC field")
            cdata = self._f.read(bsize - 12 - xlen - 8)
            crc, isize = struct.unpack("<II", self._f.read(8))
            raw = zlib.decompress(cdata, -15)
            if len(raw) != isize or (zlib.crc32(raw) & 0xffffffff) != crc:
                raise ValueError("BGZF block CRC / size mismatch")
            yield raw

    def read_all(self):
        return b"".join(self.blocks())

    def close(self):
        self._f.close()


# ---------------------------------------------------------------------------------------------- records
def _reg2bin(beg, end):   # SAMv1 §5.3
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def _encode_tag(tag):
    """`TG:T:value` (SAM text) -> BAM aux bytes.  Integers keep type 'i' (int32), as pbbam writes int32_t
    tags; B arrays keep their subtype."""
    name, typ, val = tag.split(":", 2)
    out = name.encode()
    if typ == "i":
        return out + b"i" + struct.pack("<i", int(val))
    if typ == "f":
        return out + b"f" + struct.pack("<f", float(val))
    if typ == "A":
        return out + b"A" + val.encode()[:1]
    if typ in ("Z", "H"):
        return out + typ.encode() + val.encode() + b"\0"
    if typ == "B":
        parts = val.split(",")
        sub, vals = parts[0], parts[1:]
        conv = float if sub == "f" else int
        return out + b"B" + sub.encode() + struct.pack("<I", len(vals)) + \
            struct.pack("<%d%s" % (len(vals), _B_TYPES[sub]), *[conv(v) for v in vals])
    raise ValueError(f"unsupported tag type {typ}")


def _f32_text(x):
    import numpy as np
    return repr(float(np.float32(x)))


def _decode_tags(buf, k):
    tags = []
    while k < len(buf):
        name = buf[k:k + 2].decode()
        t = chr(buf[k + 2])
        k += 3
        if t in "cCsSiI":
            fmt = {"c": "<b", "C": "<B", "s": "<h", "S": "<H", "i": "<i", "I": "<I"}[t]
            v = struct.unpack_from(fmt, buf, k)[0]
            k += struct.calcsize(fmt)
            tags.append(f"{name}:i:{v}")
        elif t == "f":
            tags.append(f"{name}:f:{_f32_text(struct.unpack_from('<f', buf, k)[0])}")
            k += 4
        elif t == "A":
            tags.append(f"{name}:A:{chr(buf[k])}")
            k += 1
        elif t in "ZH":
            e = buf.index(b"\0", k)
            tags.append(f"{name}:{t}:{buf[k:e].decode()}")
            k = e + 1
        elif t == "B":
            sub = chr(buf[k])
            n = struct.unpack_from("<I", buf, k + 1)[0]
            k += 5
            fmt = "<%d%s" % (n, _B_TYPES[sub])
            vals = struct.unpack_from(fmt, buf, k)
            k += struct.calcsize(fmt)
            txt = [_f32_text(v) for v in vals] if sub == "f" else [str(v) for v in vals]
            tags.append(f"{name}:B:{sub}" + "".join("," + x for x in txt))
        else:
            raise ValueError(f"unknown aux type {t}")
    return tags


def sam_to_bam_record(line, bin_=None):
    """One SAM text line (no reference sequences: RNAME '*', CIGAR '*') -> the BAM record bytes including
    block_size.  bin_ overrides the computed bin (ccs.cpp sets Bin(0) on its unmapped records)."""
    f = line.rstrip("\n").split("\t")
    qname, flag, rname, pos, mapq, cigar, rnext, pnext, tlen, seq, qual = f[:11]
    if rname != "*" or cigar != "*":
        raise ValueError("only unaligned records (RNAME and CIGAR '*')")
    seq = "" if seq == "*" else seq
    lseq = len(seq)
    packed = bytearray((lseq + 1) // 2)
    for i, c in enumerate(seq):
        packed[i >> 1] |= _SEQ_INDEX.get(c.upper(), 15) << (4 if i % 2 == 0 else 0)
    qb = bytes([0xff] * lseq) if qual == "*" else bytes(ord(c) - 33 for c in qual)
    if len(qb) != lseq:
        raise ValueError("QUAL length differs from SEQ length")
    name = qname.encode() + b"\0"
    p = int(pos) - 1
    bin_ = _reg2bin(p, p + 1) if bin_ is None else bin_
    core = struct.pack("<iiBBHHHIiii", -1, p, len(name), int(mapq), bin_, 0, int(flag), lseq,
                       -1 if rnext == "*" else 0, int(pnext) - 1, int(tlen))
    body = core + name + bytes(packed) + qb + b"".join(_encode_tag(t) for t in f[11:])
    return struct.pack("<i", len(body)) + body


def bam_record_to_sam(rec):
    """BAM record bytes (without block_size) -> the SAM text line."""
    (ref, pos, lname, mapq, _bin, ncig, flag, lseq, nref, npos, tlen) = struct.unpack_from("<iiBBHHHIiii", rec, 0)
    k = 32
    name = rec[k:k + lname - 1].decode()
    k += lname + 4 * ncig
    seq = "".join(_SEQ_CODES[(rec[k + (i >> 1)] >> (4 if i % 2 == 0 else 0)) & 15] for i in range(lseq))
    k += (lseq + 1) // 2
    q = rec[k:k + lseq]
    k += lseq
    qual = "*" if lseq == 0 or all(b == 0xff for b in q) else "".join(chr(b + 33) for b in q)
    fields = [name, str(flag), "*", str(pos + 1), str(mapq), "*", "*" if nref < 0 else "=", str(npos + 1),
              str(tlen), seq or "*", qual]
    return "\t".join(fields + _decode_tags(rec, k))


def write_bam(path, header_text, sam_lines, bin_=None):
    """Returns each record's BGZF virtual offset (the offsets pbbam's BamWriter::Write reports)."""
    offsets = []
    with BgzfWriter(path) as w:
        ht = header_text.encode()
        w.write(b"BAM\1" + struct.pack("<i", len(ht)) + ht + struct.pack("<i", 0))
        for line in sam_lines:
            offsets.append(w.tell())
            w.write(sam_to_bam_record(line, bin_))
    return offsets


def read_bam(path):
    """(header_text, [SAM text lines])"""
    r = BgzfReader(path)
    data = r.read_all()
    r.close()
    if data[:4] != b"BAM\1":
        raise ValueError("not a BAM file")
    lt = struct.unpack_from("<i", data, 4)[0]
    header = data[8:8 + lt].decode().rstrip("\0")
    k = 8 + lt
    nref = struct.unpack_from("<i", data, k)[0]
    k += 4
    for _ in range(nref):
        ln = struct.unpack_from("<i", data, k)[0]
        k += 4 + ln + 4
    lines = []
    while k < len(data):
        bs = struct.unpack_from("<i", data, k)[0]
        lines.append(bam_record_to_sam(data[k + 4:k + 4 + bs]))
        k += 4 + bs
    return header, lines


# ---------------------------------------------------------------------------------------- ccs front/back
def _tag_dict(tags):
    d = {}
    for t in tags:
        name, typ, val = t.split(":", 2)
        if typ == "i":
            d[name] = int(val)
        elif typ == "f":
            d[name] = float(val)
        elif typ == "B":
            parts = val.split(",")
            d[name] = [float(x) if parts[0] == "f" else int(x) for x in parts[1:]]
        else:
            d[name] = val
    return d


def read_subread_bam(path):
    """Subread records as ccs.cpp:402-475 reads them through pbbam: [{name, seq, hole, qs, qe, snr, flags,
    read_score}] in file order (name = movie/hole/qs_qe; snr from `sn`, flags from `cx`, read score from
    `rq`, defaults when a tag is absent: full pass, score 1.0)."""
    _, lines = read_bam(path)
    out = []
    for line in lines:
        f = line.split("\t")
        t = _tag_dict(f[11:])
        out.append({"name": f[0], "seq": "" if f[9] == "*" else f[9], "hole": t.get("zm"), "qs": t.get("qs"),
                    "qe": t.get("qe"), "snr": t.get("sn"), "flags": t.get("cx", 3), "read_score": t.get("rq", 1.0)})
    return out


def group_subread_bam(path, min_snr=4.0, min_passes=3, min_read_score=0.75):
    """ccsio.group_zmws over a subread BAM: per-ZMW SNR from the first record of the hole (ccs.cpp:431),
    read accuracy and LocalContextFlags per record."""
    from . import ccsio
    recs = read_subread_bam(path)
    by_name = {r["name"]: r for r in recs}
    first_snr = {}
    for r in recs:
        movie, hole, _, _ = ccsio.parse_subread_name(r["name"])
        first_snr.setdefault((movie, hole), r["snr"])
    return ccsio.group_zmws([(r["name"], r["seq"]) for r in recs], lambda m, h: first_snr[(m, h)], min_snr,
                            min_passes, min_read_score, read_score_of=lambda n: by_name[n]["read_score"],
                            flags_of=lambda n: by_name[n]["flags"])


def write_ccs_bam(path, movies, sam_lines, pbi=False):
    """ccs.bam: ccsio.sam_header + ccsio.ccs_sam_record lines, with Bin(0) as ccs.cpp:113 sets it.  pbi: also
    write path + ".pbi" from each record's virtual offset (ccs.cpp:164-169,386, pbccs_amd.pbi)."""
    from . import ccsio
    sam_lines = list(sam_lines)
    offsets = write_bam(path, ccsio.sam_header(movies), sam_lines, bin_=0)
    if pbi:
        from .pbi import pbi_entry, write_pbi
        write_pbi(path + ".pbi", [pbi_entry(line, off) for line, off in zip(sam_lines, offsets)])


def subread_sam_line(movie, hole, qs, qe, seq, snr, flags=3, read_score=0.9, rg="00000000"):
    """A PacBio subread record as SAM text (the tags ccs.cpp reads), for building test inputs."""
    sn = ",".join(_f32_text(x) for x in snr)
    return "\t".join([f"{movie}/{hole}/{qs}_{qe}", "4", "*", "0", "255", "*", "*", "0", "0", seq, "*",
                      f"RG:Z:{rg}", f"zm:i:{hole}", f"qs:i:{qs}", f"qe:i:{qe}", f"sn:B:f,{sn}", f"cx:i:{flags}",
                      f"rq:f:{_f32_text(read_score)}"])


__all__ = ["BgzfReader", "BgzfWriter", "bam_record_to_sam", "group_subread_bam", "read_bam", "read_subread_bam",
           "sam_to_bam_record", "subread_sam_line", "write_bam", "write_ccs_bam"]
