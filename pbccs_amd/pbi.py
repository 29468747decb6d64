"""PacBio BAM index (.pbi) for ccs.bam -- ccs.cpp's `--pbi` (src/main/ccs.cpp:54,164-169,381-389: one
PbiBuilder::AddRecord(record, offset) per written CCS record, the file named OUTPUT + ".pbi").

pbbam (un-vendored, unpinned: CMakeLists.txt:53 points at a local checkout, CI clones its HEAD) owns the
format.  Restated from its published PBI specification (version 3.0.1, the basic-data section; ccs.bam is
unaligned, unbarcoded and unsorted, so pbi_flags = 0 and no mapped / coordinate / barcode sections):

    BGZF stream of
      header   magic "PBI\\1" | version uint32 (0x030001) | pbi_flags uint16 | n_reads uint32 | 18 reserved bytes
      basic    rgId int32[n] | qStart int32[n] | qEnd int32[n] | holeNumber int32[n] | readQual float[n]
               | ctxtFlag uint8[n] | fileOffset int64[n]        (each field one array, little endian)

  rgId = int32 of the 8-hex-digit read-group id; qStart / qEnd = -1 for CCS records (no qs/qe tags);
  holeNumber = zm; readQual = rq as accuracy in [0, 1] (this ccs writes rq as int32 1000 * predAcc,
  ccs.cpp:137); ctxtFlag = cx (0 when absent); fileOffset = the record's BGZF virtual offset
  (compressed block offset << 16 | offset inside the block).

Parity unpinned: no reference test or fixture holds a .pbi; tests/test_bamio.py checks the layout against
this restatement and that every fileOffset seeks to its record.
"""
import struct

from .bamio import BgzfWriter

PBI_MAGIC = b"PBI\x01"
PBI_VERSION = 0x030001
PBI_HEADER_BYTES = 32


def _int32(u):
    return u - (1 << 32) if u >= 1 << 31 else u


def pbi_entry(sam_line, offset):
    """The basic-data fields of one record (its SAM text line) written at BGZF virtual offset `offset`."""
    f = sam_line.rstrip("\n").split("\t")
    tags = {}
    for t in f[11:]:
        name, typ, val = t.split(":", 2)
        tags[name] = (typ, val)
    rg = _int32(int(tags["RG"][1], 16)) if "RG" in tags else -1
    q_start = int(tags["qs"][1]) if "qs" in tags else -1
    q_end = int(tags["qe"][1]) if "qe" in tags else -1
    hole = int(tags["zm"][1]) if "zm" in tags else -1
    if "rq" in tags:
        typ, val = tags["rq"]
        qual = int(val) / 1000.0 if typ == "i" else float(val)
    else:
        qual = 0.0
    cx = int(tags["cx"][1]) if "cx" in tags else 0
    return (rg, q_start, q_end, hole, qual, cx, offset)


def write_pbi(path, entries):
    """entries: pbi_entry tuples in file order."""
    n = len(entries)
    cols = list(zip(*entries)) if n else [()] * 7
    body = bytearray()
    body += PBI_MAGIC + struct.pack("<IHI", PBI_VERSION, 0, n) + bytes(18)
    body += struct.pack(f"<{n}i", *cols[0])
    body += struct.pack(f"<{n}i", *cols[1])
    body += struct.pack(f"<{n}i", *cols[2])
    body += struct.pack(f"<{n}i", *cols[3])
    body += struct.pack(f"<{n}f", *cols[4])
    body += struct.pack(f"<{n}B", *cols[5])
    body += struct.pack(f"<{n}q", *cols[6])
    with BgzfWriter(path) as w:
        w.write(bytes(body))


def read_pbi(path):
    """{"version", "flags", "n_reads", "rg_id", "q_start", "q_end", "hole_number", "read_qual", "ctxt_flag",
    "file_offset"}"""
    from .bamio import BgzfReader
    r = BgzfReader(path)
    data = r.read_all()
    r.close()
    if data[:4] != PBI_MAGIC:
        raise ValueError("not a PacBio BAM index")
    version, flags, n = struct.unpack_from("<IHI", data, 4)
    k = PBI_HEADER_BYTES
    out = {"version": version, "flags": flags, "n_reads": n}
    for name, fmt, size in (("rg_id", "i", 4), ("q_start", "i", 4), ("q_end", "i", 4), ("hole_number", "i", 4),
                            ("read_qual", "f", 4), ("ctxt_flag", "B", 1), ("file_offset", "q", 8)):
        out[name] = list(struct.unpack_from(f"<{n}{fmt}", data, k))
        k += n * size
    if k != len(data):
        raise ValueError("trailing bytes in the index (flags other than basic data are not written here)")
    return out


__all__ = ["PBI_VERSION", "pbi_entry", "read_pbi", "write_pbi"]
