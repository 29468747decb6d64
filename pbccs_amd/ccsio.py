"""ccs input/output around the polish path: subread grouping into ZMW chunks,
the CCS record and the results report of src/main/ccs.cpp.

The reference reads and writes PacBio BAM through pbbam, which is not vendored. Here:
- input is subread FASTA named `movie/hole/qStart_qEnd`, the naming of the reference's own test data
  (tests/data/m140905_..._X0.fasta); per-ZMW SNR and per-read flags come from the caller, because FASTA
  carries neither;
- output is the CCS record as a SAM text line with the same fields and tags as ccs.cpp:105-172 (samtools
  turns it into BAM), or FASTQ;
- the results report is ccs.cpp:233-262 line for line.
BAM parity is unpinned: no reference test holds a CCS BAM.
"""
import hashlib
import math

from . import ZMW_STATUS, QVsToASCII

# LocalContextFlags bits (pbbam LocalContextFlags.h): a full pass has an adapter on both sides
ADAPTER_BEFORE = 1
ADAPTER_AFTER = 2


def parse_subread_name(name):
    """`movie/hole/qStart_qEnd` -> (movie, hole, qStart, qEnd) (pbbam BamRecord::FullName layout)."""
    movie, hole, span = name.split()[0].rsplit("/", 2)
    qs, qe = span.split("_")
    return movie, int(hole), int(qs), int(qe)


def read_fasta(path):
    """FASTA records as (name, sequence) in file order."""
    out, name, seq = [], None, []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\r\n")
            if line.startswith(">"):
                if name is not None:
                    out.append((name, "".join(seq)))
                name, seq = line[1:].strip(), []
            elif line:
                seq.append(line.strip())
    if name is not None:
        out.append((name, "".join(seq)))
    return out


class ResultCounts:
    """ResultType<> counters (include/pacbio/ccs/Consensus.h:155-207)."""

    FIELDS = ("Success", "PoorSNR", "NoSubreads", "TooShort", "TooManyUnusable", "TooFewPasses",
              "NonConvergent", "PoorQuality", "Other")

    def __init__(self):
        for f in self.FIELDS:
            setattr(self, f, 0)

    def __iadd__(self, other):   # Consensus.h:181-193
        for f in self.FIELDS:
            setattr(self, f, getattr(self, f) + getattr(other, f))
        return self

    def total(self):   # Consensus.h:195-207
        return sum(getattr(self, f) for f in self.FIELDS)

    def add_status(self, status):
        """One polished ZMW by its status name (pbccs_amd.ZMW_STATUS)."""
        setattr(self, status, getattr(self, status) + 1)

    def report(self):
        """WriteResultsReport (src/main/ccs.cpp:233-262): `fixed << setprecision(2)` percentages.  Like the
        reference, `Other` is counted in the total but has no line of its own."""
        total = self.total()
        rows = [("Success -- CCS generated", self.Success),
                ("Failed -- Below SNR threshold", self.PoorSNR),
                ("Failed -- No usable subreads", self.NoSubreads),
                ("Failed -- Insert size too small", self.TooShort),
                ("Failed -- Not enough full passes", self.TooFewPasses),
                ("Failed -- Too many unusable subreads", self.TooManyUnusable),
                ("Failed -- CCS did not converge", self.NonConvergent),
                ("Failed -- CCS below minimum predicted accuracy", self.PoorQuality)]

        def pct(n):   # a double 0/0 prints as -nan or nan in the reference; an empty run reports 0.00 here
            return f"{100.0 * n / total:.2f}" if total else "nan"
        return "".join(f"{label},{n},{pct(n)}%\n" for label, n in rows)


def group_zmws(subreads, snr_of, min_snr=4.0, min_passes=3, min_read_score=0.75, read_score_of=None,
               flags_of=None):
    """The subread loop of src/main/ccs.cpp:402-475 over records in file order.

    subreads: iterable of (name, seq).  snr_of(movie, hole) -> 4 SNRs (A, C, G, T); read_score_of(name) ->
    read accuracy (default 1.0); flags_of(name) -> LocalContextFlags (default ADAPTER_BEFORE|ADAPTER_AFTER).
    Returns (chunks, counts): chunks = [{"movie", "hole", "snr", "reads": [{name, seq, qs, qe, flags}]}] in
    input order; counts = ResultCounts with the gates applied before polish (PoorSNR: min SNR below
    min_snr, ccs.cpp:442-447; TooFewPasses: fewer than min_passes subreads, ccs.cpp:413-420).
    """
    counts = ResultCounts()
    chunks = []
    hole_key, skip = None, False

    def close_last():
        if chunks and len(chunks[-1]["reads"]) < min_passes:
            counts.TooFewPasses += 1
            chunks.pop()

    for name, seq in subreads:
        movie, hole, qs, qe = parse_subread_name(name)
        if hole_key is None or hole_key != hole:   # ccs.cpp:411 compares the hole number only
            close_last()
            hole_key = hole
            snr = [float(x) for x in snr_of(movie, hole)]
            if min(snr) < min_snr:
                counts.PoorSNR += 1
                skip = True
            else:
                skip = False
                chunks.append({"movie": movie, "hole": hole, "snr": snr, "reads": []})
        if skip:
            continue
        score = read_score_of(name) if read_score_of else 1.0
        if float(score) < min_read_score:   # ccs.cpp:463 compares as float
            continue
        flags = flags_of(name) if flags_of else (ADAPTER_BEFORE | ADAPTER_AFTER)
        chunks[-1]["reads"].append({"name": name, "seq": seq, "qs": qs, "qe": qe, "flags": flags})
    close_last()
    return chunks, counts


def read_group_id(movie, read_type="CCS"):
    """pbbam MakeReadGroupId: the first 8 hex digits of MD5(movieName + "//" + readType) (unpinned: pbbam
    is not vendored; its published definition)."""
    return hashlib.md5(f"{movie}//{read_type}".encode()).hexdigest()[:8]


def _f32(x):
    """static_cast<float> then printed with the shortest round-trip text of that float."""
    import numpy as np
    return repr(float(np.float32(x))) if math.isfinite(x) else ("nan" if math.isnan(x) else
                                                               ("inf" if x > 0 else "-inf"))


def ccs_sam_record(movie, hole, result, snr):
    """The CCS record of src/main/ccs.cpp:105-172 as a SAM text line (unmapped, flag 4; MAPQ 255).

    result: one pbccs_amd polish result (status Success).  Tags in the reference's order: RG zm np rq sn pq
    za zs rs.  rq = int32(1000 * predAcc) (truncation, ccs.cpp:137); floats are the float32 casts.
    """
    name = f"{movie}/{hole}/ccs"
    qual = QVsToASCII(result["qvs"])
    # zs: ZScores().second -- one entry per read the scorer took (inactive ones NaN), in AddRead order
    # (MultiReadMutationScorer.hpp:208-260).  ccs_batch results index their per-read arrays by subread and carry
    # that order ("add_order": FilterReads' stable sort, Consensus.h:281); polish results are in AddRead order.
    if "add_order" in result:
        zs = [result["zscores"][k] for k in result["add_order"]]
    else:
        zs = [z for z, a in zip(result["zscores"], result["add_read_results"]) if a >= 0]
    tags = [f"RG:Z:{read_group_id(movie)}", f"zm:i:{int(hole)}", f"np:i:{int(result['n_passes'])}",
            f"rq:i:{int(1000 * result['predicted_accuracy'])}",
            "sn:B:f," + ",".join(_f32(s) for s in snr),
            f"pq:f:{_f32(result['predicted_accuracy'])}", f"za:f:{_f32(result['za'])}",
            "zs:B:f," + ",".join(_f32(z) for z in zs) if zs else "zs:B:f",
            "rs:B:i," + ",".join(str(int(c)) for c in result["status_counts"])]
    fields = [name, "4", "*", "0", "255", "*", "*", "0", "0", result["consensus"] or "*", qual or "*"]
    return "\t".join(fields + tags)


def sam_header(movies, program="ccs", version="pbccs_amd"):
    """@HD / @RG (READTYPE=CCS) / @PG lines for the records of ccs_sam_record (ccs.cpp:183-219)."""
    lines = ["@HD\tVN:1.5\tSO:unknown\tpb:3.0b7"]
    for m in movies:
        lines.append(f"@RG\tID:{read_group_id(m)}\tPL:PACBIO\tDS:READTYPE=CCS\tPU:{m}")
    lines.append(f"@PG\tID:{program}-{version}\tPN:{program}\tVN:{version}")
    return "\n".join(lines) + "\n"


def ccs_fastq_record(movie, hole, result):
    """`@movie/hole/ccs`, sequence, `+`, QVsToASCII(qvs)."""
    return f"@{movie}/{hole}/ccs\n{result['consensus']}\n+\n{QVsToASCII(result['qvs'])}\n"


def count_results(results, pre=None):
    """ResultCounts of polished ZMWs (one per result status), added to the pre-polish gate counts."""
    c = ResultCounts()
    if pre is not None:
        c += pre
    for r in results:
        c.add_status(r["status"] if r["status"] in ResultCounts.FIELDS else "Other")
    return c


__all__ = ["ADAPTER_AFTER", "ADAPTER_BEFORE", "ResultCounts", "ZMW_STATUS", "ccs_fastq_record", "ccs_sam_record",
           "count_results", "group_zmws", "parse_subread_name", "read_fasta", "read_group_id", "sam_header"]
