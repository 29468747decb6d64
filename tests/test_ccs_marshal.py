"""Host logic of pbccs_amd.driver.ccs_batch (CPU, no device): the flat subread buffer and pointer table, the per-ZMW
input / output structs filled column-wise through numpy views (nested pbccs_zmw_output, snr[4], status_counts[5]),
and the result decoding -- checked against a stand-in for pbccs_ccs_batch that reads and writes the structs through
their ctypes layout (include/pbccs_amd.h pbccs_ccs_input / pbccs_ccs_output)."""
import ctypes
import math

from pbccs_amd import driver
from pbccs_amd import lib as L


def _ptr(base, z, field_offset, size):
    return ctypes.c_void_p.from_address(base + z * size + field_offset).value


class _FakeLib:
    """pbccs_ccs_batch stand-in: status Success (0) for ZMWs with reads, NoSubreads (1) otherwise; consensus = the
    first read reversed, draft = the first read, qv k = k + z, add_read_results r = r, zscores r = r / 2 + snr[0],
    add_order = reads in reverse, and the scalars from z."""

    def pbccs_ccs_batch(self, h, ins, n, mc, opts, outs):
        obase = ctypes.cast(outs, ctypes.c_void_p).value
        osz = ctypes.sizeof(L.CCcsOutput)
        pol = L.CCcsOutput.polish.offset
        for z in range(n):
            i, o = ins[z], outs[z]
            reads = [ctypes.string_at(i.seqs[k], i.lens[k]).decode() for k in range(i.n_subreads)]
            assert [i.flags[k] for k in range(i.n_subreads)] == [(k % 3) + 1 for k in range(i.n_subreads)]
            p = o.polish
            if not reads:
                p.status = 1
                o.draft_len = 0
                continue
            cons, draft = reads[0][::-1], reads[0]
            assert len(cons) + 64 <= p.consensus_cap and o.draft_cap == p.consensus_cap
            ctypes.memmove(_ptr(obase, z, pol + L.CZmwOutput.consensus.offset, osz), cons.encode(), len(cons))
            ctypes.memmove(_ptr(obase, z, L.CCcsOutput.draft.offset, osz), draft.encode(), len(draft))
            p.status, p.consensus_len, o.draft_len = 0, len(cons), len(draft)
            for k in range(len(cons)):
                p.qvs[k] = k + z
            for r in range(len(reads)):
                p.add_read_results[r] = r
                p.zscores[r] = r / 2 + i.snr[0]
                o.add_order[r] = len(reads) - 1 - r
            p.zg, p.za, p.predicted_accuracy = z + 0.5, z + 0.25, 0.99
            p.n_tested, p.n_applied, p.n_passes = 1000 * z + (1 << 40), z, len(reads)
            for s in range(5):
                p.status_counts[s] = 10 * z + s
        return 0


class _Eng:
    _h = None


def test_ccs_batch_marshalling_round_trip(monkeypatch):
    monkeypatch.setattr(L, "load", lambda: _FakeLib())
    chunks = [{"snr": [4.0 + z, 5.0, 6.0, 7.0 + z],
               "reads": [{"seq": "ACGT" * (z + 1) + "A" * k, "flags": (k % 3) + 1} for k in range(nr)]}
              for z, nr in enumerate([3, 0, 1, 5, 2, 0, 0])]   # read-less ZMWs inside and at the end
    got = driver.ccs_batch(chunks, engine=_Eng())
    assert len(got) == len(chunks)
    for z, (c, g) in enumerate(zip(chunks, got)):
        reads = [r["seq"] for r in c["reads"]]
        if not reads:
            assert g["status"] == "NoSubreads" and not g["polished"] and g["consensus"] == "" and g["qvs"] == []
            continue
        assert g["status"] == "Success" and g["polished"]
        assert g["consensus"] == reads[0][::-1] and g["draft"] == reads[0]
        assert g["qvs"] == [k + z for k in range(len(reads[0]))]
        assert g["add_read_results"] == list(range(len(reads)))
        assert all(math.isclose(a, r / 2 + c["snr"][0]) for r, a in enumerate(g["zscores"]))
        assert g["add_order"] == list(range(len(reads)))[::-1]
        assert (g["zg"], g["za"], g["predicted_accuracy"]) == (z + 0.5, z + 0.25, 0.99)
        assert (g["n_tested"], g["n_applied"], g["n_passes"]) == (1000 * z + (1 << 40), z, len(reads))
        assert g["status_counts"] == [10 * z + s for s in range(5)]


def test_ccs_batch_non_ascii_lengths_in_bytes(monkeypatch):
    seen = []

    class Lib:
        def pbccs_ccs_batch(self, h, ins, n, mc, opts, outs):
            seen.extend(ins[0].lens[k] for k in range(ins[0].n_subreads))
            outs[0].polish.status = 1
            return 0

    monkeypatch.setattr(L, "load", lambda: Lib())
    driver.ccs_batch([{"snr": [1, 1, 1, 1], "reads": [{"seq": "ACé"}, {"seq": "GT"}]}], engine=_Eng())
    assert seen == [4, 2]
