"""Host logic of pbccs_amd.poa.poa_batch (CPU, no device): the flat read buffer, the per-ZMW input / output structs
filled column-wise through numpy views, and the result decoding -- checked against a stand-in for the native
entry point that reads the structs through their ctypes layout (include/pbccs_amd.h pbccs_poa_input/output)."""
import ctypes

import pbccs_amd.poa as poa
from pbccs_amd import lib as L


class _FakeLib:
    """pbccs_poa_batch stand-in: consensus = the ZMW's non-null reads joined, key k for read k (-1 for a dropped
    read), rc = key parity, extents (10k .. 10k+3)."""

    def pbccs_poa_batch(self, h, ins, n, mc, minc, outs):
        base = ctypes.cast(outs, ctypes.c_void_p).value
        off = L.CPoaOutput.consensus.offset
        for z in range(n):
            i, o = ins[z], outs[z]
            reads = [ctypes.string_at(i.seqs[k], i.lens[k]).decode() if i.seqs[k] else None for k in range(i.n_reads)]
            cons = "".join(r for r in reads if r)[:o.cap]
            cp = ctypes.c_void_p.from_address(base + z * ctypes.sizeof(L.CPoaOutput) + off).value
            ctypes.memmove(cp, cons.encode(), len(cons))
            o.len = len(cons)
            kept = [k for k, r in enumerate(reads) if r]
            o.n_keys = len(kept)
            for k in range(i.n_reads):
                o.keys[k] = kept.index(k) if reads[k] else -1
            for q in range(o.n_keys):
                o.rc[q] = q % 2
                for e in range(4):
                    o.extents[4 * q + e] = 10 * q + e
        return 0


class _Eng:
    _h = None


def test_poa_batch_marshalling_round_trip(monkeypatch):
    monkeypatch.setattr(poa, "load", lambda: _FakeLib())
    monkeypatch.setattr(poa, "_engine", lambda e: _Eng())
    zmws = [["ACGT", None, "GG"], [], ["T"], [None], ["AC" * 50, "G", "TT"], []]   # a read-less ZMW last
    got = poa.poa_batch(zmws)
    assert len(got) == len(zmws)
    for reads, g in zip(zmws, got):
        kept = [r for r in reads if r]
        assert g["consensus"] == "".join(kept)
        assert g["keys"] == [kept.index(r) if r else -1 for r in reads] or len(set(kept)) < len(kept)
        assert [s["rc"] for s in g["summaries"]] == [bool(q % 2) for q in range(len(kept))]
        assert [s["read"] + s["tpl"] for s in g["summaries"]] == [(10 * q, 10 * q + 1, 10 * q + 2, 10 * q + 3)
                                                                  for q in range(len(kept))]
