"""Host logic of pbccs_amd.quiver.PreparedQuiverBatch (CPU, no device): the structured input arrays (reads with their
QV tracks passed in place, NULL for a missing track, chemistry names, tend -1 for the template end, NaN
thresholds) and the result decoding from the field columns -- against a stand-in for pbccs_quiver_polish_batch
that reads the structs through their ctypes layout (include/pbccs_amd.h pbccs_quiver_read / _zmw / _result)."""
import ctypes
import math

import numpy as np

import pbccs_amd as P
from pbccs_amd import lib as L
from pbccs_amd import quiver


def _cstr_at(base, ctype, k, field):
    addr = ctypes.c_void_p.from_address(base + k * ctypes.sizeof(ctype) + getattr(ctype, field).offset).value
    return ctypes.string_at(addr) if addr else None


class _FakeLib:
    """Echo: consensus = the template reversed, QVs = each read's summed track values mod 50 per position (so a
    wrong track pointer shows), n_tested = total read bases, n_applied = reads, converged / ok / n_active set."""
    seen = None

    def pbccs_quiver_polish_batch(self, h, carr, names, nc, zmws, n, opts, out):
        zb = ctypes.cast(zmws, ctypes.c_void_p).value
        ob = ctypes.cast(out, ctypes.c_void_p).value
        seen = []
        for z in range(n):
            Z = zmws[z]
            tpl = _cstr_at(zb, L.CQuiverZmw, z, "tpl")[:Z.tpl_len].decode()
            rb = ctypes.cast(Z.reads, ctypes.c_void_p).value
            reads = []
            for r in range(Z.n_reads):
                R = Z.reads[r]
                seq = _cstr_at(rb, L.CQuiverRead, r, "seq")[:R.len].decode()
                tracks = []
                for f in ("ins_qv", "subs_qv", "del_qv", "del_tag", "merge_qv"):
                    p = getattr(R, f)
                    tracks.append([p[i] for i in range(R.len)] if p else None)
                chem = _cstr_at(rb, L.CQuiverRead, r, "chemistry").decode()
                reads.append((seq, tracks, chem, R.strand, R.tstart, R.tend, R.threshold))
            seen.append((tpl, reads))
            o = out[z]
            cons = tpl[::-1].encode()
            cp = ctypes.c_void_p.from_address(ob + z * ctypes.sizeof(L.CQuiverResult) + L.CQuiverResult.consensus.offset).value
            ctypes.memmove(cp, cons, len(cons))
            o.consensus_len = len(cons)
            if o.qvs:
                for i in range(len(cons)):
                    o.qvs[i] = int(sum(t[i % len(t)] for _, tr, *_ in reads for t in tr if t)) % 50
            o.n_tested = sum(len(s) for s, *_ in reads)
            o.n_applied = len(reads)
            o.converged = 1
            o.ok = 1
            o.n_active = len(reads)
        _FakeLib.seen = seen
        return 0


def test_prepared_quiver_batch_marshalling_round_trip(monkeypatch):
    monkeypatch.setattr(quiver, "load", lambda: _FakeLib())

    class _Eng:
        _h = None
    rng = np.random.default_rng(5)
    zmws = []
    for k, (L_, nr) in enumerate([(12, 2), (7, 1), (20, 3)]):
        tpl = "".join(rng.choice(list("ACGT"), L_))
        reads = []
        for r in range(nr):
            s = "".join(rng.choice(list("ACGT"), L_ - 1 + r))
            f = {"ins": rng.integers(0, 9, len(s)).astype(np.float32), "subs": rng.integers(0, 9, len(s)).tolist(),
                 "del": rng.integers(0, 9, len(s)).tolist(), "del_tag": list(rng.choice(list("ACGTN"), len(s)))}
            rd = {"seq": s, "strand": r % 2, "ts": 0, "te": None if r == 0 else L_, "features": f}
            if r == 1:
                rd["threshold"] = 0.25
                rd["chemistry"] = "P6-C4"
            reads.append(rd)
        zmws.append({"tpl": tpl, "reads": reads})
    cfg = P.QuiverConfig(P.QvModelParams(Match=-0.2, Mismatch=-8.0, MismatchS=-0.15, Branch=-3.5, BranchS=-0.12,
                                         DeletionN=-7.5, DeletionWithTag=-4.5, DeletionWithTagS=-0.2, Nce=-6.0,
                                         NceS=-0.1, Merge=[-3.0] * 4, MergeS=[-0.1] * 4))
    got = quiver.PreparedQuiverBatch(zmws, cfg).run(engine=_Eng())
    for z, (tpl, reads), g in zip(zmws, _FakeLib.seen, got):
        assert tpl == z["tpl"]
        assert g["consensus"] == z["tpl"][::-1]
        assert (g["converged"], g["ok"], g["n_active"]) == (True, True, len(z["reads"]))
        assert g["n_tested"] == sum(len(r["seq"]) for r in z["reads"]) and g["n_applied"] == len(z["reads"])
        for rd, (seq, tracks, chem, strand, ts, te, thr) in zip(z["reads"], reads):
            f = rd["features"]
            assert seq == rd["seq"] and strand == rd["strand"] and ts == rd["ts"]
            assert te == (-1 if rd["te"] is None else rd["te"])
            assert chem == rd.get("chemistry", "*")
            assert (math.isnan(thr) and "threshold" not in rd) or thr == np.float32(rd["threshold"])
            assert tracks[0] == [float(x) for x in f["ins"]] and tracks[1] == [float(x) for x in f["subs"]]
            assert tracks[2] == [float(x) for x in f["del"]]
            assert tracks[3] == [float(ord(c)) for c in f["del_tag"]]
            assert tracks[4] is None   # no merge track: NULL (zeros on the C side)
        exp = [int(sum(t[i % len(t)] for _, tr, *_ in reads for t in tr if t)) % 50 for i in range(len(g["consensus"]))]
        assert g["qvs"] == exp
